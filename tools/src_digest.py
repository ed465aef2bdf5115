#!/usr/bin/env python3
"""The source digest baked into libme_engine.so (me_build_info, matching_engine_amd/Makefile
DIGEST_SRCS): sha256 of the product sources and headers concatenated in this order, first 16 hex
digits. `python tools/src_digest.py` prints it for the working tree."""
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "matching_engine_amd", "csrc")
FILES = [os.path.join(CSRC, f) for f in ("me_kernels.hip", "me_match_reg.hip", "me_snapshot.hip", "me_agg.hip", "me_engine.cpp",
                                         "me_gen.cpp", "me_service.cpp", "me_cluster.cpp", "me_far.hpp", "me_layout.hpp", "me_wave.hpp")]
FILES += [os.path.join(ROOT, "include", f) for f in ("me_engine.h", "me_service.h", "me_cluster.h")]
FILES += [os.path.join(ROOT, "matching_engine_amd", "Makefile")]  # the compiler flags shape the kernels


def digest() -> str:
    h = hashlib.sha256()
    for f in FILES:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(digest())

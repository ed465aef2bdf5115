"""The C-ABI library loads and exports exactly what include/*.h declare; without a GPU the engine
refuses to start (no CPU fallback). Runs on CPU."""
import ctypes as C
import os
import re

import pytest

from tests.conftest import gpu_available

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "me_engine.h")).read()
    src += open(os.path.join(ROOT, "include", "me_service.h")).read()
    src += open(os.path.join(ROOT, "include", "me_cluster.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(me_[a-z0-9_]+)\s*\(", src)) - {"me_engine", "me_gen", "me_service", "me_cluster"})


def test_header_declares_the_boundary():
    fns = declared_functions()
    for must in ("me_create", "me_destroy", "me_submit_batch", "me_book_snapshot", "me_last_error",
                 "me_submit_batch_device", "me_normalize_to_q4"):
        assert must in fns


def test_library_exports_every_declared_symbol(built):
    from matching_engine_amd import _abi

    lib = C.CDLL(_abi.LIB_PATH)
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    # and the ctypes prototypes cover the whole header
    assert set(declared_functions()) <= set(_abi.PROTOTYPES)


def test_library_is_gfx950(built):
    from matching_engine_amd import _abi

    blob = open(_abi.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU behaviour")
def test_engine_fails_loudly_without_gpu(built):
    import matching_engine_amd as me

    with pytest.raises(me.EngineError, match="HIP"):
        me.Engine(4, 128, [1000] * 4, 1024, 1024, 1 << 20)


def test_invalid_config_rejected(built):
    import matching_engine_amd as me

    with pytest.raises(me.EngineError, match="invalid config"):
        me.Engine(4, 100, [1000] * 4, 1024, 1024, 1 << 20)  # levels not a power of two


def test_library_was_built_from_these_sources(built):
    """The loaded libme_engine.so carries the digest of the sources it was compiled from: equal to
    the working tree's, so the library a run loads (here, or shipped to the GPU box) is this tree."""
    import sys

    from matching_engine_amd import _abi

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from src_digest import digest

    info = _abi.load().me_build_info().decode()
    assert info == f"src={digest()} arch=gfx950", info

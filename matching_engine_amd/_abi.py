"""ctypes view of include/me_engine.h (the C-ABI of libme_engine.so).

The library is built in-tree (``make -C matching_engine_amd``); loading fails loudly when it is
missing — there is no Python or CPU fallback for the matching path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# ME_ENGINE_LIB selects a diagnostic variant (e.g. build/libme_engine_stamps.so) for profiling runs.
LIB_PATH = os.environ.get("ME_ENGINE_LIB") or os.path.join(_HERE, "libme_engine.so")

# ---- enums (include/me_engine.h) -------------------------------------------------------------
SIDE_UNSPECIFIED, SIDE_BUY, SIDE_SELL = 0, 1, 2
TYPE_LIMIT, TYPE_MARKET = 0, 1
OP_NEW, OP_CANCEL = 0, 1
ST_NEW, ST_PARTIALLY_FILLED, ST_FILLED, ST_CANCELED, ST_REJECTED = 0, 1, 2, 3, 4
RJ_NONE, RJ_BAD_QTY, RJ_BAD_SIDE, RJ_OUT_OF_WINDOW, RJ_BAD_SYMBOL, RJ_UNKNOWN_ORDER, RJ_BAD_SEQ, RJ_CAPACITY = range(8)
ME_OK, ME_E_INVALID, ME_E_HIP, ME_E_CAPACITY, ME_E_STATE, ME_E_SQLITE = 0, -1, -2, -3, -4, -5
CHUNK_SLOTS = 16


def kind(side: int, otype: int = TYPE_LIMIT, op: int = OP_NEW) -> int:
    """ME_KIND(side, type, op)."""
    return (side & 3) | ((otype & 1) << 2) | ((op & 1) << 3)


# ---- structs ---------------------------------------------------------------------------------
class MeConfig(C.Structure):
    _fields_ = [
        ("device", C.c_int32),
        ("num_symbols", C.c_uint32),
        ("levels", C.c_uint32),
        ("max_batch", C.c_uint32),
        ("max_resting", C.c_uint64),
        ("max_chunks", C.c_uint64),
        ("seq_ring", C.c_uint64),
        ("base_price", C.POINTER(C.c_int64)),
        ("symbol_ids", C.POINTER(C.c_uint32)),
        ("batches_per_launch", C.c_uint32),
        ("far_levels", C.c_uint32),
        ("host_slots", C.c_uint32),
        ("host_tape_cap", C.c_uint64),
    ]


class MeOrderSoa(C.Structure):
    _fields_ = [
        ("seq", C.c_void_p),
        ("price_q4", C.c_void_p),
        ("qty", C.c_void_p),
        ("symbol", C.c_void_p),
        ("kind", C.c_void_p),
    ]


class MeOrderSoaW(C.Structure):
    _fields_ = [
        ("seq", C.c_void_p),
        ("price_q4", C.c_void_p),
        ("qty", C.c_void_p),
        ("symbol", C.c_void_p),
        ("kind", C.c_void_p),
    ]


class MeGenParams(C.Structure):
    _fields_ = [
        ("config", C.c_uint32),
        ("seed", C.c_uint64),
        ("num_symbols", C.c_uint32),
        ("levels", C.c_uint32),
        ("spread_ticks", C.c_int32),
        ("max_qty", C.c_int32),
        ("market_pct", C.c_uint32),
        ("cancel_pct", C.c_uint32),
        ("zipf_s", C.c_double),
        ("market_qty_mult", C.c_int32),
        ("seq_start", C.c_uint64),
        ("drift_step", C.c_int32),
        ("drift_every", C.c_uint32),
        ("far_pct", C.c_uint32),
    ]


FILL_DTYPE = np.dtype(
    [("taker_seq", "<u8"), ("maker_seq", "<u8"), ("price_q4", "<i8"), ("qty", "<i4"), ("symbol", "<u4")]
)
RESULT_DTYPE = np.dtype(
    [
        ("filled_qty", "<i4"),
        ("remaining_qty", "<i4"),
        ("fill_count", "<u4"),
        ("tape_offset", "<u4"),
        ("status", "u1"),
        ("reason", "u1"),
        ("pad", "u1", (2,)),
    ]
)
LEVEL_DTYPE = np.dtype([("price_q4", "<i8"), ("total_qty", "<i8"), ("order_count", "<u4"), ("pad", "<u4")])
BOOK_ENTRY_DTYPE = np.dtype(
    [("seq", "<u8"), ("price_q4", "<i8"), ("qty", "<i4"), ("side", "u1"), ("pad", "u1", (3,))]
)
assert FILL_DTYPE.itemsize == 32 and RESULT_DTYPE.itemsize == 20
assert LEVEL_DTYPE.itemsize == 24 and BOOK_ENTRY_DTYPE.itemsize == 24

# every symbol include/me_engine.h declares -> (restype, argtypes)
_P = C.c_void_p
_SZ = C.c_size_t
PROTOTYPES = {
    "me_normalize_to_q4": (C.c_int, [C.c_int64, C.c_int32, C.POINTER(C.c_int64)]),
    "me_build_info": (C.c_char_p, []),
    "me_create": (_P, [C.POINTER(MeConfig)]),
    "me_destroy": (None, [_P]),
    "me_submit_batch": (C.c_int, [_P, C.POINTER(MeOrderSoa), _SZ, _P, _SZ, C.POINTER(_SZ), _P]),
    "me_fill_bound": (C.c_uint64, [_P, _SZ]),
    "me_submit_host": (C.c_int, [_P, C.POINTER(MeOrderSoa), _SZ, C.POINTER(C.c_uint64)]),
    "me_collect": (C.c_int, [_P, C.c_uint64, C.POINTER(_P), C.POINTER(_SZ), C.POINTER(_P), C.POINTER(_SZ)]),
    "me_host_inputs": (C.c_int, [_P, _SZ, C.POINTER(MeOrderSoaW)]),
    "me_get_config": (C.c_int, [_P, C.POINTER(MeConfig)]),
    "me_host_reserve": (C.c_int, [_P, C.c_uint32]),
    "me_submit_batch_device": (C.c_int, [_P, C.POINTER(MeOrderSoa), _SZ]),
    "me_submit_device_limits": (C.c_int, [_P, C.POINTER(MeOrderSoa), _SZ, C.c_uint64]),
    "me_sync": (C.c_int, [_P]),
    "me_fetch_outputs": (C.c_int, [_P, _P, _SZ, C.POINTER(_SZ), _P, _SZ]),
    "me_last_group_size": (C.c_uint32, [_P]),
    "me_fetch_group_outputs": (C.c_int, [_P, C.c_uint32, _P, _SZ, C.POINTER(_SZ), _P, _SZ]),
    "me_copy_tape_device": (C.c_int, [_P, _P, _SZ, C.POINTER(_SZ)]),
    "me_copy_results_device": (C.c_int, [_P, _P, _SZ]),
    "me_device_alloc": (C.c_int, [_P, _SZ, C.POINTER(_P)]),
    "me_device_free": (C.c_int, [_P, _P]),
    "me_memcpy_h2d": (C.c_int, [_P, _P, _P, _SZ]),
    "me_set_stream": (C.c_int, [_P, _P]),
    "me_book_snapshot": (C.c_int, [_P, C.c_uint32, _P, _P, _SZ, C.POINTER(_SZ), C.POINTER(_SZ)]),
    "me_book_dump": (C.c_int, [_P, C.c_uint32, _P, _SZ, C.POINTER(_SZ)]),
    "me_book_orders": (C.c_int, [_P, C.c_uint32, C.c_uint32, _P, _SZ, C.POINTER(_SZ), _P, _SZ, C.POINTER(_SZ),
                                 _P, _P, C.POINTER(_SZ), C.POINTER(_SZ)]),
    "me_book_levels_all": (C.c_int, [_P, C.c_uint32, _P, _P]),
    "me_resting_count": (C.c_int, [_P, C.POINTER(C.c_uint64)]),
    "me_timing_enable": (C.c_int, [_P, C.c_int]),
    "me_timing_read": (
        C.c_int,
        [_P, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
         C.POINTER(C.c_uint64)],
    ),
    "me_last_error": (C.c_int, [_P, C.c_char_p, _SZ]),
    "me_stats_read": (C.c_int, [_P, C.POINTER(C.c_uint64)]),
    "me_far_stats": (C.c_int, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "me_chunk_stats": (C.c_int, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "me_paths_read": (C.c_int, [_P, C.POINTER(C.c_uint32)]),
    "me_admission_read": (C.c_int, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "me_admission_check": (C.c_int, [_P, C.c_uint64, C.POINTER(C.c_int)]),
    "me_gen_create": (_P, [C.POINTER(MeGenParams)]),
    "me_gen_destroy": (None, [_P]),
    "me_gen_base_prices": (C.c_int, [_P, _P]),
    "me_gen_next": (C.c_int, [_P, _SZ, _P, _P, _P, _P, _P]),
    "me_gen_seed_book": (C.c_int, [_P, C.c_uint32, C.c_uint32, _P, _P, _P, _P]),
    "me_shard_of": (C.c_uint32, [C.c_uint32, C.c_uint32]),
}

_lib = None


def load() -> C.CDLL:
    """Load libme_engine.so (built in-tree). Raises if it is missing: no fallback exists."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build it with `make -C matching_engine_amd` "
            "(the matching path has no CPU/Python fallback)"
        )
    # libme_engine.so and torch's ROCm wheel both need libamdhip64.so.7; torch resolves it by a
    # different file name, so if our library were loaded first the process would end up with two
    # HIP runtimes. Letting torch (when installed) load first keeps one runtime per process.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(LIB_PATH)
    variant = bool(os.environ.get("ME_ENGINE_LIB"))  # an older build in an A/B run may lack newer entries
    for name, (res, args) in PROTOTYPES.items():
        if variant and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def ptr(a: np.ndarray) -> int:
    return a.ctypes.data


# ---- include/me_service.h ---------------------------------------------------------------------
class MeOrderRequest(C.Structure):
    _fields_ = [
        ("client_id", C.c_char_p),
        ("symbol", C.c_char_p),
        ("order_type", C.c_int32),
        ("side", C.c_int32),
        ("price", C.c_int64),
        ("scale", C.c_int32),
        ("quantity", C.c_int32),
    ]


class MeOrderResponse(C.Structure):
    _fields_ = [
        ("order_id", C.c_char * 32),
        ("success", C.c_int32),
        ("grpc_status", C.c_int32),
        ("error_message", C.c_char * 64),
    ]


class MeCancelRequest(C.Structure):
    _fields_ = [
        ("client_id", C.c_char_p),
        ("symbol", C.c_char_p),
        ("order_id", C.c_char_p),
    ]


class MeOrderUpdate(C.Structure):
    _fields_ = [
        ("order_id", C.c_char * 32),
        ("client_id", C.c_char * 64),
        ("symbol", C.c_char * 32),
        ("status", C.c_int32),
        ("scale", C.c_int32),
        ("fill_price", C.c_int64),
        ("fill_quantity", C.c_int32),
        ("remaining_quantity", C.c_int32),
    ]


assert C.sizeof(MeOrderUpdate) == 152, "me_order_update layout"


class MeMarketData(C.Structure):
    _fields_ = [
        ("best_bid", C.c_int64),
        ("best_ask", C.c_int64),
        ("scale", C.c_int32),
        ("bid_size", C.c_int32),
        ("ask_size", C.c_int32),
        ("has_bid", C.c_int32),
        ("has_ask", C.c_int32),
        ("pad", C.c_int32),
    ]

class MeBookOrder(C.Structure):
    _fields_ = [
        ("order_id", C.c_char * 32),
        ("client_id", C.c_char * 64),
        ("price", C.c_int64),
        ("scale", C.c_int32),
        ("quantity", C.c_int32),
        ("side", C.c_int32),
        ("pad", C.c_int32),
    ]


assert C.sizeof(MeBookOrder) == 120, "me_book_order layout"

MATCH_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(MeOrderSoa), C.c_size_t, C.POINTER(C.c_void_p),
                       C.POINTER(C.c_size_t), C.POINTER(C.c_void_p))
BOOK_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t),
                      C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t), C.c_void_p, C.c_void_p, C.POINTER(C.c_size_t),
                      C.POINTER(C.c_size_t))
SUBMIT_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(MeOrderSoa), C.c_size_t, C.POINTER(C.c_uint64))
COLLECT_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint64, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t),
                         C.POINTER(C.c_void_p))


class MeMatcher(C.Structure):
    _fields_ = [
        ("ctx", C.c_void_p),
        ("num_symbols", C.c_uint32),
        ("max_batch", C.c_uint32),
        ("max_resting", C.c_uint64),
        ("match", MATCH_FN),
        ("book", BOOK_FN),
        ("submit", SUBMIT_FN),
        ("collect", COLLECT_FN),
    ]


# ---- include/me_cluster.h ---------------------------------------------------------------------
TRANSPORT_RCCL, TRANSPORT_TCP = 0, 1


class MeClusterConfig(C.Structure):
    _fields_ = [
        ("rank", C.c_uint32),
        ("world", C.c_uint32),
        ("num_symbols", C.c_uint32),
        ("max_batch", C.c_uint32),
        ("transport", C.c_int32),
        ("device", C.c_int32),
        ("addr", C.c_char_p),
        ("port", C.c_uint32),
        ("timeout_ms", C.c_uint32),
    ]


ADMIT_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint64, C.POINTER(C.c_int))
LEVELS_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p)


class MeShardOps(C.Structure):
    _fields_ = [
        ("ctx", C.c_void_p),
        ("max_resting", C.c_uint64),
        ("admit", ADMIT_FN),
        ("match", MATCH_FN),
        ("book", BOOK_FN),
        ("levels_all", LEVELS_FN),
    ]


PROTOTYPES.update({
    "me_service_create_matcher": (_P, [C.POINTER(MeMatcher), C.POINTER(C.c_char_p), C.c_uint32, C.c_char_p]),
    "me_service_order_book": (C.c_int, [_P, C.c_char_p, C.c_uint32, C.POINTER(MeBookOrder), _SZ, C.POINTER(_SZ),
                                        C.POINTER(MeBookOrder), _SZ, C.POINTER(_SZ)]),
    "me_service_cancel_order": (C.c_int, [_P, C.POINTER(MeCancelRequest), C.POINTER(MeOrderResponse)]),
    "me_service_market_data": (C.c_int, [_P, C.c_char_p, C.POINTER(MeMarketData)]),
    "me_service_updates": (C.c_int, [_P, C.c_char_p, C.POINTER(MeOrderUpdate), _SZ, C.POINTER(_SZ)]),
    "me_service_create": (_P, [_P, C.POINTER(C.c_char_p), C.c_uint32, C.c_char_p]),
    "me_service_destroy": (None, [_P]),
    "me_service_submit_order": (C.c_int, [_P, C.POINTER(MeOrderRequest), C.POINTER(MeOrderResponse)]),
    "me_service_pending": (_SZ, [_P]),
    "me_service_next_oid": (C.c_uint64, [_P]),
    "me_service_flush": (C.c_int, [_P, _P, _SZ, C.POINTER(_SZ), _P, _P, _SZ, C.POINTER(_SZ)]),
    "me_service_book": (C.c_int, [_P, C.c_char_p, _P, _P, _SZ, C.POINTER(_SZ), C.POINTER(_SZ)]),
    "me_service_last_error": (C.c_int, [_P, C.c_char_p, _SZ]),
    "me_service_unpersisted": (_SZ, [_P]),
    "me_service_submit_orders": (C.c_int, [_P, C.POINTER(MeOrderRequest), _SZ, C.POINTER(MeOrderResponse)]),
    "me_service_start": (C.c_int, [_P, C.c_uint32, C.c_uint32]),
    "me_service_stop": (C.c_int, [_P]),
    "me_service_updates_dropped": (C.c_uint64, [_P]),
    "me_service_stats": (C.c_int, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "me_cluster_shard_symbols": (_SZ, [C.c_uint32, C.c_uint32, C.c_uint32, _P, _SZ]),
    "me_cluster_create": (_P, [C.POINTER(MeClusterConfig), C.POINTER(MeConfig), C.POINTER(MeShardOps)]),
    "me_cluster_stop": (C.c_int, [_P]),
    "me_cluster_destroy": (None, [_P]),
    "me_cluster_serve": (C.c_int, [_P]),
    "me_cluster_submit": (C.c_int, [_P, C.POINTER(MeOrderSoa), _SZ, C.POINTER(C.c_uint64)]),
    "me_cluster_collect": (C.c_int, [_P, C.c_uint64, C.POINTER(_P), C.POINTER(_SZ), C.POINTER(_P)]),
    "me_cluster_match": (C.c_int, [_P, C.POINTER(MeOrderSoa), _SZ, C.POINTER(_P), C.POINTER(_SZ), C.POINTER(_P)]),
    "me_cluster_book": (C.c_int, [_P, C.c_uint32, C.c_uint32, _P, _SZ, C.POINTER(_SZ), _P, _SZ, C.POINTER(_SZ),
                                  _P, _P, C.POINTER(_SZ), C.POINTER(_SZ)]),
    "me_cluster_snapshot": (C.c_int, [_P, C.c_uint32, _P, _P]),
    "me_cluster_matcher": (C.c_int, [_P, C.POINTER(MeMatcher)]),
    "me_cluster_stats": (C.c_int, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "me_cluster_phases": (C.c_int, [_P, C.POINTER(C.c_double), _SZ]),
    "me_cluster_last_error": (C.c_int, [_P, C.c_char_p, _SZ]),
    "me_cluster_host_probe": (C.c_int, [C.c_uint32, C.c_uint32, _P, _SZ, C.c_double, C.c_uint32, _P]),
})

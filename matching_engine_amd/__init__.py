"""MI355X-native batched matching core (drop-in behind julien-mrty/Matching_Engine's SubmitOrder).

The product is libme_engine.so (gfx950 HIP kernels + C++ host engine, C-ABI include/me_engine.h);
this package is the thin Python view used by tests and bench.py. Build: ``make -C matching_engine_amd``.
"""
from ._abi import (  # noqa: F401
    FILL_DTYPE, RESULT_DTYPE, LEVEL_DTYPE, BOOK_ENTRY_DTYPE, LIB_PATH, kind, load,
    SIDE_BUY, SIDE_SELL, SIDE_UNSPECIFIED, TYPE_LIMIT, TYPE_MARKET, OP_NEW, OP_CANCEL,
    ST_NEW, ST_PARTIALLY_FILLED, ST_FILLED, ST_CANCELED, ST_REJECTED,
    RJ_NONE, RJ_BAD_QTY, RJ_BAD_SIDE, RJ_OUT_OF_WINDOW, RJ_BAD_SYMBOL, RJ_UNKNOWN_ORDER, RJ_BAD_SEQ,
    ME_OK, ME_E_INVALID, ME_E_HIP, ME_E_CAPACITY, ME_E_STATE, ME_E_SQLITE,
)
from .engine import (  # noqa: F401
    Batch, DeviceBatch, Engine, EngineError, Stream, StreamConfig, normalize_to_q4, preset, shard_of, shard_table,
)
from .service import MatchingEngineService, ServiceError  # noqa: F401,E402

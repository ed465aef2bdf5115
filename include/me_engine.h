/*
 * me_engine.h — C-ABI of the MI355X batched matching core.
 *
 * This is the drop-in boundary between the (C++) submit-order host side and the
 * gfx950 HIP kernels. Plain C: no exceptions cross it, every call returns an int
 * status (0 = ok), buffers are caller-owned unless stated, no torch types.
 *
 * What each entry point replaces in the reference (julien-mrty/Matching_Engine,
 * paths relative to the reference root):
 *
 *   me_service_*        MatchingEngineServiceImpl (include/server/matching_engine_service.hpp:9-30,
 *                       src/server/matching_engine_service.cpp:17-121): ctor seeds the OID counter,
 *                       me_service_submit_order == SubmitOrder (validate :66-83 -> OID :85 ->
 *                       Order::FromRaw/normalize_to_q4 :89-97 -> persist :99-104 -> response :107-114).
 *                       Persistence is deferred to the batched flush (me_service_flush).
 *   me_normalize_to_q4  normalize_to_q4 (include/domain/price.hpp:15-29), exceptions mapped to codes.
 *   me_create/...       the engine slot include/engine/model.hpp (0 bytes in the reference): there is no
 *                       reference matcher; matching semantics are defined in DESIGN.md §2 and pinned by
 *                       the CPU oracle under oracle/.
 *   me_book_snapshot    GetOrderBook (src/server/matching_engine_service.cpp:123-129, a stub returning an
 *                       empty OrderBookResponse) and Storage::best_bid/best_ask
 *                       (src/storage/storage.cpp:212-252, broken: always nullopt).
 *   me_fill             FillRow (include/storage/storage.hpp:11-17) + fills table (src/storage/storage.cpp:53-63).
 *   ME_ST_*             OrderUpdate.Status (proto/matching_engine.proto:79-85).
 */
#ifndef ME_ENGINE_H
#define ME_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- domain encodings --------------------------------------------------------------- */
/* Side (proto/matching_engine.proto:5-9; include/domain/side.hpp:8-9 static_asserts 1/2). */
enum { ME_SIDE_UNSPECIFIED = 0, ME_SIDE_BUY = 1, ME_SIDE_SELL = 2 };
/* OrderType (proto/matching_engine.proto:11-14). Any value != LIMIT is treated as MARKET,
 * mirroring type_str / the LIMIT-only price check (matching_engine_service.cpp:50,78). */
enum { ME_TYPE_LIMIT = 0, ME_TYPE_MARKET = 1 };
/* Operation carried by a batch record. CANCEL is a build extension (no reference RPC). */
enum { ME_OP_NEW = 0, ME_OP_CANCEL = 1 };
/* OrderUpdate.Status (proto/matching_engine.proto:79-85). */
enum {
  ME_ST_NEW = 0,
  ME_ST_PARTIALLY_FILLED = 1,
  ME_ST_FILLED = 2,
  ME_ST_CANCELED = 3,
  ME_ST_REJECTED = 4
};
/* Why a batch record was rejected by the matcher (me_order_result.reason). */
enum {
  ME_RJ_NONE = 0,
  ME_RJ_BAD_QTY = 1,       /* qty <= 0 (the service rejects these before they reach a batch) */
  ME_RJ_BAD_SIDE = 2,      /* side not BUY/SELL (reference: CHECK side IN (1,2) -> "DB insert failed") */
  ME_RJ_OUT_OF_WINDOW = 3, /* retired: every int64 price is accepted (never produced) */
  ME_RJ_BAD_SYMBOL = 4,    /* symbol id >= num_symbols */
  ME_RJ_UNKNOWN_ORDER = 5, /* CANCEL target is not a live resting order of this symbol */
  ME_RJ_BAD_SEQ = 6,       /* seq == 0 (no OID is 0: the counter starts at 1, storage.cpp:254-267) */
  ME_RJ_CAPACITY = 7       /* service only: a LIMIT the shard could not admit while its books hold
                              max_resting orders (me_service.h; never produced by the engine) */
};

/* kind byte of a batch record: bits 0-1 side, bit 2 type (1 = MARKET), bit 3 op (1 = CANCEL). */
#define ME_KIND(side, type, op) ((uint8_t)(((side) & 3) | (((type) & 1) << 2) | (((op) & 1) << 3)))

/* Slots per FIFO chunk (one wave-wide load of a level's queue). */
#define ME_CHUNK_SLOTS 16

/* Error codes returned by every entry point. */
enum {
  ME_OK = 0,
  ME_E_INVALID = -1,   /* bad argument / config */
  ME_E_HIP = -2,       /* HIP runtime failure (no device, launch failure, ...) */
  ME_E_CAPACITY = -3,  /* a batch refused by admission control (max_resting; not sticky), or a
                          fixed-capacity pool (chunks, far levels, ...) overflowed inside a batch (sticky) */
  ME_E_STATE = -4,     /* engine in a failed state (a previous capacity/HIP error) */
  ME_E_SQLITE = -5     /* persistence failure */
};

/* ---- domain helper ------------------------------------------------------------------- */
/* normalize_to_q4 (include/domain/price.hpp:15-29). Returns 0 and *out on success,
 * 1 for invalid_argument("scale out of range"), 2 for overflow_error("overflow"),
 * 3 for overflow_error("underflow"). */
int me_normalize_to_q4(int64_t price, int32_t scale, int64_t* out);

/* Build record (no reference counterpart): "src=<16 hex> arch=gfx950", the first 16 hex digits of
 * the sha256 of the product sources and headers the library was compiled from (Makefile
 * DIGEST_SRCS order, restated by tools/src_digest.py). */
const char* me_build_info(void);

/* ---- the batched matching engine (one shard = one GPU) ------------------------------- */
typedef struct me_engine me_engine;

typedef struct me_config {
  int32_t device;              /* HIP device ordinal */
  uint32_t num_symbols;        /* local symbols of this shard, ids 0..num_symbols-1 */
  uint32_t levels;             /* L: price levels of each symbol's on-chip WINDOW (power of two, 64..2^20).
                                  Prices are not limited to it: levels outside live in far arrays and the
                                  window re-centres as the market moves */
  uint32_t max_batch;          /* largest n accepted by me_submit_batch* */
  uint64_t max_resting;        /* resting orders the scratch/tape bound is sized for. Admission control:
                                  a batch is accepted only while (resting orders) + (LIMIT records
                                  accepted and not yet matched) + (its LIMIT records; every record of
                                  a device batch) <= max_resting, else me_submit_* return
                                  ME_E_CAPACITY for that batch, NOT sticky: nothing of it was enqueued
                                  and the engine stays usable (me_admission_read) */
  uint64_t max_chunks;         /* FIFO chunk pool (ME_CHUNK_SLOTS slots each, 256 B); 0 = max_resting + 32*S + 64,
                                  enough for any book shape and any movement of liquidity between symbols:
                                  free chunks go back to a shared pool (me_chunk_stats) */
  uint64_t seq_ring;           /* seq-ring entries for cancels (power of two, 0 = 2^28). Any u64 seq is
                                  accepted; one launch group (batches_per_launch batches) must span fewer
                                  than seq_ring seqs */
  const int64_t* base_price;   /* [num_symbols] initial window base (price_q4 of level 0) per symbol */
  const uint32_t* symbol_ids;  /* optional [num_symbols] ids written to me_fill.symbol (NULL = local id) */
  uint32_t batches_per_launch; /* L <= 128: device batches matched per kernel launch, 1..32 (0 = 32). Back-to-back
                                  me_submit_batch_device calls fill a group; me_sync flushes a partial one */
  uint32_t far_levels;         /* far levels (price levels outside the window) each symbol and side holds in
                                  its inline region, 0 = 256. Not a limit: a side that outgrows it moves to
                                  the far arena, sized from max_resting so it never runs out (me_far_stats) */
  uint32_t host_slots;         /* pinned slots of the host-batch pipeline (me_submit_host), 0 = enough to keep
                                  four launch groups in flight (4 * batches_per_launch + 1); allocated on use */
  uint64_t host_tape_cap;      /* fills a slot holds (0 = 2 * max_batch + 4096). A longer tape is recovered at
                                  me_collect while its batch's scratch is intact (collected before 3 further
                                  launch groups were submitted), else that collect fails with ME_E_CAPACITY */
} me_config;

/* One batch in structure-of-arrays form. Seqs (= numeric OIDs) ascend across the whole stream of an
 * engine: a NEW record's seq is above every earlier record's, a CANCEL record's is at least the
 * previous record's (a cancel never rests, so it may repeat the last OID instead of taking one).
 * Checked on the device: a violation fails the batch with ME_E_INVALID. */
typedef struct me_order_soa {
  const uint64_t* seq;      /* numeric OID of the record */
  const int64_t* price_q4;  /* NEW: normalized Q4 price (ignored for MARKET); CANCEL: target seq */
  const int32_t* qty;       /* NEW: quantity (wire int32, proto:44); CANCEL: ignored */
  const uint32_t* symbol;   /* local symbol id */
  const uint8_t* kind;      /* ME_KIND(side, type, op) */
} me_order_soa;

/* One trade (32 B): the maker rests, the taker crosses; price is the maker's level. */
typedef struct me_fill {
  uint64_t taker_seq;
  uint64_t maker_seq;
  int64_t price_q4;
  int32_t qty;
  uint32_t symbol;
} me_fill;

/* Per-record outcome (20 B). For CANCEL records: status CANCELED and remaining_qty = the
 * quantity removed from the book, or REJECTED/UNKNOWN_ORDER. */
typedef struct me_order_result {
  int32_t filled_qty;
  int32_t remaining_qty;  /* LIMIT: resting remainder; MARKET: discarded remainder */
  uint32_t fill_count;
  uint32_t tape_offset;   /* index of this record's first fill in the batch tape */
  uint8_t status;         /* ME_ST_* */
  uint8_t reason;         /* ME_RJ_* */
  uint8_t pad[2];
} me_order_result;

/* One price level of a snapshot. */
typedef struct me_level {
  int64_t price_q4;
  int64_t total_qty;
  uint32_t order_count;
  uint32_t pad;
} me_level;

/* One resting order of a full book dump, in priority order (bids best-first, then asks best-first). */
typedef struct me_book_entry {
  uint64_t seq;
  int64_t price_q4;
  int32_t qty;
  uint8_t side;  /* ME_SIDE_BUY / ME_SIDE_SELL */
  uint8_t pad[3];
} me_book_entry;

/* Creation fails (NULL) without a usable HIP device; the reason is then in me_last_error(NULL,..). */
me_engine* me_create(const me_config* cfg);
void me_destroy(me_engine* e);

/* Host-memory batch, synchronous: me_submit_host + me_collect + copy-out.
 * out_fills must hold the tape (me_fill_bound(e, n) records always suffice; NULL skips the copy);
 * out_results holds n records (or NULL). *n_fills receives the tape length. */
int me_submit_batch(me_engine* e, const me_order_soa* batch, size_t n, me_fill* out_fills,
                    size_t fills_cap, size_t* n_fills, me_order_result* out_results);
/* Upper bound on the tape length of one batch of n records (resting capacity + 2n). */
uint64_t me_fill_bound(const me_engine* e, size_t n);

/* ---- pipelined host batches (the time-slice path of SubmitOrder) -----------
 * me_submit_host stages the batch in the next of the engine's pinned slots (skipped when the batch
 * already lives there, see me_host_inputs), copies it to HBM on the engine's H2D stream and enqueues
 * it behind everything submitted before; it returns at once with a ticket (0, 1, 2, ...). The H2D of
 * batch k+1, the match of batch k and the PCIe writes of batch k-1's results and tape (by the tape
 * job, straight into the slot's pinned block) overlap.
 * me_collect waits for the ticket's batch (launching a partial group first when it is still waiting
 * for one) and points into the slot's pinned outputs: valid until the next me_collect (the engine holds
 * the last collected slot back; only a submit that finds every other slot busy takes it). A slot is
 * reused only after its ticket was collected (else ME_E_STATE). Not
 * thread-safe, like every other entry point: serialize calls on one engine. */
int me_submit_host(me_engine* e, const me_order_soa* batch, size_t n, uint64_t* ticket);
int me_collect(me_engine* e, uint64_t ticket, const me_fill** fills, size_t* n_fills,
               const me_order_result** results, size_t* n_results);
/* Writable pinned arrays for the n-record batch the next me_submit_host will take (zero-copy
 * staging: fill them, then pass the same pointers to me_submit_host). ME_E_STATE while that slot's
 * previous ticket is uncollected. */
typedef struct me_order_soa_w {
  uint64_t* seq;
  int64_t* price_q4;
  int32_t* qty;
  uint32_t* symbol;
  uint8_t* kind;
} me_order_soa_w;
int me_host_inputs(me_engine* e, size_t n, me_order_soa_w* out);
/* Allocate the first nslots host slots now (0 = all of them) instead of on first use — a server's
 * start-up, so no pinned allocation lands in the request path. */
int me_host_reserve(me_engine* e, uint32_t nslots);
/* The engine's configuration as created, defaults resolved (base_price / symbol_ids NULL). */
int me_get_config(const me_engine* e, me_config* out);

/* Device-resident batch (pointers in HBM), enqueued on the engine stream, asynchronous. The batch
 * buffers must stay valid until the next me_sync (or any call that reads outputs or the book).
 * Outputs stay on the device until me_fetch_outputs (me_fetch_outputs / me_fetch_group_outputs /
 * me_copy_*_device read the most recent batch and fail with ME_E_INVALID when it was a host batch). */
int me_submit_batch_device(me_engine* e, const me_order_soa* dev_batch, size_t n);
/* The same with the batch's LIMIT-record count known to the caller (me_submit_batch_device counts
 * every record of a device batch as one that may rest): admission control takes n_limits, which must
 * be at least the batch's NEW records of type LIMIT (fewer can overflow the scratch bound: a loud,
 * sticky ME_E_CAPACITY). The cluster's shards use it (the root counted them while splitting). */
int me_submit_device_limits(me_engine* e, const me_order_soa* dev_batch, size_t n, uint64_t n_limits);
/* Wait for all enqueued work; returns ME_E_CAPACITY if a pool overflowed in any batch. */
int me_sync(me_engine* e);
/* Copy the last batch's tape/results to host memory (synchronous). */
int me_fetch_outputs(me_engine* e, me_fill* out_fills, size_t fills_cap, size_t* n_fills,
                     me_order_result* out_results, size_t n_results);
/* Batches of the most recent launch group (1..batches_per_launch; the last batch is the last one of
 * it) and the outputs of its k-th batch (synchronous, like me_fetch_outputs). */
uint32_t me_last_group_size(const me_engine* e);
int me_fetch_group_outputs(me_engine* e, uint32_t k, me_fill* out_fills, size_t fills_cap, size_t* n_fills,
                           me_order_result* out_results, size_t n_results);
/* Device-to-device copy of the last batch's tape into dst (HBM), on the engine stream;
 * *n_fills is the synchronous tape length. */
int me_copy_tape_device(me_engine* e, void* dst, size_t cap_fills, size_t* n_fills);
/* Device-to-device copy of the last batch's n_results per-record results (batch order) into dst
 * (HBM), on the engine stream. With me_copy_tape_device: the per-GPU payload of the RCCL gather to
 * the persistence root (matching_engine_amd/gather.py). */
int me_copy_results_device(me_engine* e, void* dst, size_t n_results);

/* Device memory helpers so a C/Python caller can keep batches resident without torch. */
int me_device_alloc(me_engine* e, size_t bytes, void** dptr);
int me_device_free(me_engine* e, void* dptr);
int me_memcpy_h2d(me_engine* e, void* dst, const void* src, size_t bytes);
/* Use an external hipStream_t (e.g. torch's current stream); NULL restores the engine's own. */
int me_set_stream(me_engine* e, void* hip_stream);

/* GetOrderBook: top `depth` levels per side, best first (one device snapshot launch). */
int me_book_snapshot(me_engine* e, uint32_t symbol, me_level* bids, me_level* asks, size_t depth,
                     size_t* n_bids, size_t* n_asks);
/* GetOrderBook in the reference's shape (OrderBookResponse = repeated Order, proto:16-23,57-60), from
 * ONE device snapshot launch (k_book_snapshot, one workgroup per side): every resting order of the
 * top `depth` levels of each side, best level first and FIFO order within a level, plus the levels'
 * aggregates (bid_levels / ask_levels hold `depth` entries). Any output may be NULL; the counts are
 * exact even when a cap is short (entries past it are not written). */
int me_book_orders(me_engine* e, uint32_t symbol, uint32_t depth, me_book_entry* bids, size_t bids_cap,
                   size_t* n_bids, me_book_entry* asks, size_t asks_cap, size_t* n_asks, me_level* bid_levels,
                   me_level* ask_levels, size_t* n_bid_levels, size_t* n_ask_levels);
/* The top `depth` levels per side of EVERY symbol of the shard in one launch — the periodic book
 * snapshot a multi-GPU deployment gathers to its persistence root: levels[(s * 2 + side) * depth + k]
 * (side 0 bids, 1 asks; best first; zeros past the side's levels), counts[s * 2 + side] = levels written. */
int me_book_levels_all(me_engine* e, uint32_t depth, me_level* levels, uint32_t* counts);
/* Full resting state of one symbol (side, price, FIFO). *n receives the count even when cap is short. */
int me_book_dump(me_engine* e, uint32_t symbol, me_book_entry* out, size_t cap, size_t* n);
/* Resting orders over all symbols (device counter). */
int me_resting_count(me_engine* e, uint64_t* n);

/* Kernel timing. period >= 1: every period-th match-kernel launch records its own start and end
 * (hipExtLaunchKernelGGL events: no marker packets, though each timed launch still costs the
 * stream a few microseconds, hence the sampling); period <= 0: off. Resets the counters below. */
int me_timing_enable(me_engine* e, int period);
/* match_ms / launches: sum and count of the timed match-kernel durations; orders: records of the
 * timed launches; fills: fills of ALL batches since enable; pipeline_ms: device time per batch,
 * start-to-start from the first to the last timed launch (0 with fewer than two). */
int me_timing_read(me_engine* e, double* match_ms, double* pipeline_ms, uint64_t* launches,
                   uint64_t* fills, uint64_t* orders);

/* Event counters since me_create: handoffs = symbols the register-window kernel handed to its
 * continuation launch (a far price level, a re-centre, a cancel of a far or very old order). */
int me_stats_read(me_engine* e, uint64_t* handoffs);

/* Far levels (price levels outside a symbol's window; unbounded since round 5): moves =
 * sides that outgrew their region and moved to a larger one in the far arena, collections = the
 * arena's copying collections (k_seq_sweep), arena_used = entries taken from the active half. Any
 * pointer may be NULL. No reference counterpart (the reference keeps no book). */
int me_far_stats(me_engine* e, uint64_t* moves, uint64_t* collections, uint64_t* arena_used);

/* The FIFO chunk pool: reclaims = reclamations so far (k_seq_sweep returned every symbol's free chunks
 * to the shared pool ahead of a launch group that could otherwise have run out), high_water = chunk ids
 * ever handed out, pool = max_chunks. Any pointer may be NULL. No reference counterpart. */
int me_chunk_stats(me_engine* e, uint64_t* reclaims, uint64_t* high_water, uint64_t* pool);

/* The matching paths the engine runs now (no reference counterpart: the reference has one CPU path).
 * *flags bit 0 (ME_PATH_GROUPED_AGG): launch groups of windows <= 128 levels go through the aggregate
 * path (k_agg_gwalk); bit 1 (ME_PATH_HOT_AGG): hot symbols of deeper windows do. */
#define ME_PATH_GROUPED_AGG 1u
#define ME_PATH_HOT_AGG 2u
#define ME_PATH_GROUPED_CANCELS 4u /* the grouped walk covers cancels (k_agg_gwalk_cx) */
int me_paths_read(const me_engine* e, uint32_t* flags);

/* Admission control state (any pointer may be NULL): resting = resting orders of every symbol after
 * all enqueued work (waits for it); bound = the host's current upper bound (resting orders once every
 * accepted record is matched); exact_counts = times a submit had to take an exact count (flush + sync)
 * because the published count was too stale or too close to max_resting. */
int me_admission_read(me_engine* e, uint64_t* resting, uint64_t* bound, uint64_t* exact_counts);
/* Would a batch with n_rest LIMIT records be admitted now? (*ok = 1/0; nothing is enqueued.) A submit
 * from the same thread right after a 1 is admitted. Shards that must accept a slice all-or-none
 * (cluster.ShardedMatcher) ask every engine first. */
int me_admission_check(me_engine* e, uint64_t n_rest, int* ok);

/* Last error text of e (or of the last failed me_create when e == NULL). */
int me_last_error(const me_engine* e, char* buf, size_t cap);

/* ---- synthetic order streams (bench + tests; stands in for the reference client CLI) --- */
typedef struct me_gen_params {
  uint32_t config;          /* 1..5, SURVEY.md §8(d) */
  uint64_t seed;
  uint32_t num_symbols;     /* global symbols */
  uint32_t levels;          /* window L per symbol (must cover the price spread) */
  int32_t spread_ticks;     /* LIMIT offsets U[-spread, +spread] around the symbol mid */
  int32_t max_qty;          /* qty ~ U[1, max_qty] */
  uint32_t market_pct;      /* % MARKET among new orders */
  uint32_t cancel_pct;      /* % CANCEL among records */
  double zipf_s;            /* > 0: Zipf(s) symbol popularity, 0 = uniform */
  int32_t market_qty_mult;  /* > 0: MARKET qty = U[1, market_qty_mult] * max_qty (sweeps) */
  uint64_t seq_start;       /* first seq of the stream (0 = 1) */
  int32_t drift_step;       /* > 0: a symbol's mid moves drift_step ticks (in its own fixed direction) ... */
  uint32_t drift_every;     /* ... every drift_every records of that symbol */
  uint32_t far_pct;         /* % of LIMITs priced far away: mid +- U[levels, 64 * levels] ticks */
} me_gen_params;

typedef struct me_gen me_gen;
me_gen* me_gen_create(const me_gen_params* p);
void me_gen_destroy(me_gen* g);
/* Per-symbol window base (level 0 price) for all num_symbols global symbols. */
int me_gen_base_prices(const me_gen* g, int64_t* out);
/* Next n records of the global stream (already normalized, global symbol ids, seq from 1).
 * Any pointer may be NULL. */
int me_gen_next(me_gen* g, size_t n, uint64_t* seq, int64_t* price_q4, int32_t* qty,
                uint32_t* symbol, uint8_t* kind);
/* Pre-seed records (config 4): `per_side` resting orders per side per symbol at distinct levels. */
int me_gen_seed_book(me_gen* g, uint32_t symbol, uint32_t per_side, uint64_t* seq, int64_t* price_q4,
                     int32_t* qty, uint8_t* kind);
/* shard of a global symbol: splitmix64(symbol) % shards. */
uint32_t me_shard_of(uint32_t symbol, uint32_t shards);

#ifdef __cplusplus
}
#endif
#endif /* ME_ENGINE_H */

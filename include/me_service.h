/*
 * me_service.h — the SubmitOrder drop-in: MatchingEngineServiceImpl's request path re-hosted on
 * the batched GPU core (C-ABI, plain C structs mirroring the proto messages, no gRPC types).
 *
 *   me_service_create         MatchingEngineServiceImpl(db_path) + Impl ctor
 *                             (src/server/matching_engine_service.cpp:17-22, :36): opens/creates the
 *                             SQLite DB with the reference pragmas + schema (src/storage/storage.cpp:9-69)
 *                             and seeds the OID counter from MAX(OID)+1 (storage.cpp:254-267).
 *   me_service_submit_order   SubmitOrder (matching_engine_service.cpp:41-121): identical validation
 *                             order and strings (:66-83), OID allocation (:85, consumed even when
 *                             normalisation throws), normalize_to_q4 (:89-97), side CHECK -> "DB insert
 *                             failed" with order_id set (:107-111). The order joins the open time slice.
 *                             Any non-empty symbol is accepted (:66-71): a new one takes the engine's
 *                             next unused book, or an idle symbol's book once all are taken (below);
 *                             only when every book holds orders is it refused (grpc_status 8
 *                             RESOURCE_EXHAUSTED, "symbol capacity exhausted", no OID).
 *   me_service_flush          the time-slice batcher: matches every slice submitted so far on the engine
 *                             (me_submit_host / me_collect) and ingests each in ONE SQLite transaction
 *                             (orders rows as insert_new_order writes them carrying the matched status
 *                             and remainder, fills rows, maker / cancel-target updates) — the batched
 *                             rewrite of storage.cpp:78-208. Matching and persistence run outside the
 *                             submit lock: SubmitOrder never waits for a flush.
 *   me_service_start          background flusher: a slice closes at slice_orders records or once it is
 *                             interval_us old, and is flushed without any caller.
 *   me_service_book           GetOrderBook (matching_engine_service.cpp:123-129) from the GPU book.
 *   me_service_cancel_order   CancelOrder — a build extension (the reference has no cancel RPC; SURVEY
 *                             §8(f) row 4): queues a cancel record for a resting order into the slice.
 *   me_service_market_data    StreamMarketData's MarketDataUpdate (proto:60-67) from the GPU book.
 *   me_service_updates        StreamOrderUpdates (proto/matching_engine.proto:34,71-91): drains the
 *                             OrderUpdate events the flushes produced, optionally for one client_id.
 *
 * Restart: the reference resumes only its OID counter from the DB (matching_engine_service.cpp:18-22,
 * storage.cpp:254-267). me_service_create does that and also rebuilds the books: every order the DB
 * shows resting (status NEW / PARTIALLY_FILLED, remaining_quantity > 0) is replayed into the backend
 * in OID order with its remainder, before the first SubmitOrder is matched, so it keeps its price-time
 * priority, can trade and can be cancelled.
 *
 * Symbols: any non-empty symbol is accepted (:66-71). The backend holds a fixed number of books; when
 * every book is taken, a new symbol takes over a book with no resting order and no record on its way
 * (the old symbol's book is reclaimed). Only when every book is in use is the order refused
 * (RESOURCE_EXHAUSTED, no OID).
 *
 * Capacity: a slice the backend refuses (its books near max_resting) is split and matched in parts;
 * a single LIMIT that still does not fit is answered in-band with an OrderUpdate REJECTED (reason
 * ME_RJ_CAPACITY) instead of stalling every later slice behind it. Deliberate deviation from the
 * reference, which has no capacity: admission counts every LIMIT as one that may rest (whether it fills
 * is only known once matched), so near max_resting a marketable LIMIT that would have filled completely is
 * refused too. max_resting is a deployment parameter sized to HBM; a deployment sizes it
 * above its resting high-water mark.
 */
#ifndef ME_SERVICE_H
#define ME_SERVICE_H

#include "me_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

/* OrderRequest (proto/matching_engine.proto:37-45). */
typedef struct me_order_request {
  const char* client_id;
  const char* symbol;
  int32_t order_type; /* OrderType; != LIMIT is MARKET */
  int32_t side;       /* Side */
  int64_t price;      /* raw scaled integer */
  int32_t scale;
  int32_t quantity;
} me_order_request;

/* OrderResponse (proto:47-51) + the gRPC status code of the call. */
typedef struct me_order_response {
  char order_id[32];      /* "OID-<n>", empty when none was allocated */
  int32_t success;
  int32_t grpc_status;    /* 0 OK; 2 UNKNOWN: normalize_to_q4 threw (price.hpp:16,23-24) */
  char error_message[64];
} me_order_response;

typedef struct me_service me_service;

/* engine: the shard the slices are matched on (NULL: submit works, flush fails loudly). The service
 * drives it from its own threads: no other caller may use the engine while the service lives.
 * symbols[num_symbols]: symbol strings pre-assigned to the engine's local ids 0..num_symbols-1; later
 * symbols take the following ids, up to the engine's num_symbols.
 * db_path: SQLite file (NULL: no persistence). Destroy does not flush: flush first. */
me_service* me_service_create(me_engine* engine, const char* const* symbols, uint32_t num_symbols,
                              const char* db_path);
void me_service_destroy(me_service* s);

/* A sharded deployment's matcher (matching_engine_amd/cluster.py): symbols live on
 * several engines (one per GPU, splitmix64(symbol) % G); the service on the persistence root hands
 * it each slice and gets back the merged outputs, exactly what one engine holding every symbol
 * would produce (me_collect's shapes: tape ordered by taker seq, results in slice order). */
typedef struct me_matcher {
  void* ctx;
  uint32_t num_symbols;  /* symbol ids it takes (the service interns up to this many) */
  uint32_t max_batch;    /* largest slice */
  uint64_t max_resting;  /* resting orders it holds at most (me_fill_bound's bound: max_resting + 2n) */
  /* Match one slice; outputs valid until the next call. ME_E_CAPACITY: refused, nothing of it was
   * applied (admission control; the slice stays queued). Any other nonzero: the slice is lost (the
   * service fails). */
  int (*match)(void* ctx, const me_order_soa* slice, size_t n, const me_fill** fills, size_t* n_fills,
               const me_order_result** results);
  /* me_book_orders' contract for one symbol (depth 0: the whole book). */
  int (*book)(void* ctx, uint32_t symbol, uint32_t depth, me_book_entry* bids, size_t bids_cap, size_t* n_bids,
              me_book_entry* asks, size_t asks_cap, size_t* n_asks, me_level* bid_levels, me_level* ask_levels,
              size_t* n_bid_levels, size_t* n_ask_levels);
  /* Optional, both or neither: match split in two, so the service keeps two slices in flight (slice k+1
   * is submitted before slice k is collected). submit applies the slice and returns a ticket
   * (ME_E_CAPACITY: refused, nothing applied); collect returns that ticket's outputs (valid until the
   * next collect). Tickets are collected in submission order, at most two outstanding. */
  int (*submit)(void* ctx, const me_order_soa* slice, size_t n, uint64_t* ticket);
  int (*collect)(void* ctx, uint64_t ticket, const me_fill** fills, size_t* n_fills, const me_order_result** results);
} me_matcher;

/* The service over a matcher instead of an engine (same contract otherwise). NULL on a bad matcher. */
me_service* me_service_create_matcher(const me_matcher* m, const char* const* symbols, uint32_t num_symbols,
                                      const char* db_path);

/* Always returns 0 (the RPC itself succeeded or failed in-band, like the reference). */
int me_service_submit_order(me_service* s, const me_order_request* req, me_order_response* resp);

/* n SubmitOrder calls in order (what a server's handler threads do one request at a time), for
 * drivers and benchmarks holding many requests at once; resps[i] answers reqs[i]. */
int me_service_submit_orders(me_service* s, const me_order_request* reqs, size_t n, me_order_response* resps);

/* Submitted orders not matched yet (the open slice, closed slices, the slice being matched). */
size_t me_service_pending(const me_service* s);
/* Next OID number the service will allocate. */
uint64_t me_service_next_oid(const me_service* s);

/* Match and persist every slice submitted before the call, oldest first (matching runs on the calling
 * thread, ahead of the service's persister thread by at most 4 slices, so the engine overlaps
 * SQLite); returns once every matched slice's OrderUpdates are out and its transaction committed.
 * Any output may be NULL;
 * the outputs cover the records this call matched, in submission order (tape offsets into the
 * concatenated tape): *n_results records, out_seq[i] their numeric OIDs. The capacities are checked
 * before anything is matched (results_cap >= me_service_pending, fills_cap >= me_fill_bound of it),
 * else ME_E_INVALID and nothing happens.
 * A slice the engine accepted is never matched again. When its transaction fails (e.g. SQLITE_BUSY
 * past the 5 s busy timeout) the matched slice is kept in memory, later slices still match, and every
 * later flush first retries the kept ones in order; the call returns ME_E_SQLITE meanwhile
 * (me_service_unpersisted counts the records waiting). */
int me_service_flush(me_service* s, me_fill* out_fills, size_t fills_cap, size_t* n_fills,
                     me_order_result* out_results, uint64_t* out_seq, size_t results_cap, size_t* n_results);
/* Matched records whose SQLite transaction has not committed yet (queued for the persister, or kept
 * after a failed transaction). me_service_pending + me_service_unpersisted is 0 exactly when every
 * submitted order is matched and committed. */
size_t me_service_unpersisted(const me_service* s);
/* Background flusher (one thread): a slice closes at slice_orders records (0 or more than the
 * engine's max_batch: max_batch) or once it is interval_us old (0: 1000), and is flushed at once.
 * Errors go to me_service_last_error. me_service_stop joins it and waits for the persister to
 * finish what it matched. */
int me_service_start(me_service* s, uint32_t interval_us, uint32_t slice_orders);
int me_service_stop(me_service* s);

/* Level view of GetOrderBook for a symbol string (top depth levels per side, aggregates; depth 0:
 * no levels). */
int me_service_book(me_service* s, const char* symbol, me_level* bids, me_level* asks, size_t depth,
                    size_t* n_bids, size_t* n_asks);

/* Order (proto/matching_engine.proto:16-23): one resting order of an OrderBookResponse. */
typedef struct me_book_order {
  char order_id[32];  /* "OID-<n>" */
  char client_id[64]; /* the submitting client ("" for orders that did not come through this service) */
  int64_t price;      /* Q4 */
  int32_t scale;      /* 4 */
  int32_t quantity;   /* the resting (unfilled) quantity */
  int32_t side;       /* ME_SIDE_BUY / ME_SIDE_SELL */
  int32_t pad;
} me_book_order;

/* GetOrderBook (matching_engine_service.cpp:123-129) in the reference's shape: OrderBookResponse
 * {repeated Order bids; repeated Order asks} (proto:57-60), bids best price first, asks best price
 * first, FIFO (time) order within a price; from one device snapshot launch (me_book_orders). depth:
 * price levels per side (0: the whole book, as OrderBookRequest carries no depth). Counts are exact
 * even when a cap is short; unknown symbol: empty. */
int me_service_order_book(me_service* s, const char* symbol, uint32_t depth, me_book_order* bids, size_t bids_cap,
                          size_t* n_bids, me_book_order* asks, size_t asks_cap, size_t* n_asks);

/* CancelOrder request (build extension, mirrors OrderRequest's conventions). */
typedef struct me_cancel_request {
  const char* client_id;
  const char* symbol;
  const char* order_id; /* "OID-<n>" of the order to cancel */
} me_cancel_request;

/* Validation (first failing check wins, in-band like SubmitOrder :66-83): "symbol is required",
 * "order_id is invalid" (not "OID-<n>", n >= 1), "order belongs to another client" (the target is a
 * resting or pending order of a different client_id). An accepted cancel consumes NO OID: its stream
 * position is the last OID allocated (a cancel record may repeat the previous seq, me_engine.h), so
 * accepted orders keep the reference's gap-free OID sequence. It answers success=1 with order_id = the
 * TARGET's id; whether it removed anything arrives as an OrderUpdate after the flush (CANCELED with
 * the removed quantity, or REJECTED when the target was not resting on that symbol). */
int me_service_cancel_order(me_service* s, const me_cancel_request* req, me_order_response* resp);

/* OrderUpdate (proto:71-91). Events per flushed record, in slice order: for each fill the maker's
 * update then the taker's (fill price/qty, remaining after the fill, PARTIALLY_FILLED / FILLED);
 * then a closing taker update when no fill closed it (NEW resting, CANCELED market remainder,
 * REJECTED); a cancel record emits CANCELED (remaining = removed qty) or REJECTED for its target. */
typedef struct me_order_update {
  char order_id[32];
  char client_id[64];
  char symbol[32];
  int32_t status;            /* ME_ST_* */
  int32_t scale;             /* 4: prices are Q4 */
  int64_t fill_price;        /* Q4, 0 without a fill */
  int32_t fill_quantity;
  int32_t remaining_quantity;
} me_order_update;

/* Drain up to cap queued updates (client_id NULL or "": every client; else only that client's,
 * leaving the others queued). *n = updates written; returns ME_OK. */
int me_service_updates(me_service* s, const char* client_id, me_order_update* out, size_t cap, size_t* n);
/* Events dropped because the queue held 2^24 undrained updates (the oldest go first; each drop also
 * sets me_service_last_error). */
uint64_t me_service_updates_dropped(const me_service* s);
/* Books handed from an idle symbol to a new one since create, and resting orders replayed into the
 * books from the DB at create (restart recovery). */
int me_service_stats(const me_service* s, uint64_t* reclaimed_books, uint64_t* recovered_orders);

/* MarketDataUpdate (proto:60-67) for StreamMarketData, from the GPU book: best bid / ask (Q4,
 * scale 4) and the total quantity resting there (saturated to int32). The reference's
 * Storage::best_bid / best_ask SQL (storage.cpp:212-252) query side=0 / side=1, which the schema's
 * CHECK side IN (1,2) never admits, so they always return nullopt; here a missing side reads 0
 * with has_bid / has_ask = 0 (proto3 default). Unknown symbol: both sides missing. */
typedef struct me_market_data {
  int64_t best_bid;
  int64_t best_ask;
  int32_t scale;
  int32_t bid_size;
  int32_t ask_size;
  int32_t has_bid;
  int32_t has_ask;
  int32_t pad;
} me_market_data;

int me_service_market_data(me_service* s, const char* symbol, me_market_data* out);

int me_service_last_error(const me_service* s, char* buf, size_t cap);

#ifdef __cplusplus
}
#endif
#endif /* ME_SERVICE_H */

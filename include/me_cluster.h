/*
 * me_cluster.h — the sharded deployment in C++ (north star: "symbols are
 * hash-partitioned across the 8 GPUs of one node with no cross-GPU matching; RCCL over xGMI is used
 * only to gather per-GPU trade tapes and book snapshots to the host for the storage/SQLite path").
 *
 * One process per GPU. Every rank owns the books of the symbols me_shard_of(symbol, world) == rank
 * (splitmix64 % world) on its own engine; rank 0 — the persistence root — hosts the SubmitOrder
 * service and reaches the shards through me_cluster_matcher(), a me_matcher the service is created
 * over (me_service_create_matcher). The other ranks sit in me_cluster_serve(). Per slice:
 *
 *   SUBMIT   rank 0 splits the slice by owner (local symbol ids, global seqs kept), scatters the parts
 *            (grouped ncclSend / ncclRecv, device buffers), every rank asks its engine's admission
 *            control and a MIN all-reduce decides (all-or-none: a refusal anywhere applies nothing),
 *            then every rank matches its part (me_submit_device_limits) into device staging buffers.
 *   COLLECT  tape lengths gathered to rank 0, then each rank's tape + results (ncclSend to 0, unpadded);
 *            rank 0 merges the tapes by taker seq (k-way, u64 keys) — every taker's fills live on one
 *            shard, so this is exactly the single-engine tape — and scatters the results back to slice
 *            order with tape offsets against the merged tape.
 *   BOOK     GetOrderBook of one symbol: its owner runs the device snapshot (me_book_orders) and
 *            sends the entries and levels to rank 0.
 *   SNAPSHOT the periodic book snapshot: every rank's top-N levels of all its symbols
 *            (me_book_levels_all, one launch) gathered to rank 0.
 *   STOP     the serve loops return.
 * The service keeps two slices in flight through the matcher's submit / collect (SUBMIT of slice k+1
 * runs before COLLECT of slice k), so the shards match k+1 while rank 0 merges and persists k.
 *
 * Every command ends in a status all-reduce, so a failure on any rank sends every rank down the same
 * path (no rank is left waiting in a collective the others skipped); a slice that failed after any
 * rank applied it fails the cluster (sticky, ME_E_STATE), like an engine that lost a batch.
 *
 * Transports: ME_TRANSPORT_RCCL — RCCL over xGMI with device buffers (librccl, loaded at run time;
 * the unique id is handed out over a TCP bootstrap from rank 0's addr:port); ME_TRANSPORT_TCP — the
 * same protocol over host buffers and a TCP star around rank 0 (the CPU tests, or GPUs without a
 * shared RCCL domain). Reference: the reference has no multi-process path at all (one gRPC server
 * over one SQLite file, src/server/main.cpp:32-38); this is the build's extension behind its C-ABI.
 */
#ifndef ME_CLUSTER_H
#define ME_CLUSTER_H

#include "me_engine.h"
#include "me_service.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { ME_TRANSPORT_RCCL = 0, ME_TRANSPORT_TCP = 1 };

typedef struct me_cluster_config {
  uint32_t rank;         /* this process */
  uint32_t world;        /* processes (GPUs) */
  uint32_t num_symbols;  /* global symbols, ids 0 .. num_symbols-1 */
  uint32_t max_batch;    /* largest slice */
  int32_t transport;     /* ME_TRANSPORT_RCCL / ME_TRANSPORT_TCP */
  int32_t device;        /* HIP device of this rank (RCCL) */
  const char* addr;      /* rank 0's IPv4 address (bootstrap; every message with TCP) */
  uint32_t port;         /* rank 0 listens here */
  uint32_t timeout_ms;   /* bootstrap connect / accept timeout (0: 60000) */
} me_cluster_config;

/* A shard's book when it is not an engine (the CPU tests put the oracle here). Local symbol ids. */
typedef struct me_shard_ops {
  void* ctx;
  uint64_t max_resting;  /* resting orders it holds at most */
  /* may be NULL (always admits): would a part with n_rest LIMIT records be admitted? */
  int (*admit)(void* ctx, uint64_t n_rest, int* ok);
  /* me_collect's contract: outputs valid until the next call */
  int (*match)(void* ctx, const me_order_soa* part, size_t n, const me_fill** fills, size_t* n_fills,
               const me_order_result** results);
  /* me_book_orders' contract */
  int (*book)(void* ctx, uint32_t symbol, uint32_t depth, me_book_entry* bids, size_t bids_cap, size_t* n_bids,
              me_book_entry* asks, size_t asks_cap, size_t* n_asks, me_level* bid_levels, me_level* ask_levels,
              size_t* n_bid_levels, size_t* n_ask_levels);
  /* me_book_levels_all's contract over its local symbols */
  int (*levels_all)(void* ctx, uint32_t depth, me_level* levels, uint32_t* counts);
} me_shard_ops;

typedef struct me_cluster me_cluster;

/* Global symbol ids of rank's shard, ascending (local id = position). Returns the count; writes at
 * most cap ids (out may be NULL). */
size_t me_cluster_shard_symbols(uint32_t num_symbols, uint32_t world, uint32_t rank, uint32_t* out, size_t cap);

/* Collective over all ranks (every rank calls it). The shard is `ops` when given, else an engine
 * created here from engine_cfg: its base_price indexes GLOBAL symbols, and num_symbols / symbol_ids
 * are replaced by this rank's share (device = cfg->device, max_batch = cfg->max_batch). NULL on
 * failure (me_cluster_last_error(NULL, ...)). */
me_cluster* me_cluster_create(const me_cluster_config* cfg, const me_config* engine_cfg, const me_shard_ops* ops);
/* Rank 0 only; returns after STOP has reached every rank. Other ranks: leave serve, then destroy. */
int me_cluster_stop(me_cluster* c);
void me_cluster_destroy(me_cluster* c);

/* Ranks != 0: run rank 0's commands until STOP (ME_OK) or a transport failure. */
int me_cluster_serve(me_cluster* c);

/* Rank 0. submit: the slice (global symbol ids, ascending seqs) to every shard; ME_E_CAPACITY when a
 * shard's admission control refused its part (nothing of it was applied anywhere). At most two
 * tickets outstanding. collect: the merged outputs of the oldest ticket, exactly what one engine
 * holding every symbol returns (tape ordered by taker seq, results in slice order); valid until the
 * next collect (at world 1 they are rank 0's engine slot outputs, in place). match = submit + collect. */
int me_cluster_submit(me_cluster* c, const me_order_soa* slice, size_t n, uint64_t* ticket);
int me_cluster_collect(me_cluster* c, uint64_t ticket, const me_fill** fills, size_t* n_fills,
                       const me_order_result** results);
int me_cluster_match(me_cluster* c, const me_order_soa* slice, size_t n, const me_fill** fills, size_t* n_fills,
                     const me_order_result** results);
/* Rank 0: me_book_orders for a global symbol, answered by its owner (depth 0: the whole book; level
 * arrays are then not written). */
int me_cluster_book(me_cluster* c, uint32_t symbol, uint32_t depth, me_book_entry* bids, size_t bids_cap,
                    size_t* n_bids, me_book_entry* asks, size_t asks_cap, size_t* n_asks, me_level* bid_levels,
                    me_level* ask_levels, size_t* n_bid_levels, size_t* n_ask_levels);
/* Rank 0: top `depth` levels of every global symbol from every shard:
 * levels[(symbol * 2 + side) * depth + k] (zeros past a side's levels), counts[symbol * 2 + side]. */
int me_cluster_snapshot(me_cluster* c, uint32_t depth, me_level* levels, uint32_t* counts);
/* Rank 0: the me_matcher over this cluster for me_service_create_matcher (submit / collect set: the
 * service keeps two slices in flight). max_resting = the sum over the shards. */
int me_cluster_matcher(me_cluster* c, me_matcher* out);

/* Counters: slices matched, bytes moved by the transport (this rank, both directions). */
int me_cluster_stats(const me_cluster* c, uint64_t* slices, uint64_t* bytes);
/* Rank 0's wall time per protocol phase since create, in seconds: [0] split (owner counts, stable pack:
 * rank 0's part straight into its engine's pinned slot inputs), [1] control (command broadcast), [2]
 * scatter (H2D + parts over the transport), [3] admission vote, [4] match (enqueue on every shard), [5]
 * collect (rank 0's own outputs: waits for its engine), [6] gather (sizes, tapes and results to rank 0,
 * D2H), [7] merge (results to slice order, tapes by taker); parts of [0]: [8] the owner-count pass, [9]
 * waiting for rank 0's engine slot inputs. Writes min(n, 10) values, returns 10. */
int me_cluster_phases(const me_cluster* c, double* seconds, size_t n);
int me_cluster_last_error(const me_cluster* c, char* buf, size_t cap);
/* Rank 0's host work per slice at `world` shards, without GPUs or a transport: the exact split and merge
 * code of me_cluster_submit / me_cluster_collect over `slice` (global symbol ids < num_symbols), with
 * synthetic shard outputs of fills_per_order fills per record on average, `iters` times. seconds[0] = the
 * owner-count pass, [1] = the pack, [2] = the merge, per slice; [3] = the merged tape's fills. */
int me_cluster_host_probe(uint32_t world, uint32_t num_symbols, const me_order_soa* slice, size_t n,
                          double fills_per_order, uint32_t iters, double* seconds);

#ifdef __cplusplus
}
#endif
#endif /* ME_CLUSTER_H */

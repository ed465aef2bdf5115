// me_layout.hpp — HBM layout of the resident books and of one in-flight batch.
//
// Shared by the gfx950 kernels (me_kernels.hip) and the host engine (me_engine.cpp).
// Everything is plain-old-data; the host allocates, the kernels own the contents.
//
// Book of one shard:
//   levels [S][L]   16 B {total, head chunk, tail chunk}: the fixed-depth price ladder. Bids and
//                   asks share one ladder per symbol: after every order best_bid < best_ask, so
//                   a level's side is implied by its position.
//   occ    [S][L/64] occupancy bitmap of the ladder (bit set <=> total > 0).
//   sym    [S]      32 B per-symbol scalars (window base, best bid/ask level, chunk free list).
//   tend   [S][L]   slots written in each level's tail chunk (appends need no chunk read).
//   chunks [NC]     FIFO storage: a level's queue is a doubly linked list of 256-B chunk blocks of
//                   ME_C slots {seq u64, qty i32} (SoA inside the block); a wave reads one chunk per load.
//                   A slot is live iff qty > 0. Every linked chunk holds >= 1 live order (a chunk
//                   emptied by cancels is unlinked at once), so chunks in use <= resting orders.
//   loc    [max_seq] seq -> global slot (chunk * ME_C + slot) for cancels.
//   fcache [S][64]  free chunk ids a symbol keeps between launches (the register-ladder kernel
//                   holds them in one VGPR: pops and pushes never touch memory).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "me_engine.h"

namespace me {

constexpr int ME_C = 16;                 // slots per chunk (one wave-load of qty + seq)
constexpr uint32_t NIL = 0xFFFFFFFFu;
constexpr int MAX_SORT_TILES = 256;      // sort tiles per pass (tile = records / workgroup >= 1024)
constexpr int TILE_TAPE = 64;            // records per tape tile (one side-job wave, or one k_tape_compact workgroup)
constexpr int MAX_DIGIT_BITS = 11;       // radix digit width (LDS histogram of 2048 bins)
constexpr uint32_t LDS_MAX_LEVELS = 1024; // ladders up to this depth are staged in LDS (17.5 KB/wave)

// Sticky error bits (BookDev::err).
enum : uint32_t {
  ERR_CHUNK_OOM = 1u,
  ERR_SCRATCH_OOM = 2u,
  ERR_INCONSISTENT = 4u,
};

struct alignas(16) Level {
  long long total;   // live quantity on the level (0 <=> empty, head == tail == NIL)
  uint32_t head;     // first chunk of the FIFO
  uint32_t tail;     // last chunk (appends go here)
};

struct alignas(16) ChunkHdr {
  uint32_t next;   // next chunk of the level FIFO, or of the symbol free list
  uint32_t prev;   // previous chunk of the level FIFO (NIL at the head)
  uint32_t level;  // level index the chunk belongs to
  uint32_t owner;  // symbol that allocated the chunk (chunks never change symbol)
};

// One FIFO chunk, 256 B: header, then the 16 slot quantities (one 64-B segment), then the 16 slot
// seqs (two 64-B segments). One pointer reaches all of it; slot id g = chunk * ME_C + slot.
struct alignas(256) Chunk {
  ChunkHdr hdr;
  uint32_t pad[12];
  int qty[ME_C];
  unsigned long long seq[ME_C];
};
static_assert(sizeof(Chunk) == 256, "chunk block must be 256 B");

__host__ __device__ __forceinline__ int& cq_at(Chunk* c, size_t g) { return c[g / ME_C].qty[g % ME_C]; }
__host__ __device__ __forceinline__ unsigned long long& cs_at(Chunk* c, size_t g) { return c[g / ME_C].seq[g % ME_C]; }

struct alignas(32) SymState {
  long long base;      // price_q4 of level 0
  int best_bid;        // highest occupied bid level, -1 if none
  int best_ask;        // lowest occupied ask level, L if none
  uint32_t free_head;  // chunk free list of this symbol
  uint32_t resting;    // live resting orders
  uint32_t nfree;      // free chunk ids parked in fcache[sym][0..nfree) (register-ladder kernel)
  uint32_t pad;
};

// One bucketed record (24 B, AoS): the bucket job writes it as one unit, so a record's bytes land
// in one or two lines instead of four SoA arrays' lines (fewer partially written lines per XCD).
struct alignas(8) BkRec {
  uint64_t seq;
  int64_t px;
  int32_t qty;
  uint32_t ok;  // batch index | (kind & 15) << BK_KIND_SHIFT
};

struct BookDev {
  Level* levels;
  unsigned long long* occ;
  uint8_t* tend;          // [S][L] slots written in the level's tail chunk (valid when tail != NIL)
  SymState* sym;
  Chunk* chunks;          // [NC] FIFO chunk blocks
  uint32_t* loc;
  uint32_t* chunk_top;
  uint32_t* fcache;       // [S][64] free chunk ids parked between launches (register-ladder kernel)
  uint32_t* err;
  const uint32_t* gsym;  // [S] id written into me_fill.symbol
  unsigned long long* dbg;  // [S][8] phase cycles, diagnostic (-DME_STAMPS) builds only
  unsigned long long max_seq;
  uint32_t nchunks;
  uint32_t S;
  uint32_t L;
  uint32_t Lwords;
};

struct BatchDev {
  const uint64_t* seq;
  const int64_t* px;
  const int32_t* qty;
  const uint32_t* sym;
  const uint8_t* kind;
  uint32_t n;
  const uint32_t* skeys;    // symbol of each grouped position (ascending)
  const uint32_t* perm;     // grouped position -> batch index
  me_order_result* res;     // [n], batch order
  uint32_t* fstart;         // [n] first fill of the record in scratch
  uint32_t* tile_sum;       // [ceil(n / TILE_TAPE)] fills per tape tile
  me_fill* scratch;
  unsigned long long scratch_cap;
  unsigned long long* scratch_top;
  // Register-ladder kernel: symbol s owns the scratch slab [s * slab, (s + 1) * slab); a wave whose
  // fills may outgrow it reserves the rest of its batch bound at ovf_base + atomicAdd(scratch_top).
  uint32_t slab;
  unsigned long long ovf_base;
  // Single-pass grouping sort (bins are symbols): run(s) = [bin_start[s], bin_start[s + 1]).
  const uint32_t* bin_start;
  // Bucketed grouping (register-ladder kernel, replaces the sort): k_bucket appends every record
  // to the bucket of its bin (symbol, S = bad symbol) in arbitrary order; bucket b holds its first
  // bcap records at [b * bcap, (b + 1) * bcap) and bcnt[b] counts all of them. k_match_reg orders
  // a bucket by batch index on chip and resets bcnt; a bin with more than bcap records rescans the
  // batch in order instead. Null bcnt: the sort path.
  uint32_t* bcnt;        // [(S + 1) * BK_CNT_STRIDE]
  const struct BkRec* b_rec;  // [(S + 1) * bcap] bucketed records
  uint32_t bcap;
  // Deep-window path (L > LDS_MAX_LEVELS): a symbol with >= hot_min records in the batch is handed
  // from k_match<LAD_HBM> to k_match_hot (one workgroup, LDS-resident ladder window) through
  // hot[1 + i], i < hot[0] (the count; zeroed before each match launch). hot_min 0: no hand-off.
  uint32_t* hot;
  uint32_t hot_min;
};
constexpr uint32_t HOT_MAX = 1024;   // hot symbols per batch (more are matched in place)
constexpr uint32_t HOT_GRID = 256;   // k_match_hot workgroups: one per CU (the LDS window fills it)
constexpr uint32_t HOT_MIN_RECORDS = 64;  // threshold the tests use (ME_HOT_MIN, opt-in)
// Batches per register-ladder launch at most (me_config.batches_per_launch). One launch matches a
// group of up to ME_GMAX batches: every symbol's wave runs through its records of all of them in
// order, so a launch costs the heaviest symbol's share of the whole group rather than the sum of
// each batch's heaviest share.
#ifndef ME_GROUP_MAX
#define ME_GROUP_MAX 64
#endif
constexpr int ME_GMAX = ME_GROUP_MAX;
constexpr uint32_t ME_DEFAULT_GROUP = 32;

// Side jobs of one pipelined register-ladder launch (me_match_reg.hip), run by each workgroup's
// extra waves while its matching waves work on group J-1: group the batches of group J into their
// buckets (and clear the output counters they will use), compact the tapes of group J-2.
struct AuxBucket {  // bucket + clear job of one batch
  const uint32_t* sym;
  const uint64_t* seq;
  const int64_t* px;
  const int32_t* qty;
  const uint8_t* kind;
  uint32_t n;
  uint32_t zero_tiles;
  uint32_t* bcnt;
  struct BkRec* b_rec;
  me_order_result* bres;  // the batch's results: unknown-symbol records are rejected by the bucket job
  uint32_t* bfstart;
  uint32_t* zero_tile_sum;
  unsigned long long* zero_top;
};
struct AuxTape {  // tape job of one batch
  const uint32_t* tile_sum;
  me_order_result* res;
  const uint32_t* fstart;
  const me_fill* scratch;
  me_fill* tape;
  unsigned long long* tape_count;
  uint32_t tn;
  uint32_t pad;
};
struct AuxDev {
  uint32_t S;
  uint32_t nwg;  // workgroups that run side jobs (those of the first dispatch round)
  uint32_t nb;   // bucket jobs (batches of group J)
  uint32_t nt;   // tape jobs (batches of group J-2)
  unsigned long long tape_cap;
  unsigned long long* fills_acc;
  AuxBucket b[ME_GMAX];
  AuxTape t[ME_GMAX];
};

constexpr int BK_CAP = 128;          // records per bucket (two 64-record blocks)
constexpr int BK_KIND_SHIFT = 28;    // BkRec::ok: kind bits above the batch index
constexpr uint32_t BK_IDX_MASK = (1u << BK_KIND_SHIFT) - 1u;
constexpr uint32_t BK_MAX_BATCH = 1u << 25;  // sort key (index << 7 | bucket slot) fits 32 bits
constexpr int BK_CNT_STRIDE = 32;    // bcnt[b * stride]: one 128-B line per counter (atomics on one
                                     // line serialise: packed counters made k_bucket 6x slower)

}  // namespace me

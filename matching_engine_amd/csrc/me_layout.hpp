// me_layout.hpp — HBM layout of the resident books and of one in-flight batch.
//
// Shared by the gfx950 kernels (me_kernels.hip, me_match_reg.hip) and the host engine
// (me_engine.cpp). Everything is plain-old-data; the host allocates, the kernels own the contents.
//
// Book of one shard. Prices are unbounded int64 Q4 (include/domain/price.hpp:6):
//   levels [S][L]   16 B {total, head chunk, tail chunk}: the fixed-depth WINDOW of price levels
//                   [base, base + L). Bids and asks share it: after every order best_bid < best_ask,
//                   so a level's side is implied by its position.
//   far    arena    32 B {price, total, head, tail, tend}: levels OUTSIDE the window, one sorted array
//                   per (symbol, side) located by fdir [S][2]. Side 0 holds bids below the window
//                   (ascending price, best last), side 1 asks above it (descending price, best last).
//                   Invariant: no bid rests above the window and no ask below it; a rest that would
//                   break this re-centres the window first. Unbounded: a side outgrowing its region
//                   moves to a larger one (me_far.hpp).
//   occ    [S][L/64] occupancy bitmap of the window (bit set <=> total > 0).
//   sym    [S]      64 B per-symbol scalars (window base, best bid/ask level, chunk free list,
//                   far-level counts).
//   tend   [S][L]   slots written in each level's tail chunk (appends need no chunk read).
//   chunks [NC]     FIFO storage: a level's queue is a doubly linked list of 256-B chunk blocks of
//                   ME_C slots {seq u64, qty i32} (SoA inside the block) plus the level's price; a
//                   wave reads one chunk per load. A slot is live iff qty > 0. Every linked chunk
//                   holds >= 1 live order (a chunk emptied by cancels is unlinked at once), so
//                   chunks in use <= resting orders.
//   loc    [R]      seq ring: loc[seq & (R - 1)] = global slot (chunk * ME_C + slot) of the order
//                   that rested with that seq. Never deleted; a lookup verifies the slot still
//                   holds the seq. Entries of orders older than the ring horizon are copied into
//                   the old-order table by k_seq_sweep before anything could overwrite them.
//   old    [H]      old-order table (open addressing by seq): rebuilt by k_seq_sweep.
//   fcache [S][64]  free chunk ids a symbol keeps between launches (the register-window kernel
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

// Batches per register-ladder launch at most (me_config.batches_per_launch). One launch matches a
// group of up to ME_GMAX batches: every symbol's wave runs through its records of all of them in
// order, so a launch costs the heaviest symbol's share of the whole group rather than the sum of
// each batch's heaviest share.
#ifndef ME_GROUP_MAX
#define ME_GROUP_MAX 32  // (the launch arguments k_match_reg copies to LDS grow with it: 32 leaves room
                         // for two workgroups per CU)
#endif
constexpr int ME_GMAX = ME_GROUP_MAX;
constexpr uint32_t ME_DEFAULT_GROUP = 32;

// Sticky error bits (BookDev::err).
enum : uint32_t {
  ERR_CHUNK_OOM = 1u,
  ERR_SCRATCH_OOM = 2u,
  ERR_INCONSISTENT = 4u,
  ERR_FAR_OOM = 8u,      // the far arena is exhausted (sized so admission control rules it out: internal)
  ERR_OLD_OOM = 16u,     // the old-order table overflowed (sized from max_resting)
  ERR_SEQ_ORDER = 32u,   // seqs not ascending across the stream (API precondition, seq_follows)
  ERR_SEQ_SPAN = 64u,    // one launch group spans >= the seq ring (raise me_config.seq_ring)
};

// API precondition the seq ring relies on: seqs ascend through an engine's stream. A CANCEL record
// (it never rests, so no ring entry is keyed by its seq) may repeat the previous record's seq: the
// service gives a cancel the last allocated OID as its stream position instead of consuming one.
__host__ __device__ __forceinline__ bool seq_follows(unsigned long long prev, unsigned long long cur, uint32_t kind) {
  return cur > prev || (cur == prev && ((kind >> 3) & 1u) != 0u);
}

struct alignas(16) Level {
  long long total;   // live quantity on the level (0 <=> empty, head == tail == NIL)
  uint32_t head;     // first chunk of the FIFO
  uint32_t tail;     // last chunk (appends go here)
};

// Written as one 16-B store whenever a chunk joins a level. The price (not a window index) names the
// level, so re-centring a window never touches chunks.
struct alignas(16) ChunkHdr {
  uint32_t next;    // next chunk of the level FIFO, or of the symbol free list
  uint32_t prev;    // previous chunk of the level FIFO (NIL at the head)
  long long price;  // price_q4 of the level the chunk belongs to
};

// One FIFO chunk, 256 B: header and owner (one 64-B segment), then the 16 slot quantities (one 64-B
// segment), then the 16 slot seqs (two 64-B segments). One pointer reaches all of it; slot id
// g = chunk * ME_C + slot.
struct alignas(256) Chunk {
  ChunkHdr hdr;
  uint32_t owner;  // symbol that took the chunk from the global pool (written whenever the pool hands
                   // the chunk out: a reclaimed chunk may go to another symbol)
  uint32_t pad[11];
  int qty[ME_C];
  unsigned long long seq[ME_C];
};
static_assert(sizeof(Chunk) == 256, "chunk block must be 256 B");

__host__ __device__ __forceinline__ int& cq_at(Chunk* c, size_t g) { return c[g / ME_C].qty[g % ME_C]; }
__host__ __device__ __forceinline__ unsigned long long& cs_at(Chunk* c, size_t g) { return c[g / ME_C].seq[g % ME_C]; }

struct alignas(64) SymState {
  long long base;      // price_q4 of level 0 of the window
  int best_bid;        // highest occupied bid level of the window, -1 if none
  int best_ask;        // lowest occupied ask level of the window, L if none
  uint32_t free_head;  // chunk free list of this symbol
  uint32_t resting;    // live resting orders (window and far levels)
  uint32_t nfree;      // free chunk ids parked in fcache[sym][0..nfree) (register-window kernel)
  uint32_t nfar[2];    // far levels: [0] bids below the window, [1] asks above it
  uint32_t pad[5];
};
static_assert(sizeof(SymState) == 64, "SymState is one 64-B segment");

// A price level outside its symbol's window (BookDev::far). Same FIFO chunks as window levels.
struct alignas(32) FarLevel {
  long long price;
  long long total;
  uint32_t head, tail;
  uint32_t tend;  // slots written in the tail chunk
  uint32_t pad;
};
static_assert(sizeof(FarLevel) == 32, "FarLevel is 32 B");

// Where the far levels of one (symbol, side) live (BookDev::fdir, me_far.hpp): entries
// [off, off + cap) of the far arena. Every side starts in its own inline region of `far_levels`
// entries; a side that outgrows it moves into a region twice as large in the active half of the arena
// (and again, doubling, as it grows), and k_seq_sweep's collection pass brings every moved side back to
// a compact region of the other half — or to its inline region when it fits again.
struct alignas(16) FarDir {
  unsigned long long off;
  uint32_t cap;
  uint32_t pad;
};
// BookDev::far_ctl words: the allocation tops of the two halves, the active half, the collection's ticket
enum : uint32_t { FC_TOP0 = 0, FC_TOP1 = 1, FC_HALF = 2, FC_TICKET = 3, FC_N = 4 };

// Old-order table entry: the claim word {epoch, slot} is CAS'd by k_seq_sweep; an entry is empty
// unless its epoch is the current one (no clearing pass).
struct alignas(16) OldEnt {
  uint32_t epoch;
  uint32_t slot;
  unsigned long long seq;
};

// Seq-ring horizon, double-buffered: k_seq_sweep reads state[p] and writes state[p ^ 1]; the match
// launches after it read state[p ^ 1] (BookDev::sq_idx). Every live order with seq >= horizon has
// an intact ring entry; every older live order is in the old-order table of `epoch`.
struct alignas(32) SeqState {
  unsigned long long horizon;
  unsigned long long last;   // largest seq of the stream so far (0 = none)
  uint32_t epoch;
  uint32_t pad[3];
};

// One bucketed record (24 B, AoS): the bucket job writes it as one unit, so a record's bytes land
// in one or two lines instead of four SoA arrays' lines (fewer partially written lines per XCD).
struct alignas(8) BkRec {
  uint64_t seq;
  int64_t px;
  int32_t qty;
  uint32_t ok;  // batch index | (kind & 15) << BK_KIND_SHIFT
};

// A symbol the register-window kernel handed to its continuation launch (me_match_reg.hip): its
// records from position `pos` (in the symbol's batch order) of batch `g` of the group on. Written
// before the record at `pos` changed anything; wptr / wend: the scratch run of batch g.
struct Handoff {
  uint32_t s, g, pos, nsg;
  uint32_t wptr, wend;
  uint32_t pad[2];
};

// ---- hot symbols in aggregate form (me_agg.hip) ------------------------------------
// A hot symbol's records are matched against LEVEL TOTALS only (one serial wave: which levels a taker
// empties, how much it takes from the last, where a remainder rests), logged as events; the FIFO
// detail — which makers each take consumed — is resolved afterwards for all levels in parallel.
struct AggEv {       // one event of the log, in record order
  uint32_t lvl;      // window level
  uint32_t j;        // grouped position of the record | AGG_TAKE for a take
  int32_t qty;       // quantity taken from / rested on the level
  uint32_t pad;
};
constexpr uint32_t AGG_TAKE = 1u << 31;
// Grouped launches (k_agg_gwalk -> k_agg_gres) log 8-B events: the level (L <= 128) and the record's
// number in the symbol's walk order (< ME_GMAX x BK_CAP) in one word. The records' seqs (offsets from the
// group's first seq) and grouped positions sit beside the log in two arrays the walk writes 64 at a time,
// so the resolve reads a seq from the symbol's own small array instead of gathering it from the batches.
struct AggGEv {
  uint32_t w;        // level | record << AGG_GREC_SHIFT | AGG_TAKE for a take
  int32_t qty;
};
constexpr uint32_t AGG_GREC_SHIFT = 7;
constexpr uint32_t AGG_GLVL_MASK = (1u << AGG_GREC_SHIFT) - 1u;
constexpr uint32_t AGG_MAX_L = 32768;  // windows up to this depth (level histogram in LDS)
struct AggRec {      // a record the walk handled (indexed by grouped position)
  int32_t filled, rem;
  uint32_t st;       // status | reason << 8
  uint32_t ev_lo;    // its first take event (log index) ...
  uint32_t ev_n;     // ... and its take events
  uint32_t pad;
};
struct AggSeg {      // the events of one (slot, level), in log order: evs[start, start + cnt)
  uint32_t slot, lvl, start, cnt;
};
struct AggSegS {     // what the first per-level pass found (k_agg_levels), for the second (k_agg_place)
  unsigned long long C;   // quantity taken from the level by the batch
  unsigned long long T0;  // live quantity of the initial FIFO if the takes exhausted it, else ~0
  uint32_t newhead;       // first surviving chunk of the initial FIFO (NIL: none)
  uint32_t mk_base, nmk;  // consumed makers in AggDev::mk
  uint32_t fr_base, nfreed;  // initial chunks the takes emptied, in AggDev::fr
  uint32_t need;          // chunks the surviving rests need beyond the tail's free slots
  uint32_t d_off;         // this level's share of the slot's deficit (need beyond its own freed chunks)
  uint32_t ks;            // surviving rests
};
struct AggMk {       // a consumed maker: seq and the end of its interval in the level's maker space
  unsigned long long seq, end;
};
struct AggSlot {     // one hot symbol of the launch (index = k_hot_pick's hand-off index)
  uint32_t s, lo, hi, pos;   // symbol, grouped records [lo, hi), first record left to k_match_hot_cont
                             // (grouped launches: lo = the 8-B events the log region holds before the
                             // records' seq array, hi = that array's length; pos = the hand-off batch)
  unsigned long long wbase;  // scratch run
  long long base;
  uint32_t ev_base, ev_cnt, seg_base, nseg;
  uint32_t deficit, alloc_base, free_head, resting0;
  int32_t dresting;
  int32_t bb, ba;
  uint32_t active, hidx, gs;
  uint32_t mk_base, mk_cur;  // the slot's region of AggDev::mk (reserved by the walk) and its cursor
  uint32_t fr_base, fr_cur;  // the same for AggDev::fr
  uint32_t pad;
};
enum : uint32_t { AC_EV = 0, AC_SEG = 1, AC_MK = 2, AC_FR = 3, AC_N = 8 };
struct AggDev {
  AggSlot* slot;               // [S]
  AggEv* ev;                   // [ev_cap] event log (per-slot regions)
  uint32_t* evs;               // [ev_cap] log indices grouped by level (stable)
  AggEv* evq;                  // [ev_cap] the entries in that order (pad: the log index)
  unsigned long long* eva;     // [ev_cap] take: start of its interval in the level's maker space
  uint32_t* evf;               // [ev_cap] take: its first maker (AggDev::mk index)
  uint32_t* evn;               // [ev_cap] fills of the event (0 for rests)
  uint32_t* evx;               // [ev_cap] exclusive scan of evn over the slot's log
  AggSeg* seg;                 // [ev_cap]
  AggSegS* segs;               // [ev_cap]
  AggMk* mk;                   // [mk_cap]
  uint32_t* fr;                // [fr_cap] chunk ids: freed by levels, surpluses, allocations
  AggRec* rec;                 // [max_batch]
  uint32_t* ctr;               // [AC_N] pool tops (zeroed by k_seq_sweep)
  uint32_t ev_cap, mk_cap, fr_cap;
  uint32_t nslots;             // grouped launches: slot = symbol, nslots = S (0: k_hot_pick's hcount)
  uint32_t ladder_max;         // k_agg_walk: windows up to this many levels take the ladder walk
  uint32_t lw_occ;             // k_agg_walk: ladders deeper than this search the next level through an LDS
                               // occupancy bitmap (0: the 64-level total scan at every depth)
  uint32_t gw_cx;              // grouped launches: the walk that covers cancels (k_agg_gwalk_cx) and its resolve
  // grouped launches (register-window path, k_agg_gwalk): per symbol and batch of the group, [S][ME_GMAX + 1]
  uint32_t* gev;               // the symbol's first log index of batch g (g = ng: the log's end)
  uint32_t* gex;               // the fill offset (k_agg_fin's scan) at gev
  uint32_t* gbase;             // scratch position of the symbol's first fill of batch g
};
// Where the record of a log entry lives (k_agg_levels / k_agg_place read the seq of a rest there).
struct AggSrc {
  const uint32_t* perm;          // sort path: j = grouped position, its batch index perm[j] in seq[0]
  const uint64_t* seq[ME_GMAX];  // grouped launches (perm null): j = g << AGG_GSHIFT | batch index
};
constexpr uint32_t AGG_GSHIFT = 25;  // batch index bits of a grouped log entry (BK_MAX_BATCH)
constexpr uint32_t AGG_IMASK = (1u << AGG_GSHIFT) - 1u;

// Host side of a deep-window launch with hot symbols: k_match_hot (or the aggregate path) runs on `st`,
// forked from and joined back into the engine stream by two events (me_kernels.hip launch_match).
struct HotLaunch {
  hipStream_t st = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  bool agg = false;  // the aggregate path (me_agg.hip) instead of k_match_hot
  bool agg_reg = false;  // L <= 128: grouped launches through the aggregate path (me_agg.hip k_agg_gwalk)
  AggDev ag{};
  // grouped aggregate launches: the side jobs (bucketing of the next group, tapes of the one before) on
  // their own stream, forked before and joined after the group's walk / per-level launch / continuation
  hipStream_t sst = nullptr;
  hipEvent_t sfork = nullptr, sjoin = nullptr;
};

// Event counters kept on the device (BookDev::stats, me_stats_read).
// ST_RESTING: resting orders of every symbol (each wave adds its symbol's change when it writes the
// symbol state back); k_seq_sweep publishes it to the host for admission control (me_engine.cpp).
// ST_LAUNCH: the match launches enqueued before the current group (k_seq_sweep), for the continuation's
// hand-off publication.
// ST_FAR_GROW / ST_FAR_GC: far sides moved to a larger arena region / collection passes (me_far_stats).
// ST_CHUNK_GC: chunk-pool reclamations (k_seq_sweep, me_chunk_stats).
enum : uint32_t { ST_HANDOFFS = 0, ST_RESTING = 1, ST_LAUNCH = 2, ST_FAR_GROW = 3, ST_FAR_GC = 4, ST_CHUNK_GC = 5, ME_STATS = 8 };

struct BookDev {
  Level* levels;
  unsigned long long* occ;
  uint8_t* tend;          // [S][L] slots written in the level's tail chunk (valid when tail != NIL)
  SymState* sym;
  Chunk* chunks;          // [NC] FIFO chunk blocks
  uint32_t* loc;          // [ring_mask + 1] seq ring
  uint32_t* chunk_top;
  uint32_t* fcache;       // [S][64] free chunk ids parked between launches (register-window kernel)
  uint32_t* err;
  const uint32_t* gsym;  // [S] id written into me_fill.symbol
  unsigned long long* dbg;  // [S][8] phase cycles, diagnostic (-DME_STAMPS) builds only
  FarLevel* far;          // far arena: [2S][fcap] inline regions, then two halves of far_half entries
  FarDir* fdir;           // [S][2] each side's region of the arena (me_far.hpp)
  unsigned long long* far_ctl;  // [FC_N] half tops, active half, collection ticket
  unsigned long long far_half;  // entries per half (6 x max_resting + slack: the bound of me_far.hpp)
  unsigned long long far_gc_at; // a half's top above this at k_seq_sweep: collect (2 x max_resting)
  OldEnt* old;            // [old_mask + 1]
  SeqState* sq;           // [2]
  uint32_t* hcount;       // hand-offs of the current match launch (zeroed by k_seq_sweep)
  Handoff* hand;          // [S]
  unsigned long long* stats;  // [ME_STATS] event counters (me_stats_read)
  unsigned long long* pub;    // host-mapped [0] {launches << 32 | resting}, [1] {launches << 32 |
                              // hand-offs} (k_seq_sweep), or null
  unsigned long long ring_mask;
  unsigned long long old_mask;
  uint32_t fcap;          // inline far levels per (symbol, side) (me_config.far_levels)
  uint32_t sq_idx;       // state the match launches read (k_seq_sweep wrote it)
  uint32_t nchunks;
  uint32_t S;
  uint32_t L;
  uint32_t Lwords;
  uint32_t hot_min;       // deep windows: a symbol with at least this many records in a batch is matched
                          // by k_match_hot (me_kernels.hip) or the aggregate path (me_agg.hip) instead
                          // of k_match; 0 = never
  uint32_t* agg_ctr;      // AggDev::ctr (zeroed by k_seq_sweep with hcount), or null
  // Chunk pool (cp_id below): *chunk_top counts the allocations since the last reclamation; the v-th of
  // them is recl[v] while v < nrecl (a chunk the reclamation found free), then fresh + (v - nrecl).
  uint32_t* recl;         // [nchunks] free chunk ids found by the last reclamation (k_seq_sweep)
  uint32_t* cpool;        // [CP_N] {nrecl, fresh, found counter, ticket}
};

// ---- chunk pool ------------------------------------------------------------------------------------
// Chunks are drawn by one atomic add on *chunk_top (a block of consecutive allocation numbers); the
// number maps to a chunk id through the reclamation's list, then past it to never-used ids from `fresh`
// on. A symbol keeps the chunks its levels free (its free list, fcache row) until k_seq_sweep's
// reclamation — due when the high-water mark plus the group's bound could pass the pool — returns every
// free chunk of every symbol to the list: so chunks in use never exceed resting orders
// and the pool needs max_resting + the launch group's reservation slack, whichever symbols the
// liquidity moves between.
enum : uint32_t { CP_NRECL = 0, CP_FRESH = 1, CP_FOUND = 2, CP_TICKET = 3, CP_N = 4 };
struct CPool {
  uint32_t nrecl, fresh;
};
#ifdef __HIPCC__
__device__ __forceinline__ CPool cp_read(const uint32_t* cpool) {
  CPool p;
  p.nrecl = __builtin_amdgcn_readfirstlane(cpool[CP_NRECL]);
  p.fresh = __builtin_amdgcn_readfirstlane(cpool[CP_FRESH]);
  return p;
}
// allocation numbers [0, vcap) name distinct chunks (recl ids are < fresh, so nrecl <= fresh <= nchunks)
__device__ __forceinline__ uint32_t cp_vcap(const CPool& p, uint32_t nchunks) { return p.nrecl + (nchunks - p.fresh); }
__device__ __forceinline__ uint32_t cp_id(const uint32_t* recl, const CPool& p, uint32_t v) {
  return v < p.nrecl ? recl[v] : p.fresh + (v - p.nrecl);
}
// chunk ids below this have been handed out at some point (the scans of k_seq_sweep stop here)
__device__ __forceinline__ uint32_t cp_hw(const CPool& p, uint32_t top, uint32_t nchunks) {
  const uint32_t h = top > p.nrecl ? p.fresh + (top - p.nrecl) : p.fresh;
  return h < nchunks ? h : nchunks;
}
#endif

// Far levels of (symbol s, side k) (k = 0 bids below the window, 1 asks above it): device code, read
// between launches (the snapshot kernel); the matching kernels go through me_far.hpp's far_dir.
__device__ __forceinline__ FarLevel* far_of(const BookDev& bk, uint32_t s, uint32_t k) {
  return bk.far + bk.fdir[(size_t)s * 2u + k].off;
}
// Hash of a seq into the old-order table.
__host__ __device__ __forceinline__ unsigned long long old_hash(unsigned long long q) {
  q ^= q >> 33;
  q *= 0xff51afd7ed558ccdull;
  q ^= q >> 33;
  return q;
}

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
};

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
  uint32_t* fstart;
  const me_fill* scratch;
  me_fill* tape;
  unsigned long long* tape_count;
  // Host batches (me_submit_host): the tape buffer is the slot's, `cap` records long and SOFT — fills
  // past it are not copied (me_collect recovers them from scratch) and raise no error; the final
  // results go to hres, each record's scratch start to fstart, the error word to err_out.
  // Device batches: hres == nullptr, cap = the tape bound (exceeding it is ERR_SCRATCH_OOM).
  me_order_result* hres;
  uint32_t* err_out;
  unsigned long long cap;
  uint32_t tn;
  uint32_t pad;
};
struct AuxDev {
  uint32_t S;
  uint32_t nwg;  // workgroups that run side jobs (those of the first dispatch round)
  uint32_t nb;   // bucket jobs (batches of group J)
  uint32_t nt;   // tape jobs (batches of group J-2)
  uint32_t xseq; // k_side beside a walk: each XCD buckets its batches one after another (me_match_reg.hip)
  uint32_t rsv;
  unsigned long long* fills_acc;
  AuxBucket b[ME_GMAX];
  AuxTape t[ME_GMAX];
};

// A book snapshot request (me_snapshot.hip k_book_snapshot): one workgroup per (symbol, side).
struct SnapReq {
  const uint32_t* sym;       // [nsym] symbols
  uint32_t nsym;
  uint32_t depth;            // levels per side at most
  me_level* lv;              // [nsym][2][depth] level aggregates, best first
  uint32_t* nlv;             // [nsym][2] levels written
  me_book_entry* ord;        // [nsym][2][ocap] orders in priority order (nullptr: levels only)
  unsigned long long ocap;   // orders per (symbol, side) region
  unsigned long long* nord;  // [nsym][2] orders on those levels (exact, even past ocap)
  uint32_t* err;             // set on a corrupt chain
};

constexpr int BK_CAP = 128;          // records per bucket (two 64-record blocks)
constexpr int BK_KIND_SHIFT = 28;    // BkRec::ok: kind bits above the batch index
constexpr uint32_t BK_IDX_MASK = (1u << BK_KIND_SHIFT) - 1u;
constexpr uint32_t BK_MAX_BATCH = 1u << 25;  // sort key (index << 7 | bucket slot) fits 32 bits
constexpr int BK_CNT_STRIDE = 32;    // bcnt[b * stride]: one 128-B line per counter (atomics on one
                                     // line serialise: packed counters made k_bucket 6x slower)

}  // namespace me

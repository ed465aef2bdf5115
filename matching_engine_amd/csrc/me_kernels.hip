// me_kernels.hip — gfx950 kernels of the batched matching core.
//
// One batch (n records, ascending seq) goes through:
//   1. k_sort_hist / k_sort_colscan / k_sort_scatter
//                                    stable LSD counting sort of the records by symbol
//                                    (1 pass for <= 2047 symbols, 2 passes up to 4M): groups
//                                    every symbol's records contiguously, seq order kept.
//   2. k_match                       one wavefront per symbol walks its records in seq order
//                                    against the HBM-resident book (price-time priority), using
//                                    ballot + 64-lane prefix scans over levels and FIFO chunks;
//                                    fills go to a per-wave scratch run. (Windows of <= 128
//                                    levels use k_match_reg, me_match_reg.hip.)
//   3. k_tape_compact                exclusive scan of per-record fill counts (batch order) and
//                                    a coalesced copy scratch -> tape ordered (taker_seq, fill#).
//
// Matching semantics are pinned by oracle/oracle_book.cpp; there is no
// reference matcher (include/engine/model.hpp is empty in julien-mrty/Matching_Engine).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "me_far.hpp"
#include "me_layout.hpp"
#include "me_wave.hpp"

namespace me {


// ------------------------------------------------------------------ grouping sort
// One pass of a stable LSD counting sort of the batch by symbol id. digit(key) =
// (min(key, clamp) >> shift) & mask over nbins <= 2048 bins (the last pass uses only the bins that
// occur). Three launches, none of them a single-workgroup stage:
//   k_sort_hist     per-tile histograms (tile-major rows [tile][bin]);
//   k_sort_colscan  one lane per bin: exclusive scan down its column (all tile loads in flight at
//                   once) -> start of every (tile, bin) run within the bin, plus the bin total;
//   k_sort_scatter  every tile adds the exclusive scan of the bin totals (LDS) and scatters its
//                   records stably (ballot multisplit). The final pass also publishes the run
//                   table bin_start[0..nbins] (single pass: bins are symbols).
struct SortPass {
  uint32_t shift, mask, nbins, tile, ntiles, clamp;
};

__device__ __forceinline__ uint32_t sort_digit(uint32_t k, const SortPass& p) {
  if (k > p.clamp) k = p.clamp;
  return (k >> p.shift) & p.mask;
}

// Per-tile histograms, tile-major [tile][bin].
// The first pass also checks the API precondition the seq ring relies on (seqs ascending, seq_follows).
__global__ __launch_bounds__(256) void k_sort_hist(const uint32_t* __restrict__ keys_in, uint32_t n, SortPass p,
                                                   uint32_t* __restrict__ hist, uint32_t* zero_buf,
                                                   uint32_t zero_words, unsigned long long* scratch_top,
                                                   const uint64_t* __restrict__ seq,
                                                   const uint8_t* __restrict__ kind, uint32_t* err) {
  __shared__ uint32_t h[1u << MAX_DIGIT_BITS];
  for (uint32_t b = threadIdx.x; b < p.nbins; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const uint32_t t0 = blockIdx.x * p.tile;
  const uint32_t t1 = min(n, t0 + p.tile);
  bool order_ok = true;
  for (uint32_t i = t0 + threadIdx.x; i < t1; i += blockDim.x) {
    atomicAdd(&h[sort_digit(keys_in[i], p)], 1u);
    if (seq && i > 0) order_ok &= seq_follows(seq[i - 1], seq[i], kind[i]);
  }
  if (!order_ok) atomicOr(err, ERR_SEQ_ORDER);
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < p.nbins; b += blockDim.x) hist[(size_t)blockIdx.x * p.nbins + b] = h[b];
  // Per-batch resets folded into the first kernel of the batch.
  if (zero_buf) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < zero_words; i += gridDim.x * blockDim.x)
      zero_buf[i] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) *scratch_top = 0ull;
  }
}

// In place: hist[t][b] <- sum of hist[t'][b] over t' < t; tot[b] <- column total. One lane per bin;
// the column's loads are all issued before the first add (ntiles <= MAX_SORT_TILES).
__global__ __launch_bounds__(64) void k_sort_colscan(uint32_t* __restrict__ hist, uint32_t* __restrict__ tot,
                                                     uint32_t nbins, uint32_t ntiles) {
  const uint32_t b = blockIdx.x * 64 + threadIdx.x;
  if (b >= nbins) return;
  uint32_t run = 0;
  for (uint32_t t0 = 0; t0 < ntiles; t0 += 32) {
    uint32_t v[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) v[u] = hist[(size_t)min(t0 + u, ntiles - 1) * nbins + b];
#pragma unroll
    for (int u = 0; u < 32; ++u)
      if (t0 + u < ntiles) {
        hist[(size_t)(t0 + u) * nbins + b] = run;
        run += v[u];
      }
  }
  tot[b] = run;
}

// Block-wide exclusive scan of LDS array a[0..cnt) (cnt <= 2048) with 256 threads; returns total.
__device__ uint32_t block_excl_scan_lds(uint32_t* a, uint32_t cnt, uint32_t* wsum) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t per = (cnt + 255) / 256;
  uint32_t b0 = tid * per, local = 0;
  for (uint32_t j = 0; j < per; ++j)
    if (b0 + j < cnt) local += a[b0 + j];
  uint32_t x = local;
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t t = __shfl_up(x, d, 64);
    if (lane >= d) x += t;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t wpre = 0, total = 0;
  for (int k = 0; k < 4; ++k) {
    if (k < w) wpre += wsum[k];
    total += wsum[k];
  }
  uint32_t run = wpre + x - local;
  for (uint32_t j = 0; j < per; ++j)
    if (b0 + j < cnt) {
      uint32_t v = a[b0 + j];
      a[b0 + j] = run;
      run += v;
    }
  __syncthreads();
  return total;
}

// Stable scatter of one tile: dest = start of this tile's run of its digit + rank among equal
// digits earlier in the tile. Each wave owns a quarter of the tile and ranks 64 records at a time
// with a ballot multisplit (one ballot per digit bit).
__global__ __launch_bounds__(256) void k_sort_scatter(const uint32_t* __restrict__ keys_in,
                                                      const uint32_t* __restrict__ idx_in, uint32_t n, SortPass p,
                                                      uint32_t dbits, const uint32_t* __restrict__ colpre,
                                                      const uint32_t* __restrict__ tot,
                                                      uint32_t* __restrict__ keys_out,
                                                      uint32_t* __restrict__ idx_out, uint32_t* bin_start) {
  __shared__ uint32_t base[1u << MAX_DIGIT_BITS];
  __shared__ uint32_t wcnt[4][1u << MAX_DIGIT_BITS];
  __shared__ uint32_t wsum[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t tile = blockIdx.x;
  for (uint32_t b = tid; b < p.nbins; b += 256) {
    base[b] = tot[b];
    wcnt[0][b] = wcnt[1][b] = wcnt[2][b] = wcnt[3][b] = 0;
  }
  __syncthreads();
  block_excl_scan_lds(base, p.nbins, wsum);  // global start of every bin
  const uint32_t t0 = tile * p.tile, t1 = min(n, t0 + p.tile);
  const uint32_t q = p.tile / 4;
  const uint32_t w0 = min(t1, t0 + w * q), w1 = min(t1, w0 + q);
  for (uint32_t i = w0 + lane; i < w1; i += 64) atomicAdd(&wcnt[w][sort_digit(keys_in[i], p)], 1u);
  __syncthreads();
  if (tile == 0 && bin_start) {
    for (uint32_t b = tid; b < p.nbins; b += 256) bin_start[b] = base[b];
    if (tid == 0) bin_start[p.nbins] = n;
  }
  // this tile's run start of every bin: + records of the bin in earlier tiles (k_sort_colscan)
  for (uint32_t b = tid; b < p.nbins; b += 256) base[b] += colpre[(size_t)tile * p.nbins + b];
  __syncthreads();
  for (uint32_t b = tid; b < p.nbins; b += 256) {  // per-bin start of each wave's quarter
    uint32_t run = base[b];
    for (int k = 0; k < 4; ++k) {
      const uint32_t c = wcnt[k][b];
      wcnt[k][b] = run;
      run += c;
    }
  }
  __syncthreads();
  for (uint32_t c0 = w0; c0 < w1; c0 += 64) {
    const uint32_t i = c0 + lane;
    const bool v = i < w1;
    const uint32_t ic = v ? i : w0;  // clamp: never branch around a load
    uint32_t k = keys_in[ic];
    if (k > p.clamp) k = p.clamp;
    const uint32_t val = idx_in ? idx_in[ic] : ic;
    const uint32_t d = (k >> p.shift) & p.mask;
    unsigned long long peers = __ballot(v);
    for (uint32_t bit = 0; bit < dbits; ++bit) {
      const unsigned long long bb = __ballot((d >> bit) & 1u);
      peers &= ((d >> bit) & 1u) ? bb : ~bb;
    }
    const uint32_t rank = (uint32_t)__popcll(peers & lanemask_lt());
    const uint32_t cnt = (uint32_t)__popcll(peers);
    const uint32_t start = wcnt[w][d];
    if (v) {
      keys_out[start + rank] = k;
      idx_out[start + rank] = val;
    }
    __builtin_amdgcn_wave_barrier();
    if (v && rank == 0) wcnt[w][d] = start + cnt;
    __builtin_amdgcn_wave_barrier();
  }
}

// ------------------------------------------------------------------ matching
// Deep windows (L > 128): one wavefront per symbol walks its records in seq order against the
// ladder (levels / occupancy / tail fills in LDS for L <= LDS_MAX_LEVELS, else in HBM) and the far
// levels outside the window (me_far.hpp).
//
// Head-chunk cache (LDS, ladders in LDS only): entry (lvl & cmask) holds the FIFO head chunk of one
// level — its 16 slot quantities/seqs and its next pointer — so walks and appends on top-of-book
// levels stay on chip. The HBM copy is stale while an entry is dirty; write-back on eviction, on free
// (freed chunks must hold qty 0 in HBM), before a re-centre and at kernel end.
constexpr int CK_MEM = 64;  // entries (direct-mapped by level)
constexpr uint32_t HOT_MAX_WORDS = 1024;  // k_match_hot keeps occupancy in LDS: windows up to 65,536 levels
struct alignas(16) CacheEntry {
  uint32_t cid;    // cached chunk id, NIL = empty
  uint32_t dirty;  // slots differ from HBM
  uint32_t next;   // chdr[cid].next (kept in sync by set_next)
  uint32_t pad;
  int qty[ME_C];
  unsigned long long seq[ME_C];
};

// Where a wave keeps its symbol's window: levels / occupancy / tail-fill arrays behind pointers.
struct LadderMem {
  Level* lv;
  unsigned long long* occ;
  uint8_t* tend;
  uint32_t L, Lwords;
  // words the first step of an occupancy scan reads past the start word: the HBM ladder (k_match<LAD_HBM>,
  // config 4's cold symbols) reads one 64-B line first — a sparse book's next level is usually within
  // 512 levels — before 512-B steps
  int span0 = 64;
  bool occ_reads = false;  // window scans read only the occupied levels (k_match<LAD_HBM>)

  __device__ __forceinline__ Level get(int l) const {
    Level x = lv[l];
    x.total = rli64(x.total, 0);
    x.head = rl32(x.head, 0);
    x.tail = rl32(x.tail, 0);
    return x;
  }
  __device__ __forceinline__ void set(int l, const Level& x) {
    if (lane_id() == 0) lv[l] = x;
  }
  __device__ __forceinline__ uint32_t head(int l) const { return rl32(lv[l].head, 0); }
  // per-lane level read (the sweep's 64-level windows); lanes with !valid read nothing
  __device__ __forceinline__ Level lane_get(int l, bool valid) const {
    Level x{0, NIL, NIL};
    if (valid) x = lv[l];
    return x;
  }
  __device__ __forceinline__ uint32_t get_te(int l) const { return rl32((uint32_t)tend[l], 0); }
  __device__ __forceinline__ void set_te(int l, uint32_t v) {
    if (lane_id() == 0) tend[l] = (uint8_t)v;
  }
  __device__ __forceinline__ void occ_set(int l) {
    if (lane_id() == 0) occ[l >> 6] |= (1ull << (l & 63));
  }
  __device__ __forceinline__ void occ_clear(int l) {
    if (lane_id() == 0) occ[l >> 6] &= ~(1ull << (l & 63));
  }
  // Smallest occupied level >= x, or L.
  __device__ int next_occ(int x) const {
    const int Li = (int)L;
    if (x >= Li) return Li;
    if (x < 0) x = 0;
    wave_mem_order();
    int w = x >> 6;
    unsigned long long word = occ[w] & (~0ull << (x & 63));
    if (word) return (w << 6) + __builtin_ctzll(word);
    const int lane = lane_id();
    const int nw = (int)Lwords;
    for (int b = w + 1, span = span0; b < nw; b += span, span = 64) {
      int idx = b + lane;
      unsigned long long v = lane < span && idx < nw ? occ[idx] : 0ull;
      unsigned long long m = __ballot(v != 0ull);
      if (m) {
        int t = __builtin_ctzll(m);
        unsigned long long wv = rl64(v, t);
        return ((b + t) << 6) + __builtin_ctzll(wv);
      }
    }
    return Li;
  }
  // Largest occupied level <= x, or -1.
  __device__ int prev_occ(int x) const {
    if (x < 0) return -1;
    if (x >= (int)L) x = (int)L - 1;
    wave_mem_order();
    int w = x >> 6;
    int r = x & 63;
    unsigned long long keep = (r == 63) ? ~0ull : ((1ull << (r + 1)) - 1ull);
    unsigned long long word = occ[w] & keep;
    if (word) return (w << 6) + 63 - __builtin_clzll(word);
    const int lane = lane_id();
    for (int t0 = w - 1, span = span0; t0 >= 0; t0 -= span, span = 64) {
      int idx = t0 - lane;
      unsigned long long v = lane < span && idx >= 0 ? occ[idx] : 0ull;
      unsigned long long m = __ballot(v != 0ull);
      if (m) {
        int t = __builtin_ctzll(m);
        unsigned long long wv = rl64(v, t);
        return ((t0 - t) << 6) + 63 - __builtin_clzll(wv);
      }
    }
    return -1;
  }
};

struct WaveCtx;
__device__ __forceinline__ uint32_t alloc_chunk(WaveCtx& c);
__device__ __forceinline__ void free_chunk(WaveCtx& c, uint32_t ch);

__device__ __forceinline__ void set_err(const BookDev& bk, uint32_t bits) {
  if (lane_id() == 0) atomicOr(bk.err, bits);
}

struct WaveCtx {
  BookDev bk;
  LadderMem lad;
  CacheEntry* cache;         // head-chunk cache in LDS, or nullptr (HBM ladder)
  uint32_t cmask;            // cache entry of level l = l & cmask
  uint32_t s;                // local symbol
  uint32_t gs;               // symbol id written in fills
  long long base;
  int bb, ba;                // best bid / best ask level of the window
  uint32_t free_head;        // chunk free list of this symbol ...
  uint32_t free_next;        // ... and chdr[free_head].next, loaded ahead of the pop that needs it
  uint32_t bump_ids;         // VGPR: chunk ids reserved from the global pool (lane i: entry i) ...
  uint32_t bump_cur, bump_end;  // ... entries [bump_cur, bump_end) are still unused
  uint32_t recs_left;        // records of this wave not processed yet (>= chunks it can still need)
  int resting_delta;
  unsigned long long wptr;   // next scratch slot of this wave
  me_fill* scratch;
  uint32_t nfar0, nfar1;     // far-level counts (me_far.hpp)
  unsigned long long horizon;  // seq-ring horizon of this launch
  uint32_t epoch;            // old-order table epoch of this launch
  uint32_t resting0;         // the symbol's resting orders when the wave started
#ifdef ME_STAMPS
  unsigned long long st[PH_N];
  unsigned long long st_t;
#endif
  // far-level interface (me_far.hpp)
  __device__ __forceinline__ gptr<Chunk> fchunks() const { return (gptr<Chunk>)bk.chunks; }
  __device__ __forceinline__ uint32_t fnchunks() const { return bk.nchunks; }
  __device__ __forceinline__ uint32_t fsym() const { return s; }
  __device__ __forceinline__ uint32_t fgsym() const { return gs; }
  __device__ __forceinline__ FarDir* fdirp(uint32_t k) const { return bk.fdir + (size_t)s * 2u + k; }
  __device__ __forceinline__ FarLevel* farena() const { return bk.far; }
  __device__ __forceinline__ unsigned long long* fctl() const { return bk.far_ctl; }
  __device__ __forceinline__ unsigned long long* fstats() const { return bk.stats; }
  __device__ __forceinline__ uint32_t fcap0() const { return bk.fcap; }
  __device__ __forceinline__ unsigned long long finline() const { return 2ull * bk.S * bk.fcap; }
  __device__ __forceinline__ unsigned long long fhalf() const { return bk.far_half; }
  __device__ __forceinline__ gptr<FarLevel> farr(uint32_t k) const { return far_arr(*this, k); }
  __device__ __forceinline__ uint32_t fcount(uint32_t k) const { return k ? nfar1 : nfar0; }
  __device__ __forceinline__ void fset_count(uint32_t k, uint32_t n) {
    if (k)
      nfar1 = n;
    else
      nfar0 = n;
  }
  __device__ __forceinline__ void femit(bool fe, unsigned long long fm, const me_fill& F) {
    if (fe) scratch[wptr + (unsigned long long)__popcll(fm & lanemask_lt())] = F;
    wptr += (unsigned long long)__popcll(fm);
  }
  __device__ __forceinline__ void fresting(int d) { resting_delta += d; }
  __device__ __forceinline__ void ferr(uint32_t bits) { set_err(bk, bits); }
  __device__ __forceinline__ void floc(unsigned long long seq, uint32_t g) {
    if (lane_id() == 0) bk.loc[seq & bk.ring_mask] = g;
  }
  __device__ __forceinline__ uint32_t falloc() { return alloc_chunk(*this); }
  __device__ __forceinline__ void ffree(uint32_t ch) { free_chunk(*this, ch); }
};

// ---- head-chunk cache -------------------------------------------------------------------
__device__ __forceinline__ CacheEntry* centry(const WaveCtx& c, int lvl) { return c.cache + ((uint32_t)lvl & c.cmask); }

__device__ __forceinline__ bool cache_holds(const WaveCtx& c, int lvl, uint32_t ch) {
  return c.cache && rl32(centry(c, lvl)->cid, 0) == ch;
}

__device__ __forceinline__ void cache_mark_dirty(WaveCtx& c, int lvl) {
  if (lane_id() == 0) centry(c, lvl)->dirty = 1;
}

// Write entry E back to HBM if dirty.
__device__ __forceinline__ void cache_writeback(const WaveCtx& c, CacheEntry* E) {
  const uint32_t cid = rl32(E->cid, 0);
  if (cid == NIL || !rl32(E->dirty, 0)) return;
  const int lane = lane_id();
  if (lane < ME_C) {
    const size_t g = (size_t)cid * ME_C + lane;
    cq_at(c.bk.chunks, g) = E->qty[lane];
    cs_at(c.bk.chunks, g) = E->seq[lane];
  }
}

__device__ __forceinline__ void cache_set_state(WaveCtx& c, CacheEntry* E, uint32_t ch, bool dirty) {
  if (lane_id() == 0) {
    E->cid = ch;
    E->dirty = dirty ? 1u : 0u;
  }
}

// Make `ch` (the head chunk of level lvl) the cached chunk of its entry; returns the entry.
__device__ __forceinline__ CacheEntry* cache_get(WaveCtx& c, int lvl, uint32_t ch) {
  CacheEntry* E = centry(c, lvl);
  const uint32_t cur = rl32(E->cid, 0);
  if (cur == ch) return E;
  if (cur != NIL) COUNT(c, CT_EVICT);
  cache_writeback(c, E);
  COUNT(c, CT_MISS);
  const int lane = lane_id();
  const bool act = lane < ME_C;
  const size_t g = (size_t)ch * ME_C + (act ? lane : 0);
  const int q = act ? cq_at(c.bk.chunks, g) : 0;
  const unsigned long long sq = act ? cs_at(c.bk.chunks, g) : 0ull;
  const uint32_t nx = c.bk.chunks[ch].hdr.next;
  if (act) {
    E->qty[lane] = q;
    E->seq[lane] = sq;
  }
  if (lane == 0) E->next = nx;
  cache_set_state(c, E, ch, false);
  return E;
}

// A brand-new (all-empty) chunk becomes the head of an empty level: install it without a load.
__device__ __forceinline__ void cache_install_new(WaveCtx& c, int lvl, uint32_t ch) {
  CacheEntry* E = centry(c, lvl);
  cache_writeback(c, E);
  const int lane = lane_id();
  if (lane < ME_C) {
    E->qty[lane] = 0;
    E->seq[lane] = 0ull;
  }
  if (lane == 0) E->next = NIL;
  cache_set_state(c, E, ch, true);
}

// The cached chunk ch of lvl is being freed or unlinked: HBM must hold its final (all-zero)
// quantities before the chunk is reused.
__device__ __forceinline__ void cache_drop(WaveCtx& c, int lvl, uint32_t ch) {
  if (!c.cache) return;
  CacheEntry* E = centry(c, lvl);
  if (rl32(E->cid, 0) != ch) return;
  cache_writeback(c, E);
  if (lane_id() == 0) E->cid = NIL;
}

// chdr[ch].next = v, mirrored into the cache entry of lvl when it holds ch.
__device__ __forceinline__ void set_next(WaveCtx& c, int lvl, uint32_t ch, uint32_t v) {
  const bool mirror = cache_holds(c, lvl, ch);
  if (lane_id() == 0) {
    c.bk.chunks[ch].hdr.next = v;
    if (mirror) centry(c, lvl)->next = v;
  }
}

// Dirty cached head chunks back to HBM: lane = (entry, slot) pairs, 4 entries per pass.
__device__ __forceinline__ void cache_flush_all(WaveCtx& c, uint32_t entries) {
  const int lane = lane_id();
  wave_mem_order();
  for (uint32_t e0 = 0; e0 < entries; e0 += 64 / ME_C) {
    const uint32_t e = e0 + lane / ME_C, sl = lane % ME_C;
    const CacheEntry* E = c.cache + e;
    const uint32_t cid = E->cid;
    if (cid != NIL && E->dirty) {
      cq_at(c.bk.chunks, (size_t)cid * ME_C + sl) = E->qty[sl];
      cs_at(c.bk.chunks, (size_t)cid * ME_C + sl) = E->seq[sl];
    }
  }
}

// ---- chunk allocation -------------------------------------------------------------------
// Issue the load of chdr[free_head].next without waiting for it: the value stays in a VGPR and is
// only read (readlane -> s_waitcnt) by the next pop, usually many records later.
__device__ __forceinline__ void prefetch_free_next(WaveCtx& c) {
  const bool ok = c.free_head < c.bk.nchunks;
  const uint32_t v = c.bk.chunks[ok ? c.free_head : 0].hdr.next;
  c.free_next = ok ? v : NIL;
}

// Free-list push: the popped-next is known without a load.
__device__ __forceinline__ void free_chunk(WaveCtx& c, uint32_t ch) {
  if (lane_id() == 0) c.bk.chunks[ch].hdr.next = c.free_head;
  c.free_next = c.free_head;
  c.free_head = ch;
}

__device__ __forceinline__ uint32_t alloc_chunk(WaveCtx& c) {
  if (c.free_head != NIL) {
    const uint32_t ch = c.free_head;
    if (ch >= c.bk.nchunks) {
      set_err(c.bk, ERR_INCONSISTENT);
      return NIL;
    }
    c.free_head = rl32(c.free_next, 0);
    prefetch_free_next(c);  // consumed by the next pop, usually much later
    return ch;
  }
  if (c.bump_cur >= c.bump_end) {
    // each record needs at most one new chunk: never reserve more than the records left
    const uint32_t BLK = min(16u, max(c.recs_left, 1u));
    uint32_t got = 0;
    if (lane_id() == 0) got = atomicAdd(c.bk.chunk_top, BLK);
    got = rl32(got, 0);
    const CPool p = cp_read(c.bk.cpool);
    const uint32_t vcap = cp_vcap(p, c.bk.nchunks);
    if (got >= vcap) {
      set_err(c.bk, ERR_CHUNK_OOM);
      return NIL;
    }
    const uint32_t nb = min(BLK, vcap - got);
    const uint32_t l = (uint32_t)lane_id();
    c.bump_ids = l < nb ? cp_id(c.bk.recl, p, got + l) : NIL;
    // the chunks belong to this symbol until a reclamation finds them free (unused ones join its free list)
    if (l < nb) c.bk.chunks[c.bump_ids].owner = c.s;
    c.bump_cur = 0;
    c.bump_end = nb;
  }
  return rl32(c.bump_ids, (int)c.bump_cur++);
}

// Append one fill per lane where e holds, in lane order, to the wave's scratch run.
__device__ __forceinline__ void emit_fills(WaveCtx& c, bool e, unsigned long long taker, unsigned long long maker,
                                           long long price, int qty) {
  unsigned long long m = __ballot(e);
  if (e) {
    unsigned long long pos = c.wptr + (unsigned long long)__popcll(m & lanemask_lt());
    me_fill f;
    f.taker_seq = taker;
    f.maker_seq = maker;
    f.price_q4 = price;
    f.qty = qty;
    f.symbol = c.gs;
    c.scratch[pos] = f;
  }
  c.wptr += (unsigned long long)__popcll(m);
}

// Consume `take` (> 0, <= level total) from the FIFO of window level `lvl`, oldest first. A slot is
// live iff its qty > 0 (consumed, cancelled and unwritten slots hold 0). A chunk's 16 slots are
// ranked with one wave prefix scan; with the cache they come from LDS, otherwise one HBM round
// trip loads header and slots together. Exhausted chunks go back to the free list. Returns the
// new head chunk (NIL: level emptied).
__device__ __forceinline__ uint32_t walk_level(WaveCtx& c, int lvl, long long take, uint32_t head, uint32_t tail,
                                               unsigned long long taker) {
  const int lane = lane_id();
  const BookDev& bk = c.bk;
  const long long price = c.base + lvl;
  const bool act = lane < ME_C;
  long long need = take;
  uint32_t ch = head;
  COUNT(c, CT_WALK);
  while (need > 0) {
    if (ch >= bk.nchunks) {  // NIL or corrupt: never index with it
      set_err(bk, ERR_INCONSISTENT);
      return NIL;
    }
    CacheEntry* E = nullptr;
    int qv;
    unsigned long long sv;
    uint32_t nxt_v;
    const size_t g = (size_t)ch * ME_C + (act ? lane : 0);
    STAMP_ADD(c, PH_WALK);
    if (c.cache) {
      E = cache_get(c, lvl, ch);
      STAMP_ADD(c, WK_GET);
      qv = act ? E->qty[lane] : 0;
      sv = act ? E->seq[lane] : 0ull;
      nxt_v = E->next;
    } else {
      nxt_v = bk.chunks[ch].hdr.next;  // issue every load of the chunk before the first use
      qv = act ? cq_at(bk.chunks, g) : 0;
      sv = act ? cs_at(bk.chunks, g) : 0ull;
    }
    const long long inc = wave_incl_scan((long long)qv);
    const long long ex = inc - qv;
    long long f = need - ex;
    if (f < 0) f = 0;
    if (f > qv) f = qv;
    const bool fe = f > 0;
    STAMP_ADD(c, WK_SCAN);
    emit_fills(c, fe, taker, sv, price, (int)f);
    if (E) {
      if (fe) E->qty[lane] = qv - (int)f;
      cache_mark_dirty(c, lvl);
    } else if (fe) {
      cq_at(bk.chunks, g) = qv - (int)f;
    }
    c.resting_delta -= __popcll(__ballot(fe && f == qv));  // makers filled completely leave the book
    const long long live = rli64(inc, 63);
    need -= (need < live ? need : live);
    const unsigned long long alive = __ballot((qv - f) > 0);
    STAMP_ADD(c, WK_EMIT);
    if (!alive) {  // every slot of the chunk is consumed
      cache_drop(c, lvl, ch);
      free_chunk(c, ch);
      if (ch == tail) {
        if (need > 0) set_err(bk, ERR_INCONSISTENT);
        STAMP_ADD(c, WK_TAIL);
        return NIL;
      }
      ch = rl32(nxt_v, 0);
      STAMP_ADD(c, WK_TAIL);
    } else if (need > 0) {  // impossible: a live slot remains only once the take is met
      set_err(bk, ERR_INCONSISTENT);
      return ch;
    }
  }
  if (ch != head && ch < bk.nchunks && lane == 0) bk.chunks[ch].hdr.prev = NIL;  // new FIFO head
  return ch;
}

// Write back level lvl after `take` was consumed from it.
__device__ __forceinline__ void level_after_take(WaveCtx& c, int lvl, long long ntot, uint32_t nh, uint32_t tail) {
  Level o;
  o.total = ntot;
  o.head = ntot ? nh : NIL;
  o.tail = ntot ? tail : NIL;
  c.lad.set(lvl, o);
  if (ntot == 0) c.lad.occ_clear(lvl);
}

// Consume `take` at level lvl whose header is (tot, head, tail); returns true if it emptied.
__device__ __forceinline__ bool take_level(WaveCtx& c, int lvl, long long tot, long long take, uint32_t head,
                                           uint32_t tail, unsigned long long taker) {
  STAMP_ADD(c, PH_SWEEP);
  const uint32_t nh = walk_level(c, lvl, take, head, tail, taker);
  STAMP_ADD(c, PH_WALK);
  level_after_take(c, lvl, tot - take, nh, tail);
  STAMP_ADD(c, PH_SW_UPDATE);
  return tot == take;
}

// Sweep the opposite side of the window for a taker. dir = +1 (BUY: asks upward from best_ask) or
// -1 (SELL: bids downward from best_bid); lim = last window level the taker may trade at (-1 / L:
// none). 64-level windows: lanes load consecutive levels, an inclusive scan of their totals says how
// far the taker reaches. Returns qty filled.
__device__ __forceinline__ long long sweep(WaveCtx& c, int dir, int lim, long long want, unsigned long long taker) {
  const int lane = lane_id();
  const int L = (int)c.bk.L;
  long long rem = want;
  int cur = (dir > 0) ? c.ba : c.bb;
  bool emptied = false;
  if (dir > 0 ? (cur > lim || cur >= L) : (cur < lim || cur < 0)) return 0;  // does not cross
  // fast path: the best level alone fills the taker (no scan)
  {
    const Level B = c.lad.get(cur);
    if (B.total >= want) {
      COUNT(c, CT_FAST);
      if (take_level(c, cur, B.total, want, B.head, B.tail, taker)) {
        if (dir > 0)
          c.ba = c.lad.next_occ(cur + 1);
        else
          c.bb = c.lad.prev_occ(cur - 1);
        STAMP_ADD(c, PH_SW_BEST);
      }
      return want;
    }
  }
  while (rem > 0) {
    if (dir > 0 ? (cur > lim || cur >= L) : (cur < lim || cur < 0)) break;
    const int lv = cur + dir * lane;
    bool valid = (dir > 0) ? (lv <= lim && lv < L) : (lv >= lim && lv >= 0);
    // the HBM ladder reads only the occupied levels of the 64 (one 8-B word load per lane, the same one or
    // two words for the whole wave): an empty level holds total 0 and would add nothing to the scan
    if (c.lad.occ_reads && valid) valid = (c.lad.occ[lv >> 6] >> (lv & 63)) & 1ull;
    const Level W = c.lad.lane_get(lv, valid);
    const long long tot = W.total;
    const long long inc = wave_incl_scan(tot);
    const long long ex = inc - tot;
    const long long rem0 = rem;
    unsigned long long tm = __ballot(valid && tot > 0 && ex < rem0);
    STAMP_ADD(c, PH_SW_WINDOW);
    while (tm) {
      const int t = __builtin_ctzll(tm);
      tm &= tm - 1;
      const int lvl = cur + dir * t;
      const long long ltot = rli64(tot, t);
      const long long lex = rli64(ex, t);
      long long take = rem0 - lex;
      if (take > ltot) take = ltot;
      emptied |= take_level(c, lvl, ltot, take, rl32(W.head, t), rl32(W.tail, t), taker);
      rem -= take;
    }
    if (rem == 0) break;
    // every valid level of this window is now empty; jump to the next occupied one
    const int nxt = cur + dir * 64;
    if (dir > 0) {
      if (nxt > lim) break;
      cur = c.lad.next_occ(nxt);
    } else {
      if (nxt < lim) break;
      cur = c.lad.prev_occ(nxt);
    }
    STAMP_ADD(c, PH_SW_JUMP);
  }
  if (emptied) {
    if (dir > 0)
      c.ba = c.lad.next_occ(c.ba);
    else
      c.bb = c.lad.prev_occ(c.bb);
    STAMP_ADD(c, PH_SW_BEST);
  }
  return want - rem;
}

// Append a resting order at the tail of window level lvl's FIFO. The tail fill count lives beside
// the level, so the common case issues no HBM load; a tail that is the cached head is written on chip.
__device__ __forceinline__ bool rest_order(WaveCtx& c, int lvl, unsigned long long seq, int qty, bool buy) {
  const int lane = lane_id();
  const BookDev& bk = c.bk;
  Level L = c.lad.get(lvl);
  const uint32_t te = c.lad.get_te(lvl);
  uint32_t ch, slot;
  bool in_cache = false;  // does the slot live in the cached head chunk?
  if (L.tail != NIL && L.tail >= bk.nchunks) {
    set_err(bk, ERR_INCONSISTENT);
    return false;
  }
  if (L.tail == NIL || te >= (uint32_t)ME_C) {
    ch = alloc_chunk(c);
    if (ch == NIL) return false;
    slot = 0;
    if (lane == 0) {
      ChunkHdr h;
      h.next = NIL;
      h.prev = L.tail;
      h.price = c.base + lvl;
      bk.chunks[ch].hdr = h;
    }
    if (L.tail != NIL) set_next(c, lvl, L.tail, ch);
    if (L.tail == NIL) {
      L.head = ch;
      if (c.cache) {
        cache_install_new(c, lvl, ch);
        in_cache = true;
      }
    }
    L.tail = ch;
  } else {
    ch = L.tail;
    slot = te;
    in_cache = ch == L.head && cache_holds(c, lvl, ch);  // the ladder still names the current head
  }
  const size_t g = (size_t)ch * ME_C + slot;
  const bool was_empty = (L.total == 0);
  L.total += qty;
  if (in_cache) cache_mark_dirty(c, lvl);
  if (lane == 0) {
    if (in_cache) {
      CacheEntry* E = centry(c, lvl);
      E->seq[slot] = seq;
      E->qty[slot] = qty;
    } else {
      cs_at(bk.chunks, g) = seq;
      cq_at(bk.chunks, g) = qty;
    }
  }
  c.floc(seq, (uint32_t)g);
  c.lad.set(lvl, L);
  c.lad.set_te(lvl, slot + 1);
  if (was_empty) c.lad.occ_set(lvl);
  if (buy) {
    if (lvl > c.bb) c.bb = lvl;
  } else {
    if (lvl < c.ba) c.ba = lvl;
  }
  c.resting_delta += 1;
  return true;
}

// Cancel the window order in slot `slot` of chunk ch (level lvl, quantity q, the chunk's live
// quantities qv, FIFO links nxt / prv). A chunk left without live orders is unlinked from its FIFO
// at once (so chunks in use never exceed resting orders); a level left empty returns its whole FIFO
// to the free list.
__device__ __forceinline__ void cancel_window(WaveCtx& c, int lvl, uint32_t ch, uint32_t slot, int q, int qv,
                                              uint32_t nxt, uint32_t prv, CacheEntry* E) {
  const BookDev& bk = c.bk;
  const int lane = lane_id();
  const uint32_t live_after = (uint32_t)__popcll(__ballot(qv > 0)) - 1;
  Level L = c.lad.get(lvl);
  L.total -= q;
  if (L.tail >= bk.nchunks || L.head >= bk.nchunks) {
    set_err(bk, ERR_INCONSISTENT);
    return;
  }
  if (E) cache_mark_dirty(c, lvl);
  if (lane == 0) {
    if (E)
      E->qty[slot] = 0;
    else
      cq_at(bk.chunks, (size_t)ch * ME_C + slot) = 0;
  }
  wave_mem_order();
  if (L.total == 0) {
    // splice the whole (now dead) FIFO onto the free list
    cache_drop(c, lvl, L.head);
    if (lane == 0) bk.chunks[L.tail].hdr.next = c.free_head;
    c.free_next = (L.head == L.tail) ? c.free_head : NIL;
    c.free_head = L.head;
    if (L.head != L.tail) prefetch_free_next(c);
    L.head = NIL;
    L.tail = NIL;
    c.lad.set(lvl, L);
    c.lad.occ_clear(lvl);
    if (lvl == c.bb) c.bb = c.lad.prev_occ(lvl);
    if (lvl == c.ba) c.ba = c.lad.next_occ(lvl);
  } else if (live_after == 0) {
    // unlink the dead chunk (the level keeps live orders elsewhere, so ch is not both ends)
    uint32_t nh = L.head, nt = L.tail;
    if (ch == L.head) {
      nh = nxt;
      if (lane == 0) bk.chunks[nxt].hdr.prev = NIL;
    } else if (ch == L.tail) {
      nt = prv;
      set_next(c, lvl, prv, NIL);
      c.lad.set_te(lvl, ME_C);  // a non-tail chunk is always full
    } else {
      set_next(c, lvl, prv, nxt);
      if (lane == 0) bk.chunks[nxt].hdr.prev = prv;
    }
    if (ch == L.head) cache_drop(c, lvl, ch);  // the cache only ever holds a level's head
    L.head = nh;
    L.tail = nt;
    c.lad.set(lvl, L);
    free_chunk(c, ch);
  } else {
    c.lad.set(lvl, L);
  }
  c.resting_delta -= 1;
}

// Cancel the live resting order `tgt` of this symbol. Returns the removed qty, 0 if not live. The
// seq ring names its slot unless a later seq overwrote the entry, in which case an order older than
// the horizon is in the old-order table; every candidate slot is verified (owner, seq, qty > 0).
__device__ __forceinline__ int cancel_order(WaveCtx& c, unsigned long long tgt) {
  const BookDev& bk = c.bk;
  const int lane = lane_id();
  const bool act = lane < ME_C;
  if (tgt == 0ull) return 0;
  wave_mem_order();
  uint32_t g = rl32(bk.loc[tgt & bk.ring_mask], 0);
  for (int pass = 0;; ++pass) {
    if (g != NIL && g / ME_C < bk.nchunks) {
      const uint32_t ch = g / ME_C, slot = g % ME_C;
      // one round trip: header, price, the whole chunk's quantities and the target seq
      const ChunkHdr hd = bk.chunks[ch].hdr;
      const uint32_t owner_v = bk.chunks[ch].owner;
      const long long price = rli64(hd.price, 0);
      int qv = act ? cq_at(bk.chunks, (size_t)ch * ME_C + lane) : 0;
      unsigned long long sq = rl64(cs_at(bk.chunks, g), 0);
      const uint32_t owner = rl32(owner_v, 0);
      const long long lv64 = price - c.base;
      const bool inw = owner == c.s && (unsigned long long)lv64 < (unsigned long long)bk.L;
      const int lvl = inw ? (int)lv64 : 0;
      CacheEntry* E = inw && cache_holds(c, lvl, ch) ? centry(c, lvl) : nullptr;
      if (E) {  // the on-chip copy is authoritative
        qv = act ? E->qty[lane] : 0;
        sq = rl64(E->seq[slot], 0);
      }
      if (owner == c.s && sq == tgt) {  // the order's slot: live or dead, it never moves
        const int q = rli32(qv, (int)slot);
        if (q <= 0) return 0;
        const uint32_t nxt = rl32(hd.next, 0), prv = rl32(hd.prev, 0);
        if (!inw) return (int)far_cancel(c, price < c.base ? 0u : 1u, price, ch, slot, q, qv, nxt, prv);
        cancel_window(c, lvl, ch, slot, q, qv, nxt, prv, E);
        return q;
      }
    }
    // the ring entry is someone else's: only an order older than the horizon can still be live
    if (pass != 0 || tgt >= c.horizon) return 0;
    g = old_lookup((gptr<const OldEnt>)bk.old, bk.old_mask, c.epoch, tgt);
    if (g == NIL) return 0;
  }
}

// ---- re-centring the window (rare) ---------------------------------------------------------
// Shift the window arrays by d (level j <- level j + d, empty outside), one 64-level block per step;
// every block is exactly one occupancy word, rebuilt from the shifted totals. Ascending blocks for
// d > 0 and descending for d < 0, so no block reads what an earlier one wrote.
__device__ __forceinline__ void lad_shift(WaveCtx& c, int d) {
  const int lane = lane_id();
  const int L = (int)c.lad.L;
  wave_mem_order();
  for (int k = 0; k < L; k += 64) {
    const int j0 = d > 0 ? k : L - 64 - k;
    const int j = j0 + lane, src = j + d;
    const bool in = src >= 0 && src < L;
    Level v{0, NIL, NIL};
    uint32_t t = 0;
    if (in) {
      v = c.lad.lv[src];
      t = c.lad.tend[src];
    }
    const unsigned long long w = __ballot(v.total > 0);
    c.lad.lv[j] = v;
    c.lad.tend[j] = (uint8_t)t;
    if (lane == 0) c.lad.occ[j0 >> 6] = w;
  }
  wave_mem_order();
}

// Move the window so that it is centred on `target` as far as invariant I allows (me_far.hpp):
// cached heads go back to HBM and the cache is cleared (it is indexed by level), levels leaving the
// window become far levels at the best end of their side, the window arrays shift, and far levels
// now inside it are installed. Chunks name their level by price, so none of them changes.
__device__ void lad_recentre(WaveCtx& c, long long target) {
  const int lane = lane_id();
  const uint32_t L = c.lad.L;
  const long long base = c.base;
  const bool wb = c.bb >= 0, wa = c.ba < (int)L;
  long long bbp = 0, bap = 0;
  if (wb)
    bbp = base + c.bb;
  else if (c.nfar0)
    bbp = far_get(c.farr(0), c.nfar0 - 1u).price;
  if (wa)
    bap = base + c.ba;
  else if (c.nfar1)
    bap = far_get(c.farr(1), c.nfar1 - 1u).price;
  const long long nb = recentre_base(target, L, wb || c.nfar0 != 0u, bbp, wa || c.nfar1 != 0u, bap);
  if (nb == base) return;
  const bool up = nb > base;
  const unsigned long long dist =
      up ? (unsigned long long)nb - (unsigned long long)base : (unsigned long long)base - (unsigned long long)nb;
  const int dm = dist >= L ? (int)L : (int)dist;
  const int d = up ? dm : -dm;
  if (c.cache) {
    cache_flush_all(c, CK_MEM);
    for (uint32_t i = lane; i < (uint32_t)CK_MEM; i += 64) c.cache[i].cid = NIL;
    wave_mem_order();
  }
  if (d > 0) {  // bids leave at the bottom
    for (int l = c.lad.next_occ(0); l < d; l = c.lad.next_occ(l + 1)) {
      if (l > c.bb) set_err(c.bk, ERR_INCONSISTENT);
      const Level x = c.lad.get(l);
      FarLevel e;
      e.price = base + l;
      e.total = x.total;
      e.head = x.head;
      e.tail = x.tail;
      e.tend = c.lad.get_te(l);
      e.pad = 0;
      far_push(c, 0u, e);
    }
  } else {  // asks leave at the top
    for (int l = c.lad.prev_occ((int)L - 1); l >= (int)L + d; l = c.lad.prev_occ(l - 1)) {
      if (l < c.ba) set_err(c.bk, ERR_INCONSISTENT);
      const Level x = c.lad.get(l);
      FarLevel e;
      e.price = base + l;
      e.total = x.total;
      e.head = x.head;
      e.tail = x.tail;
      e.tend = c.lad.get_te(l);
      e.pad = 0;
      far_push(c, 1u, e);
    }
  }
  lad_shift(c, d);
  int nbb = (c.bb >= 0 && c.bb - d >= 0) ? c.bb - d : -1;
  int nba = (c.ba < (int)L && c.ba - d < (int)L) ? c.ba - d : (int)L;
  c.base = nb;
  const uint32_t k = d < 0 ? 0u : 1u;  // the side whose far levels may now be inside the window
  const gptr<FarLevel> a = c.farr(k);
  uint32_t n = c.fcount(k);
  while (n) {
    const FarLevel e = far_get(a, n - 1u);
    const unsigned long long off = (unsigned long long)e.price - (unsigned long long)nb;
    if (k == 0 ? e.price < nb : off >= L) break;
    if (off >= L) {  // impossible by recentre_base: never write outside the window
      set_err(c.bk, ERR_INCONSISTENT);
      break;
    }
    const int j = (int)off;
    Level x;
    x.total = e.total;
    x.head = e.head;
    x.tail = e.tail;
    c.lad.set(j, x);
    c.lad.set_te(j, e.tend);
    c.lad.occ_set(j);
    if (k == 0)
      nbb = j > nbb ? j : nbb;
    else
      nba = j < nba ? j : nba;
    --n;
  }
  c.fset_count(k, n);
  c.bb = nbb;
  c.ba = nba;
  wave_mem_order();
}

// Rest (seq, qty) at price p outside the window: re-centre first when the rest would put a bid above
// the window or an ask below it (invariant I) or when the window is empty; then a window or far rest.
__device__ bool far_or_window_rest(WaveCtx& c, long long p, unsigned long long seq, int qty, bool buy) {
  const uint32_t L = c.lad.L;
  const bool above = p > c.base;  // p is outside [base, base + L)
  const bool mandatory = buy == above;
  if (mandatory || (c.bb < 0 && c.ba >= (int)L)) lad_recentre(c, p);
  const unsigned long long off = (unsigned long long)p - (unsigned long long)c.base;
  if (off < L) return rest_order(c, (int)off, seq, qty, buy);
  if (mandatory) {
    set_err(c.bk, ERR_INCONSISTENT);
    return false;
  }
  return far_rest(c, p < c.base ? 0u : 1u, p, seq, (uint32_t)qty);
}

// Per-record results are collected in lane k for record k of the current 64-record block and
// stored by the whole wave once per block (a handful of vector stores instead of ~6 per record).
struct ResultLanes {
  int filled, remaining;
  uint32_t nfill, fstart, st;  // st = status | reason << 8
};

__device__ __forceinline__ void put_result(ResultLanes& r, uint32_t k, int filled, int remaining, uint32_t nfill,
                                           uint8_t status, uint8_t reason, unsigned long long fstart) {
  const bool me_ = (uint32_t)lane_id() == k;  // v_cmp + v_cndmask per field
  r.filled = me_ ? filled : r.filled;
  r.remaining = me_ ? remaining : r.remaining;
  r.nfill = me_ ? nfill : r.nfill;
  r.fstart = me_ ? (uint32_t)fstart : r.fstart;
  r.st = me_ ? (uint32_t)(status | (reason << 8)) : r.st;
}

__device__ __forceinline__ void store_results(const BatchDev& bt, const ResultLanes& r, bool v, uint32_t oi) {
  if (!v) return;
  me_order_result o;
  o.filled_qty = r.filled;
  o.remaining_qty = r.remaining;
  o.fill_count = r.nfill;
  o.tape_offset = 0;
  o.status = (uint8_t)(r.st & 0xFF);
  o.reason = (uint8_t)(r.st >> 8);
  o.pad[0] = o.pad[1] = 0;
  bt.res[oi] = o;
  bt.fstart[oi] = r.fstart;
  if (r.nfill) atomicAdd(&bt.tile_sum[oi / TILE_TAPE], r.nfill);
}

// LDS bytes of one wave: LDS ladder (levels + occupancy + tail fill) + head-chunk cache.
__host__ __device__ constexpr size_t lds_ladder_bytes(uint32_t L) {
  return (((size_t)L * sizeof(Level) + (size_t)(L / 64) * 8 + (size_t)L) + 15) & ~(size_t)15;
}
__host__ __device__ constexpr size_t lds_wave_bytes(uint32_t L) {
  return lds_ladder_bytes(L) + CK_MEM * sizeof(CacheEntry);
}

// Window placement of a k_match instantiation.
enum LadderKind { LAD_HBM = 0, LAD_LDS = 1 };

// One record's outcome (ok = false: a pool is exhausted, the batch fails with the sticky error word).
struct RecOut {
  int filled, remaining;
  uint32_t nfill;
  uint32_t st;  // status | reason << 8
  unsigned long long fstart;
  bool ok;
};
__device__ __forceinline__ RecOut rec_out(int filled, int remaining, uint32_t nfill, uint8_t status, uint8_t reason,
                                          unsigned long long fstart) {
  RecOut o;
  o.filled = filled;
  o.remaining = remaining;
  o.nfill = nfill;
  o.st = (uint32_t)status | ((uint32_t)reason << 8);
  o.fstart = fstart;
  o.ok = true;
  return o;
}

// One record in the generic way (deep windows): reject reasons, sweep, far levels, rest or cancel.
__device__ __forceinline__ RecOut generic_record(WaveCtx& c, unsigned long long seq, long long px, int q,
                                                 uint32_t kind) {
  const uint32_t Lw = c.bk.L;
  const uint32_t side = kind & 3u;
  const bool market = (kind >> 2) & 1u;
  const bool cancel = (kind >> 3) & 1u;
  const unsigned long long fstart = c.wptr;
  if (cancel) {
    const int got = cancel_order(c, (unsigned long long)px);
    STAMP_ADD(c, PH_CANCEL);
    return got > 0 ? rec_out(0, got, 0, ME_ST_CANCELED, ME_RJ_NONE, fstart)
                   : rec_out(0, 0, 0, ME_ST_REJECTED, ME_RJ_UNKNOWN_ORDER, fstart);
  }
  if (q <= 0) return rec_out(0, 0, 0, ME_ST_REJECTED, ME_RJ_BAD_QTY, fstart);
  if (side != ME_SIDE_BUY && side != ME_SIDE_SELL) return rec_out(0, q, 0, ME_ST_REJECTED, ME_RJ_BAD_SIDE, fstart);
  // no OID is 0 (the counter starts at 1, storage.cpp:254-267)
  if (seq == 0ull) return rec_out(0, q, 0, ME_ST_REJECTED, ME_RJ_BAD_SEQ, fstart);
  const bool buy = side == ME_SIDE_BUY;
  const unsigned long long off = (unsigned long long)px - (unsigned long long)c.base;
  const bool inw = off < (unsigned long long)Lw;
  const bool above = !inw && px > c.base;
  // last window level the taker may trade at (-1 / L: none) and whether it reaches past the window
  const int lim = market ? (buy ? (int)Lw - 1 : 0)
                : inw    ? (int)off
                : buy    ? (above ? (int)Lw - 1 : -1)
                         : (above ? (int)Lw : 0);
  const bool far = market || (buy ? above : (!inw && !above));
  long long got = sweep(c, buy ? 1 : -1, lim, (long long)q, seq);
  if (got < q && far && c.fcount(buy ? 1u : 0u) != 0u)
    got += far_take(c, buy, market, px, (uint32_t)(q - got), seq);
  STAMP_ADD(c, PH_SWEEP);
  const uint32_t nfill = (uint32_t)(c.wptr - fstart);
  const int filled = (int)got;
  const int rem = q - filled;
  uint8_t stt;
  if (market) {
    stt = rem == 0 ? ME_ST_FILLED : ME_ST_CANCELED;
  } else {
    const bool failed = rem > 0 && !(inw ? rest_order(c, (int)off, seq, rem, buy)
                                         : far_or_window_rest(c, px, seq, rem, buy));
    STAMP_ADD(c, PH_REST);
    if (failed) {
      RecOut o = rec_out(0, 0, 0, 0, 0, fstart);
      o.ok = false;
      return o;
    }
    stt = rem == 0 ? ME_ST_FILLED : (filled > 0 ? ME_ST_PARTIALLY_FILLED : ME_ST_NEW);
  }
  return rec_out(filled, rem, nfill, stt, ME_RJ_NONE, fstart);
}

__device__ __forceinline__ void put_rec(ResultLanes& r, uint32_t k, const RecOut& o) {
  const bool me_ = (uint32_t)lane_id() == k;
  r.filled = me_ ? o.filled : r.filled;
  r.remaining = me_ ? o.remaining : r.remaining;
  r.nfill = me_ ? o.nfill : r.nfill;
  r.fstart = me_ ? (uint32_t)o.fstart : r.fstart;
  r.st = me_ ? o.st : r.st;
}

// The per-record loop of one symbol.
__device__ __forceinline__ void match_records(WaveCtx& c, const BatchDev& bt, uint32_t lo, uint32_t hi) {
  const int lane = lane_id();
  bool ok = true;
  for (uint32_t blk = lo; blk < hi && ok; blk += 64) {
    const uint32_t j = blk + (uint32_t)lane;
    const bool v = j < hi;
    const uint32_t oi = v ? bt.perm[j] : 0u;
    const unsigned long long oseq = v ? bt.seq[oi] : 0ull;
    const long long opx = v ? bt.px[oi] : 0ll;
    const int oq = v ? bt.qty[oi] : 0;
    const uint32_t ok_ = v ? (uint32_t)bt.kind[oi] : 0u;
    const uint32_t cnt = min(64u, hi - blk);
    ResultLanes R;
    R.filled = R.remaining = 0;
    R.nfill = R.fstart = R.st = 0;
    STAMP_ADD(c, PH_FETCH);
    uint32_t k = 0;
    for (; k < cnt; ++k) {
      c.recs_left = hi - (blk + k);
      const RecOut o = generic_record(c, rl64(oseq, (int)k), rli64(opx, (int)k), rli32(oq, (int)k), rl32(ok_, (int)k));
      if (!o.ok) {
        ok = false;  // a pool is exhausted: the batch fails (sticky error word)
        break;
      }
      put_rec(R, k, o);
    }
    store_results(bt, R, v && (uint32_t)lane < k, oi);
    STAMP_ADD(c, PH_RESULT);
  }
  // return unused bump-reserved chunks to this symbol's free list
  while (c.bump_cur < c.bump_end) free_chunk(c, rl32(c.bump_ids, (int)c.bump_cur++));
}

// cont_w != ~0: a continuation (k_match_hot_cont) that writes its fills from cont_w on, inside the
// scratch run the symbol's first wave reserved for all its records of the batch.
__device__ __forceinline__ bool wave_begin(WaveCtx& c, const BookDev& bk, const BatchDev& bt, uint32_t s, uint32_t lo,
                                           uint32_t hi, unsigned long long cont_w = ~0ull) {
  const int lane = lane_id();
  c.bk = bk;
  c.s = s;
  c.gs = bk.gsym ? bk.gsym[s] : s;
  const SymState st = bk.sym[s];
  const SeqState sqs = bk.sq[bk.sq_idx];
  c.base = rli64(st.base, 0);
  c.bb = rli32(st.best_bid, 0);
  c.ba = rli32(st.best_ask, 0);
  c.free_head = rl32(st.free_head, 0);
  c.nfar0 = rl32(st.nfar[0], 0);
  c.nfar1 = rl32(st.nfar[1], 0);
  c.horizon = rl64(sqs.horizon, 0);
  c.epoch = rl32(sqs.epoch, 0);
  prefetch_free_next(c);
  c.bump_cur = c.bump_end = 0;
  c.resting_delta = (int)rl32(st.resting, 0);  // becomes the new resting count
  c.resting0 = rl32(st.resting, 0);
  c.scratch = bt.scratch;
  if (cont_w != ~0ull) {
    c.wptr = cont_w;
    return true;
  }
  // scratch run of this wave: fills <= resting makers + 2 * records
  const unsigned long long need = (unsigned long long)rl32(st.resting, 0) + 2ull * (hi - lo);
  unsigned long long w0 = 0;
  if (lane == 0) w0 = atomicAdd(bt.scratch_top, need);
  w0 = rl64(w0, 0);
  if (w0 + need > bt.scratch_cap) {
    set_err(bk, ERR_SCRATCH_OOM);
    return false;
  }
  c.wptr = w0;
  return true;
}

__device__ __forceinline__ void wave_end(WaveCtx& c) {
  if (lane_id() == 0) {
    SymState o;
    o.base = c.base;
    o.best_bid = c.bb;
    o.best_ask = c.ba;
    o.free_head = c.free_head;
    o.resting = (uint32_t)c.resting_delta;
    o.nfree = 0;
    o.nfar[0] = c.nfar0;
    o.nfar[1] = c.nfar1;
    for (int k = 0; k < 5; ++k) o.pad[k] = 0;
    c.bk.sym[c.s] = o;
    const long long d = (long long)(uint32_t)c.resting_delta - (long long)c.resting0;
    if (d) atomicAdd(c.bk.stats + ST_RESTING, (unsigned long long)d);
  }
#ifdef ME_STAMPS
  STAMP_ADD(c, PH_EPILOGUE);
  if (lane_id() == 0 && c.bk.dbg)
    for (int p = 0; p < PH_N; ++p) c.bk.dbg[(size_t)c.s * 24 + p] = c.st[p];
#endif
}

// One wavefront per symbol (4 per workgroup). Block s/4, wave s%4. Symbol S is the reject bin
// of records whose symbol id is out of range.
template <int kLad>
__global__ __launch_bounds__(256) void k_match(BookDev bk, BatchDev bt) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = lane_id();
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t s = blockIdx.x * 4u + wv;
  if (s > bk.S) return;
  const uint32_t lo = bt.bin_start ? bt.bin_start[s] : wave_lower_bound(bt.skeys, bt.n, s);
  const uint32_t hi = bt.bin_start ? bt.bin_start[s + 1] : wave_lower_bound(bt.skeys, bt.n, s + 1);
  if (lo >= hi) return;
  if (s == bk.S) {
    reject_bad_symbols(bt, lo, hi);
    return;
  }
  if (bk.hot_min && hi - lo >= bk.hot_min) return;  // k_match_hot's / the aggregate path's (k_hot_pick)
  const uint32_t L = bk.L;
  Level* g_lv = bk.levels + (size_t)s * L;
  unsigned long long* g_occ = bk.occ + (size_t)s * bk.Lwords;
  uint8_t* g_tend = bk.tend + (size_t)s * L;
  WaveCtx c;
#ifdef ME_STAMPS
  for (int p = 0; p < PH_N; ++p) c.st[p] = 0;
  STAMP_MARK(c);
#endif
  c.lad.L = L;
  c.lad.Lwords = bk.Lwords;
  if constexpr (kLad == LAD_LDS) {
    unsigned char* base = smem + (size_t)wv * lds_wave_bytes(L);
    c.lad.lv = (Level*)base;
    c.lad.occ = (unsigned long long*)(base + (size_t)L * sizeof(Level));
    c.lad.tend = base + (size_t)L * sizeof(Level) + (size_t)(L / 64) * 8;
    c.cache = (CacheEntry*)(base + lds_ladder_bytes(L));
    c.cmask = CK_MEM - 1;
    for (uint32_t i = lane; i < L; i += 64) {
      c.lad.lv[i] = g_lv[i];
      c.lad.tend[i] = g_tend[i];
    }
    for (uint32_t i = lane; i < bk.Lwords; i += 64) c.lad.occ[i] = g_occ[i];
    for (uint32_t i = lane; i < (uint32_t)CK_MEM; i += 64) c.cache[i].cid = NIL;
    wave_mem_order();
  } else {
    c.lad.lv = g_lv;
    c.lad.occ = g_occ;
    c.lad.tend = g_tend;
    c.lad.span0 = 8;
    c.lad.occ_reads = true;
    c.cache = nullptr;
    c.cmask = 0;
  }
  if (!wave_begin(c, bk, bt, s, lo, hi)) return;
  STAMP_ADD(c, PH_PROLOGUE);
  match_records(c, bt, lo, hi);
  if constexpr (kLad == LAD_LDS) {
    cache_flush_all(c, CK_MEM);
    for (uint32_t i = lane; i < L; i += 64) {
      g_lv[i] = c.lad.lv[i];
      g_tend[i] = c.lad.tend[i];
    }
    for (uint32_t i = lane; i < bk.Lwords; i += 64) g_occ[i] = c.lad.occ[i];
  }
  wave_end(c);
}

// ---- hot symbols of deep windows (k_match_hot) ------------------------------------------------
// A Zipf-hot symbol (config 4: one symbol draws ~14 % of the stream) is a serial chain on one wave,
// so its record loop sets the launch length. k_match's loop pays HBM round trips inside that chain —
// window and chunk loads per sweep, level reads per rest — and gfx9's single in-order vmcnt makes each
// of those loads also wait for every store the chain issued before it (measured: 2.25 us per record,
// half of it waiting). This path moves every load to the boundary of a 64-record block:
//
//   * top-of-book lists: per side the next HT occupied levels from the best, entry i in lane i (level,
//     total, head / tail chunk, tail fill, the head's next, its LDS row) with each head chunk's 16
//     slots in an LDS row — rebuilt in vector form (occupancy scan in LDS, one round trip for the
//     levels, one for their head chunks) when a side runs low; takers walk them as k_match_reg walks
//     its ladder; a level emptied at the front leaves by a one-lane rotation, a new level inside the
//     list's span enters at its sorted position by a one-lane shift (DPP wave_rol / wave_shr), so the
//     list always is the exact prefix of the side's occupied levels;
//   * deep rests: every record's own level (total, head, tail, tail fill) is loaded in vector form at
//     the block start and kept current: an update of an unlisted level, and a level leaving a list
//     (popped or truncated), is broadcast to the lanes of that level;
//   * the occupancy bitmap lives in LDS (windows up to HOT_MAX_WORDS * 64 levels);
//   * free chunks in a VGPR stack.
// Every change is written through to HBM at once (fire-and-forget global stores: nothing in the chain
// waits for them), so the HBM book is always current: at the first record the lists do not cover — a
// cancel, a price outside the window, a taker while far levels exist — the wave hands the symbol's
// remaining records to k_match_hot_cont (the generic record loop) and ends. Same semantics and HBM
// layout as k_match.
// The chain's state stays in registers (HotState): the generic code's WaveCtx lives in scratch memory
// and is touched only at those sync points.
constexpr int HT = 64;                  // list entries per side (one per lane)
constexpr uint32_t HOT_STACK_LOW = 16;  // top the free-chunk stack up at a block start below this ...
constexpr uint32_t HOT_STACK_FILL = 32; // ... to this

struct HotLds {
  int cq[2][HT][ME_C];                 // head chunk of the list entry owning row (side, row): slot quantities ...
  unsigned long long cs[2][HT][ME_C];  // ... and seqs (side 0 bids, 1 asks)
  unsigned long long occ[HOT_MAX_WORDS];
};

struct HSide {  // a top-of-book list of side k, best first: a ring over the lanes, entry i in lane (f + i) & 63
  int m;          // the entry's level in side coordinates (asks: the level; bids: L - 1 - level): smaller is better
  long long tot;
  uint32_t hd, tl, te, hn;
  uint32_t row;   // the entry's LDS row; lanes past the entries hold the free rows (the rows are a permutation)
  int f, n;       // wave-uniform: the front lane, the entries
  int more;       // wave-uniform: occupied levels of this side may lie beyond the last entry
  int k;          // wave-uniform: the side (0 bids, 1 asks)
};
__device__ __forceinline__ int hlane(const HSide& S, int i) { return (S.f + i) & (HT - 1); }

// A one-lane rotation of a ring (gfx9 DPP wavefront rotate): lane i <- lane i - 1, lane 0 <- lane 63.
// An entry enters mid-list by the rotation of the entries behind it.
__device__ __forceinline__ uint32_t lanes_up(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x13C, 0xf, 0xf, false);  // wave_ror:1
}
__device__ __forceinline__ long long lanes_up64(long long v) {
  return (long long)(((unsigned long long)lanes_up((uint32_t)((unsigned long long)v >> 32)) << 32) |
                     lanes_up((uint32_t)v));
}

struct HotState {
  gptr<Chunk> chunks;  // the HBM book (global address space: global_* instructions, never flat_*)
  gptr<uint32_t> loc;
  gptr<me_fill> scratch;
  gptr<Level> lv;
  gptr<unsigned long long> occ;
  gptr<uint8_t> tend;
  gptr<uint32_t> err;
  unsigned long long rmask;
  uint32_t nchunks, L, W;
  uint32_t gs;
  long long base;
  unsigned long long wptr;
  int resting;
  uint32_t free_head;  // HBM free list (hot frees only push onto it: a store) ...
  uint32_t free_next;  // ... and free_head's next (the generic pop reads it instead of loading it)
  uint32_t nfar0, nfar1;
  uint32_t fstk, nfs;  // VGPR free-chunk stack: lane i holds entry i, entries [0, nfs)
  HotLds* H;
  HSide A, B;  // the asks (k = 1) and the bids (k = 0)
  // per-record lane state of the current block (lane k = record k): the window level it rests at
  // (-1: none) and that level's total / head / tail / tail fill, loaded at the block start, kept current
  int rlvl;
  long long rtot;
  uint32_t rhd, rtl, rte;
#ifdef ME_STAMPS
  unsigned long long ev[8];   // event counts (stamps build): see HEV_*
  unsigned long long cyc[8];  // cycles of the hot helpers' parts: see HC_*
  unsigned long long ct;
#endif
};
#ifdef ME_STAMPS
enum { HEV_TAKE_REBUILD, HEV_ADVANCE, HEV_TRUNC_ENTRIES, HEV_GAP, HEV_NEWBEST, HEV_APPEND, HEV_DEEP, HEV_POP };
enum { HC_CHUNK, HC_POP, HC_PARTIAL, HC_APPEND, HC_INSERT, HC_DEEP, HC_RESTHEAD, HC_TAKEHEAD };
#define HEV(h, e) ((h).ev[e] += 1)
#define HC_MARK(h) ((h).ct = stamp_now())
#define HC_ADD(h, i)                          \
  do {                                        \
    const unsigned long long n_ = stamp_now(); \
    (h).cyc[i] += n_ - (h).ct;                \
    (h).ct = n_;                              \
  } while (0)
#else
#define HEV(h, e) ((void)0)
#define HC_MARK(h) ((void)0)
#define HC_ADD(h, i) ((void)0)
#endif

// Diagnostic ablation builds only (-DHOT_ABL=bits, never the product): drop classes of HBM stores to
// measure what they cost the chain (results are then wrong).
#ifndef HOT_ABL
#define HOT_ABL 0
#endif
#define ABL(b) ((HOT_ABL & (b)) != 0)
#ifdef HOT_MARKS  // asm listing landmarks (make asm HOT_MARKS=1): no instructions
#define HMARK(s) asm volatile(";@@ " s)
#else
#define HMARK(s) ((void)0)
#endif

// Side coordinates <-> window levels (the same map both ways).
__device__ __forceinline__ int side_lvl(const HotState& h, int k, int m) { return k ? m : (int)h.L - 1 - m; }

// Pins a wave-uniform value to an SGPR (values that come back from memory or calls are otherwise
// treated as divergent, and so is every branch on them).
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// The generic code's view (sync points only): hot fields in, run, hot fields out. The best levels come
// from the list fronts (a list is empty only with its side).
__device__ __forceinline__ void hot_to_wave(const HotState& h, WaveCtx& c) {
  const int L = (int)h.L;
  const int a0 = h.A.n ? rli32(h.A.m, h.A.f) : L, b0 = h.B.n ? rli32(h.B.m, h.B.f) : L;
  c.ba = h.A.k ? a0 : b0;
  c.bb = L - 1 - (h.A.k ? b0 : a0);
  c.base = h.base;
  c.wptr = h.wptr;
  c.resting_delta = h.resting;
  c.free_head = h.free_head;
  c.free_next = h.free_next;
  c.nfar0 = h.nfar0;
  c.nfar1 = h.nfar1;
}
// (The WaveCtx lives in scratch memory: whatever comes back from it is pinned to SGPRs, or the
// compiler would treat it — and every branch on it — as divergent.)
__device__ __forceinline__ void wave_to_hot(const WaveCtx& c, HotState& h) {
  h.base = rli64(c.base, 0);
  h.wptr = rl64(c.wptr, 0);
  h.resting = rli32(c.resting_delta, 0);
  h.free_head = rl32(c.free_head, 0);
  h.free_next = rl32(c.free_next, 0);
  h.nfar0 = rl32(c.nfar0, 0);
  h.nfar1 = rl32(c.nfar1, 0);
}

// ---- occupancy (LDS copy, written through to HBM one word at a time)
__device__ __forceinline__ void hot_occ_load(HotState& h) {
  for (uint32_t i = (uint32_t)lane_id(); i < h.W; i += 64) h.H->occ[i] = h.occ[i];
  wave_mem_order();
}
// Non-returning atomics on both copies: nothing in the chain waits for them (a read-modify-write
// would wait for the LDS read).
__device__ __forceinline__ void hot_occ_set(HotState& h, int lvl, bool on) {
  const uint32_t w = (uint32_t)lvl >> 6;
  const unsigned long long bit = 1ull << (lvl & 63);
  if (lane_id() == 0) {
    if (on) {
      __atomic_fetch_or(&h.H->occ[w], bit, __ATOMIC_RELAXED);
      if (!ABL(8)) __atomic_fetch_or(&h.occ[w], bit, __ATOMIC_RELAXED);
    } else {
      __atomic_fetch_and(&h.H->occ[w], ~bit, __ATOMIC_RELAXED);
      if (!ABL(8)) __atomic_fetch_and(&h.occ[w], ~bit, __ATOMIC_RELAXED);
    }
  }
}

// The r-th (0-based) set bit of w (w has more than r set bits).
__device__ __forceinline__ uint32_t nth_set(unsigned long long w, uint32_t r) {
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t hsz = 32; hsz >= 1; hsz >>= 1) {
    const uint32_t c = (uint32_t)__popcll(w & ((1ull << hsz) - 1ull));
    const bool up = r >= c;
    r = up ? r - c : r;
    w = up ? (w >> hsz) : w;
    pos += up ? hsz : 0u;
  }
  return pos;
}

// Lanes 0..n-1 <- the first (up to) HT occupied levels from window level `start` going up (K = 1) or
// down (K = 0), from the LDS occupancy copy. *more: the list filled before the window ended.
template <int K>
__device__ __forceinline__ int hot_scan(const HotState& h, int start, int& out_lvl, bool& more) {
  const int lane = lane_id();
  const int W = (int)h.W;
  out_lvl = -1;
  more = false;
  if (start < 0 || start >= (int)h.L) return 0;
  int found = 0;
  const int w0 = start >> 6;
  for (int base = 0;; base += 64) {
    const int wi = K ? w0 + base + lane : w0 - base - lane;
    const bool in = wi >= 0 && wi < W;
    unsigned long long w = in ? h.H->occ[wi] : 0ull;
    if (wi == w0)  // the start word: only levels at / beyond start
      w &= K ? (~0ull << (start & 63)) : (~0ull >> (63 - (start & 63)));
    if (!K) w = __builtin_bitreverse64(w);  // descending: bit 0 = the word's highest level
    const uint32_t cnt = (uint32_t)__popcll(w);
    const long long inc = wave_incl_scan((long long)cnt);
    const uint32_t ex = (uint32_t)(inc - cnt);
    const uint32_t tot = (uint32_t)rli64(inc, 63);
    const int i = lane - found;  // output lane i takes bit (i - ex_j) of the lane j holding it
    int lo = 0;
#pragma unroll
    for (int st = 32; st >= 1; st >>= 1) {
      const uint32_t e = (uint32_t)__shfl((int)ex, min(lo + st, 63), 64);
      if (lo + st < 64 && (int)e <= i) lo += st;
    }
    const unsigned long long wj = (unsigned long long)__shfl((long long)w, lo, 64);
    const uint32_t r = (uint32_t)(i - __shfl((int)ex, lo, 64));
    const uint32_t b = nth_set(wj, r);
    const int wdx = K ? w0 + base + lo : w0 - base - lo;
    if (i >= 0 && (uint32_t)i < tot) out_lvl = wdx * 64 + (K ? (int)b : 63 - (int)b);
    found = min(found + (int)tot, HT);
    const bool end = K ? (w0 + base + 64 >= W) : (w0 - base - 64 < 0);
    if (found >= HT) {
      more = true;  // conservative: a later rebuild finds out
      return HT;
    }
    if (end) return found;
  }
}

// Rebuild list S from side coordinate start_m (the best, or a bound no level of either side lies
// inside): occupancy scan (LDS), the levels (one round trip) and their head chunks (one round trip)
// into lanes / LDS rows. The caller has waited for every store.
template <int K>
__device__ __forceinline__ void hot_rebuild(HotState& h, HSide& S, int start_m) {
  const int lane = lane_id();
  const int L = (int)h.L;
  int lvl = -1, n = 0;
  bool more = false;
  if (start_m < L) n = hot_scan<K>(h, K ? (start_m < 0 ? 0 : start_m) : L - 1 - (start_m < 0 ? 0 : start_m), lvl, more);
  const bool v = lane < n;
  const int li = v ? lvl : 0;
  Level x{0, NIL, NIL};
  uint32_t te = 0;
  if (v) {
    x = h.lv[li];
    te = h.tend[li];
  }
  const bool hv = v && x.head < h.nchunks;
  const gptr<Chunk> ch = h.chunks + (hv ? x.head : 0u);
  // the head chunk's 16 quantities and seqs: 12 x 16-B loads per lane, all in flight, then into LDS
  typedef int v4i __attribute__((ext_vector_type(4)));
  const gptr<const v4i> src = reinterpret_cast<gptr<const v4i>>(ch->qty);  // qty[16] then seq[16]
  const v4i a0 = src[0], a1 = src[1], a2 = src[2], a3 = src[3], b0 = src[4], b1 = src[5], b2 = src[6],
            b3 = src[7], b4 = src[8], b5 = src[9], b6 = src[10], b7 = src[11];
  const uint32_t hn = ch->hdr.next;
  v4i* dq = reinterpret_cast<v4i*>(h.H->cq[K][lane]);
  v4i* ds = reinterpret_cast<v4i*>(h.H->cs[K][lane]);
  dq[0] = a0;
  dq[1] = a1;
  dq[2] = a2;
  dq[3] = a3;
  ds[0] = b0;
  ds[1] = b1;
  ds[2] = b2;
  ds[3] = b3;
  ds[4] = b4;
  ds[5] = b5;
  ds[6] = b6;
  ds[7] = b7;
  S.m = v ? side_lvl(h, K, lvl) : L;
  S.tot = v ? x.total : 0;
  S.hd = v ? x.head : NIL;
  S.tl = v ? x.tail : NIL;
  S.te = te;
  S.hn = hv ? hn : NIL;
  S.row = (uint32_t)lane;
  S.f = 0;
  S.n = n;
  S.more = more;
}

// The block's per-record level states, loaded in vector form (lanes with rlvl >= 0).
__device__ __forceinline__ void hot_prefetch(HotState& h) {
  const bool v = h.rlvl >= 0;
  const int li = v ? h.rlvl : 0;
  Level x{0, NIL, NIL};
  uint32_t te = 0;
  if (v) {
    x = h.lv[li];
    te = h.tend[li];
  }
  h.rtot = x.total;
  h.rhd = x.head;
  h.rtl = x.tail;
  h.rte = te;
}

__device__ __forceinline__ void hot_drain() {
  __builtin_amdgcn_s_waitcnt(0);
  wave_mem_order();
}

// ---- chunks: VGPR stack
__device__ __forceinline__ void hot_free(HotState& h, uint32_t ch) {
  if (ME_LIKELY(h.nfs < (uint32_t)HT)) {
    h.fstk = lane_id() == (int)h.nfs ? ch : h.fstk;
    h.nfs += 1;
  } else {  // onto the symbol's HBM free list: a store (as free_chunk)
    if (lane_id() == 0) h.chunks[ch].hdr.next = h.free_head;
    h.free_next = h.free_head;
    h.free_head = ch;
  }
}

// Record the level's header and tail fill in HBM.
__device__ __forceinline__ void hot_level_store(HotState& h, int lvl, long long tot, uint32_t hd, uint32_t tl,
                                                uint32_t te) {
  if (lane_id() == 0 && !ABL(4)) {
    Level o;
    o.total = tot;
    o.head = tot ? hd : NIL;
    o.tail = tot ? tl : NIL;
    h.lv[lvl] = o;
    h.tend[lvl] = (uint8_t)te;
  }
}

// New chunk ch holding one order (seq, q) at level lvl, behind tail `prev` (NIL: the level's only chunk).
__device__ __forceinline__ void hot_new_chunk(HotState& h, uint32_t ch, uint32_t prev, int lvl,
                                              unsigned long long seq, int q) {
  if (lane_id() == 0 && !ABL(16)) {
    ChunkHdr hh;
    hh.next = NIL;
    hh.prev = prev;
    hh.price = h.base + lvl;
    h.chunks[ch].hdr = hh;
    h.chunks[ch].qty[0] = q;
    h.chunks[ch].seq[0] = seq;
    if (prev != NIL) h.chunks[prev].hdr.next = ch;
    h.loc[seq & h.rmask] = ch * ME_C;
  }
}

// Record lanes of level lvl take its state (a level that leaves a list, or a deep level just changed).
__device__ __forceinline__ void hot_broadcast(HotState& h, int lvl, long long tot, uint32_t hd, uint32_t tl,
                                             uint32_t te) {
  const bool m = h.rlvl == lvl;
  h.rtot = m ? tot : h.rtot;
  h.rhd = m ? hd : h.rhd;
  h.rtl = m ? tl : h.rtl;
  h.rte = m ? te : h.rte;
}

// The last entry of a full list leaves it (a level entering the list takes its place and row).
__device__ __forceinline__ void hot_drop_last(HotState& h, HSide& S) {
  HEV(h, HEV_TRUNC_ENTRIES);
  const int j = hlane(S, S.n - 1);
  hot_broadcast(h, side_lvl(h, S.k, rli32(S.m, j)), rli64(S.tot, j), rl32(S.hd, j), rl32(S.tl, j), rl32(S.te, j));
  S.n -= 1;
  S.more = true;
}

__device__ __noinline__ uint32_t hot_alloc_slow(WaveCtx* c);

// A free chunk: the VGPR stack, else (rare) the symbol's free list or the bump allocator through the
// generic allocator, after one full wait (its free-list loads must see this wave's stores). NIL: the
// chunk pool is exhausted (sticky error word).
__device__ __forceinline__ uint32_t hot_alloc(HotState& h, WaveCtx& c) {
  if (ME_LIKELY(h.nfs)) {
    h.nfs -= 1;
    return rl32(h.fstk, (int)h.nfs);
  }
  hot_drain();
  hot_to_wave(h, c);
  const uint32_t ch = (uint32_t)uni((int)hot_alloc_slow(&c));
  wave_to_hot(c, h);
  return ch;
}

// Take up to rem from list O (side K) front levels while they cross lim (side coordinates). One pass
// per chunk of the front level: a partial take ends the taker, an exhausted chunk frees it and then
// pops the level (its last chunk) or moves the level's head to the next chunk (a load, rare).
template <int K>
__device__ __forceinline__ void hot_take(HotState& h, HSide& O, int lim, uint32_t& rem, unsigned long long taker) {
  const int lane = lane_id();
  const bool act = lane < ME_C;
  const int sl = lane & (ME_C - 1);
  HC_MARK(h);
  HMARK("take-entry");
  while (rem && O.n) {
    HMARK("take-level");
    const int f = O.f;
    const int m0 = rli32(O.m, f);
    if (m0 > lim) break;
    const int lvl = side_lvl(h, K, m0);
    const uint32_t hd = rl32(O.hd, f), tl = rl32(O.tl, f), r = rl32(O.row, f);
    const long long tot = rli64(O.tot, f);
    if (ME_UNLIKELY(hd >= h.nchunks)) {  // a corrupt list entry: never index with it
      if (lane == 0) atomicOr(h.err, ERR_INCONSISTENT);
      rem = 0;
      break;
    }
    int* rq = h.H->cq[K][r];
    unsigned long long* rs = h.H->cs[K][r];
    HC_ADD(h, HC_TAKEHEAD);
    HMARK("take-chunk");
    const int q_ = rq[sl];
    const unsigned long long mseq = vreg64(rs[sl]);
    const uint32_t uq = act ? (uint32_t)q_ : 0u;
    const uint32_t inc = scan16_sat(uq);
    const uint32_t ex = inc - uq;
    uint32_t fq = rem > ex ? rem - ex : 0u;
    fq = fq < uq ? fq : uq;
    const bool fe = fq != 0u;
    const unsigned long long fm = __ballot(fe);
    if (fe) {
      me_fill F;
      F.taker_seq = taker;
      F.maker_seq = mseq;
      F.price_q4 = h.base + lvl;
      F.qty = (int)fq;
      F.symbol = h.gs;
      if (!ABL(1)) h.scratch[h.wptr + (unsigned long long)__builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u)] = F;
      rq[sl] = (int)(uq - fq);
      if (!ABL(2)) h.chunks[hd].qty[sl] = (int)(uq - fq);
    }
    h.wptr += (unsigned long long)__popcll(fm);
    h.resting -= __popcll(__ballot(fq == uq) & fm);
    const uint32_t live = rl32(inc, 15);
    const uint32_t t = rem < live ? rem : live;
    rem -= t;
    const long long ntot = tot - t;
    HC_ADD(h, HC_CHUNK);
    HMARK("take-chunk-done");
    if (__ballot(uq > fq) & 0xFFFFull) {  // live slots remain: the taker is done, the level stays
      HMARK("take-partial");
      O.tot = lane == f ? ntot : O.tot;
      hot_level_store(h, lvl, ntot, hd, tl, rl32(O.te, f));
      HC_ADD(h, HC_PARTIAL);
      break;
    }
    // the chunk is exhausted (its HBM slots read 0 already)
    hot_free(h, hd);
    if (ntot == 0) {  // the level emptied: pop it (record lanes of it learn: a later rest may find it deep)
      HMARK("take-pop");
      HEV(h, HEV_POP);
      hot_level_store(h, lvl, 0, NIL, NIL, 0);
      hot_occ_set(h, lvl, false);
      hot_broadcast(h, lvl, 0, NIL, NIL, 0);
      O.f = (f + 1) & (HT - 1);  // the front lane and its row join the free ones
      O.n -= 1;
      if (ME_UNLIKELY(!O.n && O.more)) {
        // the list ran dry with levels beyond it: rebuild it now, so that an empty list always means
        // an empty side (a scan from a mere bound could run into the other side's levels later: the
        // occupancy bitmap holds both)
        HEV(h, HEV_TAKE_REBUILD);
        hot_drain();
        hot_rebuild<K>(h, O, m0 + 1);
        __builtin_amdgcn_s_waitcnt(0);
      }
      HC_ADD(h, HC_POP);
      HMARK("take-pop-done");
      continue;
    }
    // a multi-chunk level: its head moves to the next chunk (the one load of a walk; the chain's own
    // stores to it land first); the next pass takes from it
    const uint32_t nx = rl32(O.hn, f);
    if (ME_UNLIKELY(hd == tl || nx >= h.nchunks)) {  // a corrupt FIFO: stop the taker, report it
      if (lane == 0) atomicOr(h.err, ERR_INCONSISTENT);
      rem = 0;
      break;
    }
    HEV(h, HEV_ADVANCE);
    hot_drain();
    const int nq = h.chunks[nx].qty[sl];
    const unsigned long long ns = h.chunks[nx].seq[sl];
    const uint32_t nn = h.chunks[nx].hdr.next;
    __builtin_amdgcn_s_waitcnt(0);
    if (act) {
      rq[sl] = nq;
      rs[sl] = ns;
    }
    if (lane == 0) h.chunks[nx].hdr.prev = NIL;
    O.hd = lane == f ? nx : O.hd;
    O.hn = lane == f ? rl32(nn, 0) : O.hn;
    O.tot = lane == f ? ntot : O.tot;
    if (!rem) {
      hot_level_store(h, lvl, ntot, nx, tl, rl32(O.te, f));
      break;
    }
  }
}

// Rest (seq, q) on list M (side K) at side coordinate mm (window level lvl); record lane kr holds the
// level's state. False: the chunk pool is exhausted.
template <int K>
__device__ __forceinline__ bool hot_rest(HotState& h, WaveCtx& c, HSide& M, int mm, int lvl, unsigned long long seq,
                                         int q, int kr) {
  const int lane = lane_id();
  HC_MARK(h);
  HMARK("rest-entry");
  const int rel = (lane - M.f) & (HT - 1);
  const bool ent = rel < M.n;
  const int p = __popcll(__ballot(ent && M.m < mm));  // entries better than the level
  HC_ADD(h, HC_RESTHEAD);
  if (p < M.n && rli32(M.m, hlane(M, p)) == mm) {  // a listed level: append
    HMARK("rest-append");
    HEV(h, HEV_APPEND);
    const int j = hlane(M, p);
    const uint32_t te = rl32(M.te, j), tl = rl32(M.tl, j), hd = rl32(M.hd, j);
    const long long tot = rli64(M.tot, j) + q;
    uint32_t ntl = tl, nte = te + 1;
    if (ME_UNLIKELY(tl >= h.nchunks)) {
      if (lane == 0) atomicOr(h.err, ERR_INCONSISTENT);
      return true;
    }
    if (te < (uint32_t)ME_C) {
      if (tl == hd) {
        const uint32_t r = rl32(M.row, j);
        if (lane == 0) {
          h.H->cq[K][r][te] = q;
          h.H->cs[K][r][te] = seq;
        }
      }
      if (lane == 0) {
        h.chunks[tl].qty[te] = q;
        h.chunks[tl].seq[te] = seq;
        h.loc[seq & h.rmask] = tl * ME_C + te;
      }
    } else {
      const uint32_t ch = hot_alloc(h, c);
      if (ME_UNLIKELY(ch == NIL)) return false;
      hot_new_chunk(h, ch, tl, lvl, seq, q);
      if (tl == hd) M.hn = lane == j ? ch : M.hn;
      ntl = ch;
      nte = 1;
    }
    hot_level_store(h, lvl, tot, hd, ntl, nte);
    M.tot = lane == j ? tot : M.tot;
    M.tl = lane == j ? ntl : M.tl;
    M.te = lane == j ? nte : M.te;
    h.resting += 1;
    HC_ADD(h, HC_APPEND);
    return true;
  }
  if (p < M.n || (!M.more && p < HT)) {
    // an empty level inside the list's span (or past its end when nothing lies beyond): it enters
    // at position p, the entries behind it move one lane up (a full list drops its last entry)
    HMARK("rest-insert");
    if (p == 0)
      HEV(h, HEV_NEWBEST);
    else
      HEV(h, HEV_GAP);
    const uint32_t ch = hot_alloc(h, c);
    if (ME_UNLIKELY(ch == NIL)) return false;
    if (M.n == HT) hot_drop_last(h, M);
    hot_new_chunk(h, ch, NIL, lvl, seq, q);
    hot_level_store(h, lvl, q, ch, ch, 1);
    hot_occ_set(h, lvl, true);
    int j;
    uint32_t r;
    if (p == 0) {  // a new best: the front moves one lane back, onto a free lane and its row
      M.f = (M.f - 1) & (HT - 1);
      j = M.f;
      r = rl32(M.row, j);
    } else {  // entries p.. move one lane up (the ring rotates under them); the new one takes the
              // row of the first free lane
      j = hlane(M, p);
      r = rl32(M.row, hlane(M, M.n));
      const bool up = rel > p && rel <= M.n;
      const int um = (int)lanes_up((uint32_t)M.m);
      const long long utot = lanes_up64(M.tot);
      const uint32_t uhd = lanes_up(M.hd), utl = lanes_up(M.tl), ute = lanes_up(M.te), uhn = lanes_up(M.hn),
                     urow = lanes_up(M.row);
      M.m = up ? um : M.m;
      M.tot = up ? utot : M.tot;
      M.hd = up ? uhd : M.hd;
      M.tl = up ? utl : M.tl;
      M.te = up ? ute : M.te;
      M.hn = up ? uhn : M.hn;
      M.row = up ? urow : M.row;
    }
    const bool at = lane == j;
    M.m = at ? mm : M.m;
    M.tot = at ? (long long)q : M.tot;
    M.hd = at ? ch : M.hd;
    M.tl = at ? ch : M.tl;
    M.te = at ? 1u : M.te;
    M.hn = at ? NIL : M.hn;
    M.row = at ? r : M.row;
    if (lane < ME_C) {
      h.H->cq[K][r][lane] = lane == 0 ? q : 0;
      h.H->cs[K][r][lane] = lane == 0 ? seq : 0ull;
    }
    M.n += 1;
    hot_broadcast(h, lvl, q, ch, ch, 1);
    h.resting += 1;
    HC_ADD(h, HC_INSERT);
    return true;
  }
  // deep (beyond the list's last entry, with unlisted levels there): the record lane's level state
  HMARK("rest-deep");
  HEV(h, HEV_DEEP);
  const long long tot0 = rli64(h.rtot, kr);
  const uint32_t hd0 = rl32(h.rhd, kr), tl0 = rl32(h.rtl, kr), te0 = rl32(h.rte, kr);
  const long long tot = tot0 + q;
  uint32_t hd = hd0, tl = tl0, te = te0 + 1;
  if (ME_UNLIKELY(tot0 != 0 && tl0 >= h.nchunks)) {
    if (lane == 0) atomicOr(h.err, ERR_INCONSISTENT);
    return true;
  }
  if (tot0 == 0 || te0 >= (uint32_t)ME_C) {
    const uint32_t ch = hot_alloc(h, c);
    if (ME_UNLIKELY(ch == NIL)) return false;
    hot_new_chunk(h, ch, tot0 ? tl0 : NIL, lvl, seq, q);
    if (!tot0) {
      hd = ch;
      hot_occ_set(h, lvl, true);
    }
    tl = ch;
    te = 1;
  } else if (lane == 0) {
    h.chunks[tl0].qty[te0] = q;
    h.chunks[tl0].seq[te0] = seq;
    h.loc[seq & h.rmask] = tl0 * ME_C + te0;
  }
  hot_level_store(h, lvl, tot, hd, tl, te);
  hot_broadcast(h, lvl, tot, hd, tl, te);
  h.resting += 1;
  HC_ADD(h, HC_DEEP);
  return true;
}

// The generic allocator out of line: the hot loop's registers do not pay for it (its WaveCtx lives in
// scratch memory anyway, since the generic helpers take its address).
__device__ __noinline__ uint32_t hot_alloc_slow(WaveCtx* c) { return alloc_chunk(*c); }
__device__ __noinline__ void hot_free_slow(WaveCtx* c, uint32_t ch) { free_chunk(*c, ch); }

// The stack top-up (and the end of the wave) at a sync point: every store landed, the WaveCtx takes
// the hot state.
__device__ __forceinline__ void hot_sync_in(HotState& h, WaveCtx& c) {
  hot_drain();
  hot_to_wave(h, c);
}
__device__ __forceinline__ void hot_topup(HotState& h, WaveCtx& c) {
  hot_sync_in(h, c);
  while (h.nfs < HOT_STACK_FILL) {
    const uint32_t ch = (uint32_t)uni((int)hot_alloc_slow(&c));
    if (ch == NIL) break;
    h.fstk = lane_id() == (int)h.nfs ? ch : h.fstk;
    h.nfs += 1;
  }
  wave_to_hot(c, h);
}

#ifdef ME_HOT_CHECK
// Diagnostic build only (make hotcheck): after every record, the lists, record-lane states and LDS
// copies against the HBM book; the first mismatch is printed and stops the wave (ERR_INCONSISTENT).
// other_best: the other side's best window level (-1 / L: none); no level lies between the two.
__device__ bool hot_check_side(HotState& h, const HSide& S, int other_best, unsigned long long seq, int what) {
  const int lane = lane_id();
  const int L = (int)h.L;
  const int rel = (lane - S.f) & (HT - 1);
  const bool ent = rel < S.n;
  bool bad = false;
  int code = 0;
  long long a0 = 0, a1 = 0;
  const int l = side_lvl(h, S.k, S.m);
  if (ent) {
    if (l < 0 || l >= L) {
      bad = true, code = 1, a0 = l;
    } else {
      const Level x = h.lv[l];
      const uint32_t te = h.tend[l];
      const bool occ = (h.occ[l >> 6] >> (l & 63)) & 1ull;
      const bool locc = (h.H->occ[l >> 6] >> (l & 63)) & 1ull;
      if (x.total != S.tot || x.total <= 0) bad = true, code = 2, a0 = x.total, a1 = S.tot;
      else if (x.head != S.hd) bad = true, code = 3, a0 = x.head, a1 = S.hd;
      else if (x.tail != S.tl) bad = true, code = 4, a0 = x.tail, a1 = S.tl;
      else if (te != S.te) bad = true, code = 5, a0 = te, a1 = S.te;
      else if (!occ || !locc) bad = true, code = 6, a0 = occ, a1 = locc;
      else if (S.hd >= h.nchunks || S.tl >= h.nchunks) bad = true, code = 7, a0 = S.hd, a1 = S.tl;
      else {
        const Chunk& C = h.chunks[S.hd];
        if (C.hdr.next != (S.hd == S.tl ? NIL : S.hn)) bad = true, code = 8, a0 = C.hdr.next, a1 = S.hn;
        else if (C.hdr.price != h.base + l) bad = true, code = 9, a0 = C.hdr.price, a1 = h.base + l;
        else {
          for (int j = 0; j < ME_C; ++j) {
            if (C.qty[j] != h.H->cq[S.k][S.row][j]) {
              bad = true, code = 10, a0 = C.qty[j], a1 = h.H->cq[S.k][S.row][j];
              break;
            }
            if (C.qty[j] > 0 && C.seq[j] != h.H->cs[S.k][S.row][j]) {
              bad = true, code = 11, a0 = (long long)C.seq[j], a1 = (long long)h.H->cs[S.k][S.row][j];
              break;
            }
          }
        }
      }
    }
  }
  // the entries are the first n occupied levels beyond the other side's best, in order
  int sl;
  bool more;
  const int n2 = S.k ? hot_scan<1>(h, other_best + 1, sl, more) : hot_scan<0>(h, other_best - 1, sl, more);
  if (!bad && S.n > n2) bad = true, code = 12, a0 = S.n, a1 = n2;
  if (!bad && !S.n && n2) bad = true, code = 14, a0 = rli32(sl, 0), a1 = n2;
  {
    const int mine = __shfl(l, hlane(S, lane), 64);  // entry `lane` of the list
    if (!bad && lane < S.n && mine != sl) bad = true, code = 15, a0 = mine, a1 = sl;
  }
  {  // the rows are a permutation of 0..63
    unsigned long long seen = 0;
    for (int i = 0; i < HT; ++i) seen |= 1ull << (rl32(S.row, i) & 63u);
    if (!bad && (seen != ~0ull || S.row >= (uint32_t)HT)) bad = true, code = 17, a0 = (long long)seen, a1 = S.row;
  }
  const unsigned long long bm = __ballot(bad);
  if (!bm) return true;
  const int j = __builtin_ctzll(bm);
  if (lane == j)
    printf("HOTCHECK s=%u side=%d what=%d seq=%llu lane=%d code=%d a0=%lld a1=%lld n=%d row=%u more=%d lvl=%d other=%d\n",
           h.gs, S.k, what, seq, lane, code, a0, a1, S.n, S.row, (int)S.more, l, other_best);
  return false;
}
__device__ bool hot_check_lists(HotState& h, unsigned long long seq, int what) {
  const int L = (int)h.L;
  const int fa = h.A.n ? side_lvl(h, h.A.k, rli32(h.A.m, h.A.f)) : (h.A.k ? L : -1);
  const int fb = h.B.n ? side_lvl(h, h.B.k, rli32(h.B.m, h.B.f)) : (h.B.k ? L : -1);
  if (h.A.k == h.B.k) {
    if (lane_id() == 0) printf("HOTCHECK both lists hold side %d\n", h.A.k);
    return false;
  }
  if (!hot_check_side(h, h.A, fb, seq, what) || !hot_check_side(h, h.B, fa, seq, what)) return false;
  const int lane = lane_id();
  bool bad = false;
  for (uint32_t i = (uint32_t)lane; i < h.W; i += 64)
    if (h.occ[i] != h.H->occ[i]) bad = true;
  if (__ballot(bad)) {
    if (lane == 0) printf("HOTCHECK occ copy differs what=%d seq=%llu\n", what, seq);
    return false;
  }
  // record lanes of unlisted levels hold their HBM state
  const int l = h.rlvl;
  bool listed = false;
  for (int i = 0; i < h.A.n; ++i) listed |= side_lvl(h, h.A.k, rli32(h.A.m, hlane(h.A, i))) == l;
  for (int i = 0; i < h.B.n; ++i) listed |= side_lvl(h, h.B.k, rli32(h.B.m, hlane(h.B, i))) == l;
  if (l >= 0 && !listed) {
    const Level x = h.lv[l];
    const uint32_t te = h.tend[l];
    if (x.total != h.rtot || (x.total && (x.head != h.rhd || x.tail != h.rtl || te != h.rte))) bad = true;
  }
  const unsigned long long bm = __ballot(bad);
  if (bm) {
    if (lane == __builtin_ctzll(bm))
      printf("HOTCHECK record lane %d lvl=%d what=%d seq=%llu rtot=%lld tot=%lld\n", lane, l, what, seq, h.rtot,
             h.lv[l].total);
    return false;
  }
  if (h.nfs > (uint32_t)HT || (lane < (int)h.nfs && h.fstk >= h.nchunks)) {
    if (lane == 0) printf("HOTCHECK stack what=%d\n", what);
    return false;
  }
  return true;
}
__device__ bool hot_check(HotState& h, unsigned long long seq, int what, uint32_t kd = 0, int lm = 0, int q = 0,
                          int rem = 0) {
  hot_drain();
  if (!hot_check_lists(h, seq, what)) {
    if (lane_id() == 0)
      printf("HOTCHECK after record s=%u seq=%llu kind=%u lm=%d q=%d rem=%d nA=%d nB=%d kA=%d\n", h.gs, seq, kd, lm, q,
             rem, h.A.n, h.B.n, h.A.k);
    return false;
  }
  return true;
}
#define HOT_CHECK(what, seq_, ...)                                     \
  if (!hot_check(h, (seq_), (what), ##__VA_ARGS__)) {                  \
    if (lane == 0) atomicOr(h.err, ERR_INCONSISTENT);                  \
    ok = false;                                                        \
    break;                                                             \
  }
#else
#define HOT_CHECK(what, seq_, ...)
#endif

// Diagnostic stamps of the hot loop (-DME_STAMPS): cycles in registers, into the WaveCtx at the end
// (fetch: block starts; sweep: takes; rest: rests; cancel: generic records; result: results).
#ifdef ME_STAMPS
#define HS_DECL unsigned long long hs_[PH_N] = {}, hst_ = stamp_now()
#define HS(ph)                          \
  do {                                  \
    const unsigned long long n_ = stamp_now(); \
    hs_[ph] += n_ - hst_;               \
    hst_ = n_;                          \
  } while (0)
#define HS_COUNT(ct) (hs_[ct] += 1)
#define HS_FLUSH(c)                                    \
  for (int p_ = 0; p_ < PH_N; ++p_) (c).st[p_] += hs_[p_]; \
  for (int e_ = 0; e_ < 4; ++e_) (c).st[PH_SW_WINDOW + e_] += h.cyc[e_]; \
  for (int e_ = 0; e_ < 4; ++e_) (c).st[WK_GET + e_] += h.cyc[4 + e_]
#else
#define HS_DECL
#define HS(ph) ((void)0)
#define HS_COUNT(ct) ((void)0)
#define HS_FLUSH(c) ((void)0)
#endif

// Records [lo, hi) of the hot symbol in seq order, blocks of 64.
__device__ __forceinline__ void match_records_hot(HotState& h, WaveCtx& c, const BatchDev& bt, uint32_t lo,
                                                  uint32_t hi) {
  const int lane = lane_id();
  HS_DECL;
#ifdef ME_STAMPS
  for (int e_ = 0; e_ < 8; ++e_) h.ev[e_] = h.cyc[e_] = 0;
#endif
  const int L = (int)h.L;
  h.nfs = 0;
  h.fstk = NIL;
  h.rlvl = -1;
  h.A.k = 1;  // asks
  h.B.k = 0;  // bids
  hot_occ_load(h);
  hot_rebuild<1>(h, h.A, rli32(c.ba, 0));
  hot_rebuild<0>(h, h.B, L - 1 - rli32(c.bb, 0));
  bool ok = true, handed = false;
  for (uint32_t blk = lo; blk < hi && ok && !handed; blk += 64) {
    c.recs_left = hi - blk;
    HS(PH_RESULT);
    if (h.nfs < HOT_STACK_LOW) {
      hot_topup(h, c);
      HS_COUNT(CT_WALK);
    }
    const uint32_t j = blk + (uint32_t)lane;
    const bool v = j < hi;
    const uint32_t oi = v ? bt.perm[j] : 0u;
    const unsigned long long oseq = v ? bt.seq[oi] : 0ull;
    const long long opx = v ? bt.px[oi] : 0ll;
    const int oq = v ? bt.qty[oi] : 0;
    const uint32_t okd = v ? (uint32_t)bt.kind[oi] : 0u;
    const uint32_t cnt = min(64u, hi - blk);
    const uint32_t side = okd & 3u;
    const bool market = (okd >> 2) & 1u, cancel = (okd >> 3) & 1u;
    const bool good = v && !cancel && oq > 0 && (side == ME_SIDE_BUY || side == ME_SIDE_SELL) && oseq != 0ull;
    // which records the lists take (vector form; again after a generic record moved the window):
    // cancels, LIMITs outside the window and takers while the side they cross has far levels are generic
    unsigned long long fastm;
    auto classify = [&]() {
      const unsigned long long off = (unsigned long long)opx - (unsigned long long)h.base;
      const bool inw = off < (unsigned long long)L;
      const bool farx = (side == ME_SIDE_BUY ? h.nfar1 : h.nfar0) != 0u;
      const bool fast = good && (market || inw) && !farx;
      h.rlvl = fast && !market ? (int)off : -1;
      fastm = __ballot(fast);
    };
    classify();
    if (h.A.n < HT / 2 && h.A.more) {
      hot_drain();
      hot_rebuild<1>(h, h.A, rli32(h.A.m, h.A.f));
      HS_COUNT(CT_MISS);
    }
    if (h.B.n < HT / 2 && h.B.more) {
      hot_drain();
      hot_rebuild<0>(h, h.B, rli32(h.B.m, h.B.f));
      HS_COUNT(CT_MISS);
    }
    hot_prefetch(h);
    __builtin_amdgcn_s_waitcnt(0);
    HOT_CHECK(0, 0ull);
    HS(PH_FETCH);
    ResultLanes R;
    R.filled = R.remaining = 0;
    R.nfill = R.fstart = R.st = 0;
    uint32_t k = 0;
    for (; k < cnt; ++k) {
      HMARK("record-start");
      const unsigned long long seq = rl64(oseq, (int)k);
      const int q = rli32(oq, (int)k);
      const uint32_t kd = rl32(okd, (int)k);
      if (ME_UNLIKELY(!((fastm >> k) & 1ull))) {
        // a record the lists do not cover (a cancel, a price outside the window, a taker while far
        // levels exist, a reject): the symbol's records from here on go to k_match_hot_cont, the
        // generic record loop, behind this wave (no generic code on the hot loop's paths)
        HMARK("record-generic");
        HS_COUNT(CT_EVICT);
        if (lane == 0) {
          const uint32_t idx = atomicAdd(c.bk.hcount + 1, 1u);
          Handoff ho{};
          ho.s = c.s;
          ho.pos = blk + k;
          ho.nsg = hi;
          ho.wptr = (uint32_t)h.wptr;
          ho.wend = (uint32_t)(h.wptr >> 32);
          c.bk.hand[c.bk.S + idx] = ho;
        }
        handed = true;
        break;
      }
      HMARK("record-fast");
      const bool buy = (kd & 3u) == ME_SIDE_BUY;
      const bool mkt = (kd >> 2) & 1u;
      const int lm = mkt ? 0 : rli32(h.rlvl, (int)k);  // the LIMIT's window level
      const unsigned long long fstart = h.wptr;
      uint32_t rem = (uint32_t)q;
      HS_COUNT(CT_FAST);
      // A holds the asks, B the bids: a BUY takes from A and rests on B, a SELL the other way round
      // (one instance of the code per side: no list state moves between registers)
      bool rested = true;
      if (buy) {
        hot_take<1>(h, h.A, mkt ? L - 1 : lm, rem, seq);
        HS(PH_SWEEP);
        if (!mkt && rem) rested = hot_rest<0>(h, c, h.B, L - 1 - lm, lm, seq, (int)rem, (int)k);
      } else {
        hot_take<0>(h, h.B, mkt ? L - 1 : L - 1 - lm, rem, seq);
        HS(PH_SWEEP);
        if (!mkt && rem) rested = hot_rest<1>(h, c, h.A, lm, lm, seq, (int)rem, (int)k);
      }
      if (ME_UNLIKELY(!rested)) {
        ok = false;  // the chunk pool is exhausted (sticky error word from alloc_chunk)
        break;
      }
      const int filled = q - (int)rem;
      const uint32_t nfill = (uint32_t)(h.wptr - fstart);
      uint8_t stt;
      if (mkt)
        stt = rem == 0 ? ME_ST_FILLED : ME_ST_CANCELED;
      else
        stt = rem == 0 ? ME_ST_FILLED : (filled > 0 ? ME_ST_PARTIALLY_FILLED : ME_ST_NEW);
      HS(PH_REST);
      HMARK("record-result");
      put_result(R, k, filled, (int)rem, nfill, stt, ME_RJ_NONE, fstart);
      HOT_CHECK(1, seq, kd, lm, q, (int)rem);
    }
    store_results(bt, R, v && (uint32_t)lane < k, oi);
  }
  HS(PH_RESULT);
  HS_FLUSH(c);
  // the generic state for wave_end: exact best levels, the stack's chunks back onto the free list
  hot_sync_in(h, c);
  while (h.nfs) {
    h.nfs -= 1;
    hot_free_slow(&c, rl32(h.fstk, (int)h.nfs));
  }
  while (c.bump_cur < c.bump_end) hot_free_slow(&c, rl32(c.bump_ids, (int)c.bump_cur++));
}

// The hot symbols of a launch (at least hot_min records in the batch) into bk.hand[] = {s, pos = lo,
// nsg = hi}: one thread per symbol over the run table. k_match skips them; k_match_hot, on a second
// stream, runs them concurrently.
// Without a run table (a multi-pass sort), one thread per grouped position: a run start whose run
// reaches hot_min records finds the run's end by a binary search.
__global__ __launch_bounds__(256) void k_hot_pick(BookDev bk, BatchDev bt) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  uint32_t s, lo, hi;
  if (bt.bin_start) {
    s = t;
    if (s >= bk.S) return;
    lo = bt.bin_start[s];
    hi = bt.bin_start[s + 1];
  } else {
    const uint32_t n = bt.n;
    if (t >= n) return;
    s = bt.skeys[t];
    if (s >= bk.S || (t > 0 && bt.skeys[t - 1] == s)) return;  // not a run start (or the reject bin)
    if (t + bk.hot_min > n || bt.skeys[t + bk.hot_min - 1] != s) return;  // too short to be hot
    uint32_t a = t + bk.hot_min, b = n;  // the run ends in [a - 1, b): first position with a larger key
    while (a < b) {
      const uint32_t m = (a + b) / 2;
      if (bt.skeys[m] == s)
        a = m + 1;
      else
        b = m;
    }
    lo = t;
    hi = a;
  }
  if (hi - lo < bk.hot_min) return;
  const uint32_t idx = atomicAdd(bk.hcount, 1u);
  Handoff ho{};
  ho.s = s;
  ho.pos = lo;
  ho.nsg = hi;
  bk.hand[idx] = ho;
}

// One wave per hot symbol of the launch (k_hot_pick listed them: bk.hand[i] = {s, pos = lo, nsg = hi}).
__global__ __launch_bounds__(64) void k_match_hot(BookDev bk, BatchDev bt) {
  __shared__ HotLds H;
  const uint32_t nh = min(*(volatile uint32_t*)bk.hcount, bk.S);
  for (uint32_t i = blockIdx.x; i < nh; i += gridDim.x) {
    const Handoff ho = bk.hand[i];
    const uint32_t s = rl32(ho.s, 0), lo = rl32(ho.pos, 0), hi = rl32(ho.nsg, 0);
    WaveCtx c;
#ifdef ME_STAMPS
    for (int p = 0; p < PH_N; ++p) c.st[p] = 0;
    STAMP_MARK(c);
#endif
    c.lad.L = bk.L;
    c.lad.Lwords = bk.Lwords;
    c.lad.lv = bk.levels + (size_t)s * bk.L;
    c.lad.occ = bk.occ + (size_t)s * bk.Lwords;
    c.lad.tend = bk.tend + (size_t)s * bk.L;
    c.cache = nullptr;
    c.cmask = 0;
    if (!wave_begin(c, bk, bt, s, lo, hi)) return;
    HotState h;
    h.chunks = (gptr<Chunk>)vptr(bk.chunks);
    h.loc = (gptr<uint32_t>)vptr(bk.loc);
    h.scratch = (gptr<me_fill>)vptr(bt.scratch);
    h.lv = (gptr<Level>)vptr(c.lad.lv);
    h.occ = (gptr<unsigned long long>)vptr(c.lad.occ);
    h.tend = (gptr<uint8_t>)vptr(c.lad.tend);
    h.err = (gptr<uint32_t>)vptr(bk.err);
    h.rmask = bk.ring_mask;
    h.nchunks = bk.nchunks;
    h.L = bk.L;
    h.W = bk.Lwords;
    h.gs = rl32(c.gs, 0);
    h.H = &H;
    wave_to_hot(c, h);
    match_records_hot(h, c, bt, lo, hi);
    wave_end(c);
  }
}
// The rest of a hot symbol's records after the first one k_match_hot does not cover: the generic
// record loop (k_match's), on the same stream right after k_match_hot; hand-off i is bk.hand[S + i].
__global__ __launch_bounds__(64) void k_match_hot_cont(BookDev bk, BatchDev bt) {
  const uint32_t nh = min(*(volatile uint32_t*)(bk.hcount + 1), bk.S);
  for (uint32_t i = blockIdx.x; i < nh; i += gridDim.x) {
    const Handoff ho = bk.hand[bk.S + i];
    const uint32_t s = rl32(ho.s, 0), pos = rl32(ho.pos, 0), hi = rl32(ho.nsg, 0);
    const unsigned long long w = ((unsigned long long)rl32(ho.wend, 0) << 32) | rl32(ho.wptr, 0);
    WaveCtx c;
#ifdef ME_STAMPS
    for (int p = 0; p < PH_N; ++p) c.st[p] = 0;
    STAMP_MARK(c);
#endif
    c.lad.L = bk.L;
    c.lad.Lwords = bk.Lwords;
    c.lad.lv = bk.levels + (size_t)s * bk.L;
    c.lad.occ = bk.occ + (size_t)s * bk.Lwords;
    c.lad.tend = bk.tend + (size_t)s * bk.L;
    c.cache = nullptr;
    c.cmask = 0;
    if (!wave_begin(c, bk, bt, s, pos, hi, w)) return;
    match_records(c, bt, pos, hi);
    wave_end(c);
  }
}

// ---- seq ring horizon ---------------------------------------------------------
// Runs before every match launch. The ring holds loc[seq & (R - 1)]; a rest of seq y overwrites the
// entry of y - R. Every live order at or above the horizon has its entry, every older live order is
// in the old-order table, so the ring is safe while every seq matched stays below horizon + R. When
// the next group's largest seq would reach that, this kernel moves the horizon to the group's first
// seq and rebuilds the old-order table from the chunk pool (all live orders, which are older than
// the group since seqs ascend), in a new epoch: entries of earlier epochs read as empty. Every
// workgroup makes the same decision from state[in] and the group's first / last seqs.
struct SeqGroup {
  const uint64_t* seq[ME_GMAX];
  const uint8_t* kind[ME_GMAX];  // the first record's kind: a cancel may repeat the previous seq
  uint32_t n[ME_GMAX];
  uint32_t ng;
  uint32_t in;  // state index read; the kernel writes state[in ^ 1]
  uint32_t launch;  // match launches enqueued before this group's (all finished when this runs)
  uint32_t recs;    // records of the group (each draws at most one chunk from the pool)
};

// Chunk-pool reclamation (me_layout.hpp cp_id), by k_seq_sweep's workgroups ahead of a launch
// group when the pool's high-water mark hw plus what the group can draw (<= one chunk per record and one
// reservation block per wave that has none left) could pass the pool. Between launches a chunk is free iff
// all its quantities are 0 (every linked chunk holds a live order; a freed chunk is zeroed in HBM before it
// is listed anywhere), so one pass over [0, hw) finds every free chunk, wherever it is parked — symbols' free
// lists, fcache rows, the last reclamation's unused tail. Every symbol's free list and fcache row are
// dropped, the chunks found become the list allocation numbers map to first, and the last workgroup
// (ticket) publishes it: {nrecl = found, fresh = hw}, allocation counter 0. Afterwards chunks held = chunks
// in use <= resting orders, so max_resting + the group's reservation slack always suffices.
__device__ void chunk_reclaim(const BookDev& bk, uint32_t hw) {
  const int lane = lane_id();
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < bk.S; i += gridDim.x * blockDim.x) {
    bk.sym[i].free_head = NIL;
    bk.sym[i].nfree = 0;
  }
  const uint32_t nwv = blockDim.x >> 6;
  const uint32_t wid = blockIdx.x * nwv + (threadIdx.x >> 6), nw = gridDim.x * nwv;
  for (uint32_t c0 = wid * 64u; c0 < hw; c0 += nw * 64u) {
    const uint32_t c = c0 + (uint32_t)lane;
    bool fr = false;
    if (c < hw) {
      const int4* q = reinterpret_cast<const int4*>(bk.chunks[c].qty);
      const int4 a = q[0], b = q[1], d = q[2], e = q[3];
      fr = ((a.x | a.y | a.z | a.w) | (b.x | b.y | b.z | b.w) | (d.x | d.y | d.z | d.w) | (e.x | e.y | e.z | e.w)) == 0;
    }
    const unsigned long long m = __ballot(fr);
    uint32_t off = 0;
    if (lane == 0 && m) off = atomicAdd(bk.cpool + CP_FOUND, (uint32_t)__popcll(m));
    off = rl32(off, 0);
    if (fr) bk.recl[off + (uint32_t)__popcll(m & lanemask_lt())] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const uint32_t t = atomicAdd(bk.cpool + CP_TICKET, 1u);
    if (t == gridDim.x - 1u) {  // every workgroup has listed its chunks
      const uint32_t found = __hip_atomic_load(bk.cpool + CP_FOUND, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      bk.cpool[CP_NRECL] = found;
      bk.cpool[CP_FRESH] = hw;
      bk.cpool[CP_FOUND] = 0;
      bk.cpool[CP_TICKET] = 0;
      *bk.chunk_top = 0;
      bk.stats[ST_CHUNK_GC] += 1ull;
      __threadfence();
    }
  }
}

// The far arena's copying collection (me_far.hpp), by k_seq_sweep's workgroups when the active half's top
// has passed far_gc_at: no launch allocates while this kernel runs, so every workgroup reads the same
// {half, top} and takes the same decision. Each wave takes sides in turn; a side living in the active half
// moves to the inline region when it fits, else to nextpow2(n) (>= 2 x inline) entries of the other half.
// The last workgroup to finish (ticket) swaps the halves and empties the old one.
__device__ void far_collect(const BookDev& bk) {
  unsigned long long* ctl = bk.far_ctl;
  const unsigned long long h = __hip_atomic_load(ctl + FC_HALF, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1ull;
  const unsigned long long top = __hip_atomic_load(ctl + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (top <= bk.far_gc_at) return;
  const unsigned long long nh = h ^ 1ull;
  const int lane = lane_id();
  const uint32_t nwv = blockDim.x >> 6;
  const uint32_t wid = blockIdx.x * nwv + (threadIdx.x >> 6), nw = gridDim.x * nwv;
  const unsigned long long c0 = bk.fcap, inl = 2ull * bk.S * c0;
  for (uint32_t i = wid; i < 2u * bk.S; i += nw) {
    const unsigned long long off = rl64(__hip_atomic_load(&bk.fdir[i].off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), 0);
    if (off < inl) continue;  // inline: nothing to move
    const uint32_t n = rl32(bk.sym[i >> 1].nfar[i & 1u], 0);
    unsigned long long o = i * c0, cap = c0;
    if (n > c0) {
      cap = 2ull * c0;
      while (cap < n) cap <<= 1;
      unsigned long long t = 0;
      if (lane == 0) t = atomicAdd(ctl + nh, cap);
      o = inl + nh * bk.far_half + rl64(t, 0);
      if (rl64(t, 0) + cap > bk.far_half) {  // impossible by the bound (me_far.hpp)
        if (lane == 0) atomicOr(bk.err, ERR_FAR_OOM);
        continue;
      }
    }
    const FarLevel* src = bk.far + off;
    FarLevel* dst = bk.far + o;
    for (uint32_t j = (uint32_t)lane; j < n; j += 64) dst[j] = src[j];
    if (lane == 0) {
      FarDir d;
      d.off = o;
      d.cap = (uint32_t)cap;
      d.pad = 0;
      bk.fdir[i] = d;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const uint32_t t = atomicAdd((uint32_t*)(ctl + FC_TICKET), 1u);
    if (t == gridDim.x - 1u) {  // every workgroup has moved its sides
      ctl[h] = 0;
      ctl[FC_HALF] = nh;
      ctl[FC_TICKET] = 0;
      bk.stats[ST_FAR_GC] += 1ull;
      __threadfence();
    }
  }
}

__global__ __launch_bounds__(256) void k_seq_sweep(BookDev bk, SeqGroup sg) {
  const SeqState st = bk.sq[sg.in];
  // the pool's state as the previous launches left it (only the last workgroup of a reclamation changes it,
  // after every workgroup has read it)
  const CPool cp = cp_read(bk.cpool);
  const uint32_t hw = cp_hw(cp, __builtin_amdgcn_readfirstlane(*bk.chunk_top), bk.nchunks);
  const unsigned long long gmin = sg.seq[0][0];
  const unsigned long long gmax = sg.seq[sg.ng - 1][sg.n[sg.ng - 1] - 1];
  const unsigned long long R = bk.ring_mask + 1ull;
  const bool need = gmax - st.horizon >= R;
  const uint32_t epoch = need ? st.epoch + 1u : st.epoch;
  bool order_ok = true;
  if (blockIdx.x == 0 && threadIdx.x < 64) {
    // the batch boundaries of the group, one lane each (one thread's loop waited ~0.4 us per batch:
    // 11.9 -> 4.7 us for config 2's 20-batch group, profiles/r4/ev)
    const uint32_t l = threadIdx.x;
    if (l == 0) order_ok = st.last == 0ull || seq_follows(st.last, gmin, sg.kind[0][0]);
    for (uint32_t g = l; g + 1 < sg.ng; g += 64)
      order_ok &= seq_follows(sg.seq[g][sg.n[g] - 1], sg.seq[g + 1][0], sg.kind[g + 1][0]);
    order_ok = __ballot(!order_ok) == 0ull;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    uint32_t bits = 0;
    if (!order_ok) bits |= ERR_SEQ_ORDER;
    if (gmax - gmin >= R) bits |= ERR_SEQ_SPAN;
    if (bits) atomicOr(bk.err, bits);
    SeqState o;
    o.horizon = need ? gmin : st.horizon;
    o.last = gmax > st.last ? gmax : st.last;
    o.epoch = epoch;
    o.pad[0] = o.pad[1] = o.pad[2] = 0;
    bk.sq[sg.in ^ 1u] = o;
    bk.stats[ST_LAUNCH] = sg.launch;
    bk.hcount[0] = 0;  // the match launch after this one hands symbols off from 0 ...
    bk.hcount[1] = 0;  // ... and continues them (k_match_hot_cont) from 0
    if (bk.agg_ctr)
      for (uint32_t k = 0; k < AC_N; ++k) bk.agg_ctr[k] = 0;  // the aggregate path's pools (me_agg.hip)
    if (bk.pub) {  // resting orders after sg.launch match launches, for the host's admission bound
      const unsigned long long r = bk.stats[ST_RESTING];
      *bk.pub = ((unsigned long long)sg.launch << 32) | (r < 0xFFFFFFFFull ? r : 0xFFFFFFFFull);
      // and the hand-offs so far (the engine's grouped-aggregate policy, me_engine.cpp)
      const unsigned long long h = bk.stats[ST_HANDOFFS];
      bk.pub[1] = ((unsigned long long)sg.launch << 32) | (h < 0xFFFFFFFFull ? h : 0xFFFFFFFFull);
    }
  }
  far_collect(bk);
  if ((unsigned long long)hw + sg.recs + 2ull * bk.S + 64ull > bk.nchunks) chunk_reclaim(bk, hw);
  if (!need) return;
  const size_t slots = (size_t)hw * ME_C;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < slots; i += (size_t)gridDim.x * blockDim.x) {
    if (cq_at(bk.chunks, i) <= 0) continue;
    const unsigned long long q = cs_at(bk.chunks, i);
    const unsigned long long want = ((unsigned long long)i << 32) | epoch;  // {epoch, slot}
    unsigned long long h = old_hash(q) & bk.old_mask;
    bool placed = false;
    for (unsigned long long p = 0; p <= bk.old_mask && !placed; ++p, h = (h + 1) & bk.old_mask) {
      unsigned long long* w = reinterpret_cast<unsigned long long*>(&bk.old[h]);
      unsigned long long cur = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      while ((uint32_t)cur != epoch) {  // empty in this epoch: claim it
        const unsigned long long prev = atomicCAS(w, cur, want);
        if (prev == cur) {
          bk.old[h].seq = q;
          placed = true;
          break;
        }
        cur = prev;
      }
    }
    if (!placed) atomicOr(bk.err, ERR_OLD_OOM);
  }
}

// ------------------------------------------------------------------ tape compaction
// Block b owns records [b*1024, +1024). Tape offset of record i = sum of fills of records < i
// (batch order == seq order). Fills are then copied scratch -> tape with consecutive threads
// writing consecutive 32-B records (each thread finds its record by binary search in LDS).
__global__ __launch_bounds__(256) void k_tape_compact(const uint32_t* __restrict__ tile_sum, uint32_t ntiles,
                                                      me_order_result* res, const uint32_t* __restrict__ fstart,
                                                      uint32_t n, const me_fill* __restrict__ scratch,
                                                      me_fill* __restrict__ tape, unsigned long long tape_cap,
                                                      unsigned long long* tape_count, unsigned long long* fills_acc,
                                                      uint32_t* err, me_order_result* hres, uint32_t* err_out) {
  // hres != nullptr: a host batch (see AuxTape): tape_cap is soft, final results copied to hres
  __shared__ uint32_t off[TILE_TAPE + 1];
  __shared__ unsigned long long red[4];
  __shared__ uint32_t wsum[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t b = blockIdx.x;
  unsigned long long acc = 0;
  for (uint32_t t = tid; t < b; t += 256) acc += tile_sum[t];
  for (int d = 32; d >= 1; d >>= 1) acc += __shfl_xor(acc, d, 64);
  if (lane == 0) red[w] = acc;
  const uint32_t r0 = b * TILE_TAPE;
  const uint32_t cnt = min((uint32_t)TILE_TAPE, n - r0);
  for (uint32_t k = tid; k < cnt; k += 256) off[k] = res[r0 + k].fill_count;
  __syncthreads();
  const unsigned long long base = red[0] + red[1] + red[2] + red[3];
  const uint32_t total = block_excl_scan_lds(off, cnt, wsum);
  if (tid == 0) off[cnt] = total;
  for (uint32_t k = tid; k < cnt; k += 256) {
    res[r0 + k].tape_offset = (uint32_t)(base + off[k]);
    if (hres) {
      me_order_result r = res[r0 + k];
      r.tape_offset = (uint32_t)(base + off[k]);
      hres[r0 + k] = r;
    }
  }
  __syncthreads();
  if (!hres && base + total > tape_cap) {
    if (tid == 0) atomicOr(err, ERR_SCRATCH_OOM);
    return;
  }
  const uint32_t lim = base >= tape_cap ? 0u : (uint32_t)min((unsigned long long)total, tape_cap - base);
  for (uint32_t f = tid; f < lim; f += 256) {
    // last k with off[k] <= f
    uint32_t lo = 0, hi = cnt;  // off[lo] <= f < off[hi]
    while (hi - lo > 1) {
      uint32_t mid = (lo + hi) >> 1;
      if (off[mid] <= f)
        lo = mid;
      else
        hi = mid;
    }
    const uint32_t src = fstart[r0 + lo] + (f - off[lo]);
    tape[base + f] = scratch[src];
  }
  if (b == gridDim.x - 1 && tid == 0) {
    *tape_count = base + total;
    atomicAdd(fills_acc, base + total);
    if (err_out) *err_out = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// The fills of a host batch past its slot's soft tape cap (me_collect): record i's fills sit at
// scratch[fstart[i] ..) and belong at tape[res[i].tape_offset ..); those at or past `cap` are copied
// to spill[index - cap].
__global__ __launch_bounds__(256) void k_tape_spill(const me_order_result* __restrict__ res,
                                                    const uint32_t* __restrict__ fstart, uint32_t n,
                                                    const me_fill* __restrict__ scratch, unsigned long long cap,
                                                    me_fill* __restrict__ spill) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const me_order_result r = res[i];
  for (uint32_t q = 0; q < r.fill_count; ++q) {
    const unsigned long long t = (unsigned long long)r.tape_offset + q;
    if (t >= cap) spill[t - cap] = scratch[fstart[i] + q];
  }
}

__global__ void k_init_levels(Level* lv, size_t count) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x) {
    Level o;
    o.total = 0;
    o.head = NIL;
    o.tail = NIL;
    lv[i] = o;
  }
}

}  // namespace me

// ------------------------------------------------------------------ launch wrappers (host)
namespace me {

// tile = records per sort workgroup: >= 1024 and large enough that ntiles <= 256
uint32_t sort_tile(uint32_t n) {
  uint32_t t = 1024;
  while ((n + t - 1) / t > 256) t <<= 1;
  return t;
}

hipError_t launch_sort_pass(hipStream_t st, const uint32_t* keys_in, const uint32_t* idx_in, uint32_t n,
                            uint32_t clamp_key, int shift, int dbits, uint32_t* hist, uint32_t* tot,
                            uint32_t* keys_out, uint32_t* idx_out, uint32_t* zero_buf,
                            uint32_t zero_words, unsigned long long* scratch_top, uint32_t* bin_start,
                            const uint64_t* seq, const uint8_t* kind, uint32_t* err) {
  SortPass p;
  p.shift = (uint32_t)shift;
  p.mask = (1u << dbits) - 1u;
  p.nbins = min(1u << dbits, (clamp_key >> shift) + 1u);
  p.tile = sort_tile(n);
  p.ntiles = (n + p.tile - 1) / p.tile;
  p.clamp = clamp_key;
  hipLaunchKernelGGL(k_sort_hist, dim3(p.ntiles), dim3(256), 0, st, keys_in, n, p, hist, zero_buf, zero_words,
                     scratch_top, seq, kind, err);
  hipLaunchKernelGGL(k_sort_colscan, dim3((p.nbins + 63) / 64), dim3(64), 0, st, hist, tot, p.nbins, p.ntiles);
  hipLaunchKernelGGL(k_sort_scatter, dim3(p.ntiles), dim3(256), 0, st, keys_in, idx_in, n, p, (uint32_t)dbits, hist,
                     tot, keys_out, idx_out, bin_start);
  return hipGetLastError();
}

namespace rc64 {
hipError_t launch_match_reg(hipStream_t st, const BookDev& bk, const BatchDev* bt, uint32_t ng, const AuxDev& ax,
                            hipEvent_t ev0, hipEvent_t ev1);
hipError_t launch_match_reg_cont(hipStream_t st, const BookDev& bk, const BatchDev* bt, uint32_t ng, hipEvent_t ev1);
}
namespace rc128 {
hipError_t launch_match_reg(hipStream_t st, const BookDev& bk, const BatchDev* bt, uint32_t ng, const AuxDev& ax,
                            hipEvent_t ev0, hipEvent_t ev1);
hipError_t launch_match_reg_cont(hipStream_t st, const BookDev& bk, const BatchDev* bt, uint32_t ng, hipEvent_t ev1);
}
hipError_t launch_agg_group(hipStream_t st, const BookDev& bk, const BatchDev* bt, uint32_t ng, const AggDev& ag);  // me_agg.hip
// The register-ladder launch (me_match_reg.hip, two builds): one head-cache entry per level while one
// workgroup per CU covers the symbols (rc128), 64 shared entries and two workgroups per CU beyond
// that (rc64). ax.nwg is the CU count (0: assume 256).
#ifndef ME_SIDE_XSEQ
#define ME_SIDE_XSEQ 1
#endif
hipError_t launch_match_reg(hipStream_t st, const BookDev& bk, const BatchDev* bt, uint32_t ng, const AuxDev& ax,
                            hipEvent_t ev0, hipEvent_t ev1, const HotLaunch* hot) {
  constexpr uint32_t kWaves = 4;  // matching waves per workgroup (me_match_reg.hip REG_WAVES)
  const uint32_t waves = ng && bt[0].bcnt ? bk.S : bk.S + 1;
  const uint32_t wgs = (waves + kWaves - 1) / kWaves;
  const uint32_t ncu = ax.nwg ? ax.nwg : 256u;
  const bool big = wgs > ncu;
  if (hot && hot->agg_reg && ng && bt[0].bcnt) {
    // the group through the aggregate path: side jobs (k_side), walk + per-level kernels, continuation
    hipError_t e;
    const bool side = ax.nb || ax.nt, fork = side && hot->sst;
    if (fork) {
      // the side jobs beside the group: the next group's buckets and the tapes of the group before touch
      // nothing this group's walk, per-level launch or continuation reads or writes (other bucket and
      // output sets), and everything they read was final when the fork was recorded
      if ((e = hipEventRecord(hot->sfork, st)) != hipSuccess || (e = hipStreamWaitEvent(hot->sst, hot->sfork, 0)) != hipSuccess)
        return e;
      AuxDev sx = ax;
      sx.xseq = ME_SIDE_XSEQ;  // off the critical path: bucket the batches per XCD in turn (fewer partial lines)
      e = big ? rc64::launch_match_reg(hot->sst, bk, bt, 0, sx, nullptr, nullptr)
              : rc128::launch_match_reg(hot->sst, bk, bt, 0, sx, nullptr, nullptr);
      if (e != hipSuccess || (e = hipEventRecord(hot->sjoin, hot->sst)) != hipSuccess) return e;
      e = ev0 ? hipEventRecord(ev0, st) : hipSuccess;
    } else if (side) {
      e = big ? rc64::launch_match_reg(st, bk, bt, 0, ax, ev0, nullptr)
              : rc128::launch_match_reg(st, bk, bt, 0, ax, ev0, nullptr);
    } else {
      e = ev0 ? hipEventRecord(ev0, st) : hipSuccess;
    }
    if (e != hipSuccess) return e;
    if ((e = launch_agg_group(st, bk, bt, ng, hot->ag)) != hipSuccess) return e;
    e = big ? rc64::launch_match_reg_cont(st, bk, bt, ng, ev1) : rc128::launch_match_reg_cont(st, bk, bt, ng, ev1);
    if (e != hipSuccess) return e;
    // the next launch (its walk reads the buckets made here) and every completion event recorded on st
    // after this (host batches' tapes) wait for the side jobs
    return fork ? hipStreamWaitEvent(st, hot->sjoin, 0) : hipSuccess;
  }
  // a launch with no match job (the pipeline's fill and drain): its bucket units too per XCD in turn (one
  // batch's buckets per L2 at a time; driver shape +1 %, profiles/r5/fx); ME_FILL_XSEQ=0: all at once
  static const bool fill_xseq = [] {
    const char* e = getenv("ME_FILL_XSEQ");
    return !e || atoi(e) != 0;
  }();
  AuxDev axx = ax;
  if (ng == 0 && fill_xseq) axx.xseq = 1u;
  return big ? rc64::launch_match_reg(st, bk, bt, ng, axx, ev0, ev1)
             : rc128::launch_match_reg(st, bk, bt, ng, axx, ev0, ev1);
}

// ev0 / ev1 (optional, timing): the launch records the kernel's own start and end
// (hipExtLaunchKernelGGL), so timing adds no marker packet — and no gap — to the stream.
// hot (deep windows with bk.hot_min): the stream and fork / join events k_match_hot runs with, beside
// k_match (same symbols never meet: k_match skips what k_hot_pick listed).
hipError_t launch_agg(hipStream_t hs, const BookDev& bk, const BatchDev& bt, const AggDev& ag);  // me_agg.hip

hipError_t launch_match(hipStream_t st, const BookDev& bk, const BatchDev& bt, hipEvent_t ev0, hipEvent_t ev1,
                        const HotLaunch& hot) {
  const uint32_t waves = bk.S + 1;
  const dim3 grid((waves + 3) / 4), block(256);
  if (bk.L <= 128) return launch_match_reg(st, bk, &bt, 1u, AuxDev{}, ev0, ev1, nullptr);
  const bool lds = bk.L <= LDS_MAX_LEVELS;
  // hot symbols: the aggregate path (windows up to AGG_MAX_L) or k_match_hot (HBM ladders up to
  // HOT_MAX_WORDS * 64 levels), on the hot stream beside k_match
  const bool hot_on = bk.hot_min && hot.st &&
                      (hot.agg ? bk.L <= AGG_MAX_L : (!lds && bk.L <= HOT_MAX_WORDS * 64u));
  if (!hot_on) {
    BookDev b2 = bk;
    b2.hot_min = 0;
    if (lds)
      hipExtLaunchKernelGGL(k_match<LAD_LDS>, grid, block, 4 * lds_wave_bytes(bk.L), st, ev0, ev1, 0, b2, bt);
    else
      hipExtLaunchKernelGGL(k_match<LAD_HBM>, grid, block, 0, st, ev0, ev1, 0, b2, bt);
    return hipGetLastError();
  }
  // hcount was zeroed by k_seq_sweep; the pick starts the timed span, the join ends it
  const uint32_t pick = bt.bin_start ? bk.S : bt.n;
  hipExtLaunchKernelGGL(k_hot_pick, dim3((pick + 255) / 256), dim3(256), 0, st, ev0, nullptr, 0, bk, bt);
  hipError_t e;
  if ((e = hipEventRecord(hot.fork, st)) != hipSuccess || (e = hipStreamWaitEvent(hot.st, hot.fork, 0)) != hipSuccess)
    return e;
  if (hot.agg) {
    if ((e = launch_agg(hot.st, bk, bt, hot.ag)) != hipSuccess) return e;
  } else {
    hipLaunchKernelGGL(k_match_hot, dim3(64), dim3(64), 0, hot.st, bk, bt);
  }
  hipLaunchKernelGGL(k_match_hot_cont, dim3(64), dim3(64), 0, hot.st, bk, bt);
  if ((e = hipEventRecord(hot.join, hot.st)) != hipSuccess) return e;
  if (lds)
    hipLaunchKernelGGL(k_match<LAD_LDS>, grid, block, 4 * lds_wave_bytes(bk.L), st, bk, bt);
  else
    hipLaunchKernelGGL(k_match<LAD_HBM>, grid, block, 0, st, bk, bt);
  if ((e = hipStreamWaitEvent(st, hot.join, 0)) != hipSuccess) return e;
  if (ev1 && (e = hipEventRecord(ev1, st)) != hipSuccess) return e;
  return hipGetLastError();
}

// The seq-ring horizon check (and, when due, the old-order table rebuild) ahead of a match launch
// over batches seq[0..ng) (n[g] > 0 each). Reads state in_idx, writes state in_idx ^ 1.
hipError_t launch_seq_sweep(hipStream_t st, const BookDev& bk, const uint64_t* const* seq, const uint8_t* const* kind,
                            const uint32_t* n, uint32_t ng, uint32_t in_idx, uint32_t grid, uint32_t launch) {
  if (ng == 0 || ng > (uint32_t)ME_GMAX) return hipErrorInvalidValue;
  SeqGroup sg{};
  for (uint32_t g = 0; g < ng; ++g) {
    if (!n[g]) return hipErrorInvalidValue;
    sg.seq[g] = seq[g];
    sg.kind[g] = kind[g];
    sg.n[g] = n[g];
  }
  sg.ng = ng;
  sg.in = in_idx;
  sg.launch = launch;
  for (uint32_t g = 0; g < ng; ++g) sg.recs += n[g];
  hipLaunchKernelGGL(k_seq_sweep, dim3(grid ? grid : 1), dim3(256), 0, st, bk, sg);
  return hipGetLastError();
}

hipError_t launch_tape(hipStream_t st, const BatchDev& bt, me_fill* tape, unsigned long long tape_cap,
                       unsigned long long* tape_count, unsigned long long* fills_acc, uint32_t* err,
                       me_order_result* hres, uint32_t* err_out) {
  const uint32_t ntiles = (bt.n + TILE_TAPE - 1) / TILE_TAPE;
  hipLaunchKernelGGL(k_tape_compact, dim3(ntiles), dim3(256), 0, st, bt.tile_sum, ntiles, bt.res, bt.fstart,
                     bt.n, bt.scratch, tape, tape_cap, tape_count, fills_acc, err, hres, err_out);
  return hipGetLastError();
}

hipError_t launch_tape_spill(hipStream_t st, const me_order_result* res, const uint32_t* fstart, uint32_t n,
                             const me_fill* scratch, unsigned long long cap, me_fill* spill) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_tape_spill, dim3((n + 255) / 256), dim3(256), 0, st, res, fstart, n, scratch, cap, spill);
  return hipGetLastError();
}

__global__ void k_init_chunks(Chunk* ch, size_t count) {
  // one thread per 16-B piece of the 256-B blocks: header all-NIL, everything else zero
  const size_t pieces = count * (sizeof(Chunk) / 16);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < pieces; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = (i % (sizeof(Chunk) / 16)) == 0 ? make_uint4(NIL, NIL, NIL, NIL) : make_uint4(0, 0, 0, 0);
    reinterpret_cast<uint4*>(ch)[i] = v;
  }
}

hipError_t launch_init_chunks(hipStream_t st, Chunk* chunks, size_t count) {
  hipLaunchKernelGGL(k_init_chunks, dim3(8192), dim3(256), 0, st, chunks, count);
  return hipGetLastError();
}

hipError_t launch_init_levels(hipStream_t st, Level* levels, size_t count) {
  size_t blocks = (count + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL(k_init_levels, dim3((uint32_t)blocks), dim3(256), 0, st, levels, count);
  return hipGetLastError();
}

}  // namespace me

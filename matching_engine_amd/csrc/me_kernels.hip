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
//                                    fills go to a per-wave scratch run.
//   3. k_tape_compact                exclusive scan of per-record fill counts (batch order) and
//                                    a coalesced copy scratch -> tape ordered (taker_seq, fill#).
//
// Matching semantics are pinned by oracle/oracle_book.cpp; there is no
// reference matcher (include/engine/model.hpp is empty in julien-mrty/Matching_Engine).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

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
__global__ __launch_bounds__(256) void k_sort_hist(const uint32_t* __restrict__ keys_in, uint32_t n, SortPass p,
                                                   uint32_t* __restrict__ hist, uint32_t* zero_buf,
                                                   uint32_t zero_words, unsigned long long* scratch_top) {
  __shared__ uint32_t h[1u << MAX_DIGIT_BITS];
  for (uint32_t b = threadIdx.x; b < p.nbins; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const uint32_t t0 = blockIdx.x * p.tile;
  const uint32_t t1 = min(n, t0 + p.tile);
  for (uint32_t i = t0 + threadIdx.x; i < t1; i += blockDim.x) atomicAdd(&h[sort_digit(keys_in[i], p)], 1u);
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
// Head-chunk cache (LDS): entry (lvl & cmask) holds the FIFO head chunk of one level — its 16
// slot quantities/seqs and its next pointer — so walks and appends on top-of-book levels stay
// on chip. The HBM copy is stale while an entry is dirty; write-back on eviction, on free
// (freed chunks must hold qty 0 in HBM) and at kernel end. With the register ladder (L <= 128)
// every level has its own entry (no evictions).
constexpr int CK_MEM = 64;  // entries with the LDS ladder (direct-mapped by level)
constexpr int CK_REG = 128;
struct alignas(16) CacheEntry {
  uint32_t cid;    // cached chunk id, NIL = empty
  uint32_t dirty;  // slots differ from HBM
  uint32_t next;   // chdr[cid].next (kept in sync by set_next)
  uint32_t pad;
  int qty[ME_C];
  unsigned long long seq[ME_C];
};

// ---- ladders: where a wave keeps its symbol's price levels ---------------------------------
// LadderMem: levels / occupancy / tail-fill arrays behind pointers (LDS for L <= 1024, else HBM).
struct LadderMem {
  Level* lv;
  unsigned long long* occ;
  uint8_t* tend;
  uint32_t L, Lwords;

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
    for (int b = w + 1; b < nw; b += 64) {
      int idx = b + lane;
      unsigned long long v = idx < nw ? occ[idx] : 0ull;
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
    for (int t0 = w - 1; t0 >= 0; t0 -= 64) {
      int idx = t0 - lane;
      unsigned long long v = idx >= 0 ? occ[idx] : 0ull;
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

// LadderReg (L <= 128): level l lives in lane (l & 63) of register row (l >> 6). Reads are
// readlanes, writes are per-lane selects; occupancy is a 128-bit mask in SGPRs (best-price search
// = one bit scan). The head-chunk cache entry of level l is l itself (no evictions) and its
// valid / dirty state are SGPR masks too: no memory round trip for any ladder bookkeeping.
struct LadderReg {
  long long t0, t1;  // total
  uint32_t h0, h1;   // head chunk
  uint32_t l0, l1;   // tail chunk
  uint32_t e0, e1;   // slots written in the tail chunk
  uint32_t L;
  unsigned long long occ0, occ1;  // occupancy (wave-uniform)
  unsigned long long cv0, cv1;    // cache entry l holds the head chunk of l
  unsigned long long cd0, cd1;    // cache entry l is dirty

  __device__ __forceinline__ Level get(int l) const {
    const int j = l & 63;
    Level x;
    if (l < 64) {
      x.total = rli64(t0, j);
      x.head = rl32(h0, j);
      x.tail = rl32(l0, j);
    } else {
      x.total = rli64(t1, j);
      x.head = rl32(h1, j);
      x.tail = rl32(l1, j);
    }
    return x;
  }
  // (branch-free on purpose: a row-dependent if/else over members turns into a pointer select
  // that keeps the whole context in scratch memory)
  __device__ __forceinline__ void set(int l, const Level& x) {
    const bool me = lane_id() == (l & 63);
    const bool m0 = me && l < 64, m1 = me && l >= 64;
    t0 = m0 ? x.total : t0;
    h0 = m0 ? x.head : h0;
    l0 = m0 ? x.tail : l0;
    t1 = m1 ? x.total : t1;
    h1 = m1 ? x.head : h1;
    l1 = m1 ? x.tail : l1;
  }
  __device__ __forceinline__ uint32_t get_te(int l) const { return l < 64 ? rl32(e0, l & 63) : rl32(e1, l & 63); }
  __device__ __forceinline__ void set_te(int l, uint32_t v) {
    const bool me = lane_id() == (l & 63);
    e0 = (me && l < 64) ? v : e0;
    e1 = (me && l >= 64) ? v : e1;
  }
  static __device__ __forceinline__ unsigned long long lo_bit(int l) { return l < 64 ? (1ull << (l & 63)) : 0ull; }
  static __device__ __forceinline__ unsigned long long hi_bit(int l) { return l >= 64 ? (1ull << (l & 63)) : 0ull; }
  static __device__ __forceinline__ void bit_set(unsigned long long& a, unsigned long long& b, int l) {
    a |= lo_bit(l);
    b |= hi_bit(l);
  }
  static __device__ __forceinline__ void bit_clr(unsigned long long& a, unsigned long long& b, int l) {
    a &= ~lo_bit(l);
    b &= ~hi_bit(l);
  }
  static __device__ __forceinline__ bool bit_get(unsigned long long a, unsigned long long b, int l) {
    return l < 64 ? ((a >> l) & 1ull) : ((b >> (l - 64)) & 1ull);
  }
  __device__ __forceinline__ void occ_set(int l) { bit_set(occ0, occ1, l); }
  __device__ __forceinline__ void occ_clear(int l) { bit_clr(occ0, occ1, l); }
  __device__ __forceinline__ int next_occ(int x) const {
    if (x >= (int)L) return (int)L;
    if (x < 0) x = 0;
    if (x < 64) {
      const unsigned long long w = occ0 & (~0ull << x);
      if (w) return __builtin_ctzll(w);
      return occ1 ? 64 + __builtin_ctzll(occ1) : (int)L;
    }
    const unsigned long long w = occ1 & (~0ull << (x - 64));
    return w ? 64 + __builtin_ctzll(w) : (int)L;
  }
  __device__ __forceinline__ int prev_occ(int x) const {
    if (x < 0) return -1;
    if (x >= (int)L) x = (int)L - 1;
    if (x >= 64) {
      const int r = x - 64;
      const unsigned long long w = occ1 & ((r == 63) ? ~0ull : ((1ull << (r + 1)) - 1ull));
      if (w) return 64 + 63 - __builtin_clzll(w);
      return occ0 ? 63 - __builtin_clzll(occ0) : -1;
    }
    const unsigned long long w = occ0 & ((x == 63) ? ~0ull : ((1ull << (x + 1)) - 1ull));
    return w ? 63 - __builtin_clzll(w) : -1;
  }
};


// LadderWin (k_match_hot, deep windows): one workgroup per hot symbol. The whole occupancy bitmap
// and a window [wlo, wlo + W) of the ladder (levels + tail fills) around the best prices live in
// LDS for the launch; levels outside the window stay in HBM. Every accessor branches on the
// (wave-uniform) level, so top-of-book work never leaves the CU and deep rests cost one HBM
// round trip as before. LDS pointers are address-space-3 (ds_* instructions: an LDS access never
// waits on the wave's outstanding global stores, as a flat one would).
template <class T>
using lptr = T __attribute__((address_space(3)))*;
template <class T>
using gptr1 = T __attribute__((address_space(1)))*;

// Level copies across address spaces go field by field (one 16-B access after merging).
template <class P>
__device__ __forceinline__ Level ld_level(P p) {
  Level x;
  x.total = p->total;
  x.head = p->head;
  x.tail = p->tail;
  return x;
}
template <class P>
__device__ __forceinline__ void st_level(P p, const Level& x) {
  p->total = x.total;
  p->head = x.head;
  p->tail = x.tail;
}

struct LadderWin {
  lptr<Level> wl;                 // LDS levels of the window
  lptr<uint8_t> wt;               // LDS tail fills of the window
  lptr<unsigned long long> occ;   // LDS occupancy of the whole ladder
  gptr1<Level> glv;               // HBM ladder (authoritative outside the window)
  gptr1<uint8_t> gtend;
  uint32_t L, Lwords;
  int wlo;
  uint32_t W;

  __device__ __forceinline__ bool inw(int l) const { return (uint32_t)(l - wlo) < W; }
  __device__ __forceinline__ Level get(int l) const {
    Level x;
    if (inw(l)) {
      x = ld_level(wl + (l - wlo));
    } else {
      x = ld_level(glv + l);
    }
    x.total = rli64(x.total, 0);
    x.head = rl32(x.head, 0);
    x.tail = rl32(x.tail, 0);
    return x;
  }
  __device__ __forceinline__ uint32_t head(int l) const { return get(l).head; }
  __device__ __forceinline__ void set(int l, const Level& x) {
    if (lane_id() == 0) {
      if (inw(l))
        st_level(wl + (l - wlo), x);
      else
        st_level(glv + l, x);
    }
  }
  __device__ __forceinline__ Level lane_get(int l, bool valid) const {
    Level x{0, NIL, NIL};
    if (valid) {
      if (inw(l))
        x = ld_level(wl + (l - wlo));
      else
        x = ld_level(glv + l);
    }
    return x;
  }
  __device__ __forceinline__ uint32_t get_te(int l) const {
    if (inw(l)) return rl32((uint32_t)wt[l - wlo], 0);
    return rl32((uint32_t)gtend[l], 0);
  }
  __device__ __forceinline__ void set_te(int l, uint32_t v) {
    if (lane_id() == 0) {
      if (inw(l))
        wt[l - wlo] = (uint8_t)v;
      else
        gtend[l] = (uint8_t)v;
    }
  }
  __device__ __forceinline__ void occ_set(int l) {
    if (lane_id() == 0) occ[l >> 6] |= (1ull << (l & 63));
  }
  __device__ __forceinline__ void occ_clear(int l) {
    if (lane_id() == 0) occ[l >> 6] &= ~(1ull << (l & 63));
  }
  // Smallest occupied level >= x, or L (64 bitmap words per step from LDS).
  __device__ int next_occ(int x) const {
    const int Li = (int)L;
    if (x >= Li) return Li;
    if (x < 0) x = 0;
    const int w = x >> 6;
    const unsigned long long word = occ[w] & (~0ull << (x & 63));
    if (word) return (w << 6) + __builtin_ctzll(word);
    const int lane = lane_id();
    const int nw = (int)Lwords;
    for (int b = w + 1; b < nw; b += 64) {
      const int idx = b + lane;
      const unsigned long long v = idx < nw ? occ[idx] : 0ull;
      const unsigned long long m = __ballot(v != 0ull);
      if (m) {
        const int t = __builtin_ctzll(m);
        return ((b + t) << 6) + __builtin_ctzll(rl64(v, t));
      }
    }
    return Li;
  }
  // Largest occupied level <= x, or -1.
  __device__ int prev_occ(int x) const {
    if (x < 0) return -1;
    if (x >= (int)L) x = (int)L - 1;
    const int w = x >> 6;
    const int r = x & 63;
    const unsigned long long keep = (r == 63) ? ~0ull : ((1ull << (r + 1)) - 1ull);
    const unsigned long long word = occ[w] & keep;
    if (word) return (w << 6) + 63 - __builtin_clzll(word);
    const int lane = lane_id();
    for (int t0 = w - 1; t0 >= 0; t0 -= 64) {
      const int idx = t0 - lane;
      const unsigned long long v = idx >= 0 ? occ[idx] : 0ull;
      const unsigned long long m = __ballot(v != 0ull);
      if (m) {
        const int t = __builtin_ctzll(m);
        return ((t0 - t) << 6) + 63 - __builtin_clzll(rl64(v, t));
      }
    }
    return -1;
  }
};

template <class Lad>
struct WaveCtx {
  BookDev bk;
  Lad lad;
  CacheEntry* cache;         // head-chunk cache in LDS, or nullptr (HBM ladder)
  uint32_t cmask;            // cache entry of level l = l & cmask
  uint32_t s;                // local symbol
  uint32_t gs;               // symbol id written in fills
  long long base;
  int bb, ba;                // best bid / best ask level
  uint32_t free_head;        // chunk free list of this symbol ...
  uint32_t free_next;        // ... and chdr[free_head].next, loaded ahead of the pop that needs it
  uint32_t bump_cur, bump_end;  // chunk ids reserved from the global bump allocator
  uint32_t recs_left;        // records of this wave not processed yet (>= chunks it can still need)
  int resting_delta;
  unsigned long long wptr;   // next scratch slot of this wave
  me_fill* scratch;
#ifdef ME_STAMPS
  unsigned long long st[PH_N];
  unsigned long long st_t;
#endif
};

__device__ __forceinline__ void set_err(const BookDev& bk, uint32_t bits) {
  if (lane_id() == 0) atomicOr(bk.err, bits);
}

// ---- head-chunk cache -------------------------------------------------------------------
// Generic ladders keep the entry's chunk id and dirty flag in LDS; the register ladder keeps
// them as SGPR masks (valid bit l <=> entry l holds the current head chunk of level l), so a
// lookup there is a bit test, never an LDS round trip.
template <class C>
constexpr bool kRegLadder = __is_same(decltype(C::lad), LadderReg);

template <class C>
__device__ __forceinline__ CacheEntry* centry(const C& c, int lvl) { return c.cache + ((uint32_t)lvl & c.cmask); }

template <class C>
__device__ __forceinline__ uint32_t head_of(const C& c, int lvl) {
  if constexpr (kRegLadder<C>)
    return lvl < 64 ? rl32(c.lad.h0, lvl & 63) : rl32(c.lad.h1, lvl & 63);
  else
    return c.lad.head(lvl);
}

template <class C>
__device__ __forceinline__ bool cache_holds(const C& c, int lvl, uint32_t ch) {
  if constexpr (kRegLadder<C>)
    return LadderReg::bit_get(c.lad.cv0, c.lad.cv1, lvl) && head_of(c, lvl) == ch;
  else
    return c.cache && rl32(centry(c, lvl)->cid, 0) == ch;
}

template <class C>
__device__ __forceinline__ void cache_mark_dirty(C& c, int lvl) {
  if constexpr (kRegLadder<C>)
    LadderReg::bit_set(c.lad.cd0, c.lad.cd1, lvl);
  else if (lane_id() == 0)
    centry(c, lvl)->dirty = 1;
}

// Write entry E of level lvl back to HBM if dirty. Register ladder: the caller passes the chunk
// the (valid) entry holds; generic ladders read it from the entry.
template <class C>
__device__ __forceinline__ void cache_writeback(const C& c, int lvl, CacheEntry* E, uint32_t held = NIL) {
  uint32_t cid;
  if constexpr (kRegLadder<C>) {
    if (!LadderReg::bit_get(c.lad.cv0, c.lad.cv1, lvl) || !LadderReg::bit_get(c.lad.cd0, c.lad.cd1, lvl)) return;
    cid = held;
  } else {
    cid = rl32(E->cid, 0);
    if (cid == NIL || !rl32(E->dirty, 0)) return;
  }
  const int lane = lane_id();
  if (lane < ME_C) {
    const size_t g = (size_t)cid * ME_C + lane;
    cq_at(c.bk.chunks, g) = E->qty[lane];
    cs_at(c.bk.chunks, g) = E->seq[lane];
  }
}

template <class C>
__device__ __forceinline__ void cache_set_state(C& c, int lvl, CacheEntry* E, uint32_t ch, bool dirty) {
  if constexpr (kRegLadder<C>) {
    LadderReg::bit_set(c.lad.cv0, c.lad.cv1, lvl);
    if (dirty)
      LadderReg::bit_set(c.lad.cd0, c.lad.cd1, lvl);
    else
      LadderReg::bit_clr(c.lad.cd0, c.lad.cd1, lvl);
    if (lane_id() == 0) E->cid = ch;
  } else if (lane_id() == 0) {
    E->cid = ch;
    E->dirty = dirty ? 1u : 0u;
  }
}

// Make `ch` (the head chunk of level lvl) the cached chunk of its entry; returns the entry.
template <class C>
__device__ __forceinline__ CacheEntry* cache_get(C& c, int lvl, uint32_t ch) {
  CacheEntry* E = centry(c, lvl);
  if constexpr (kRegLadder<C>) {
    if (LadderReg::bit_get(c.lad.cv0, c.lad.cv1, lvl)) return E;  // valid => holds the head
  } else {
    const uint32_t cur = rl32(E->cid, 0);
    if (cur == ch) return E;
    if (cur != NIL) COUNT(c, CT_EVICT);
    cache_writeback(c, lvl, E);
  }
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
  cache_set_state(c, lvl, E, ch, false);
  return E;
}

// A brand-new (all-empty) chunk becomes the head of an empty level: install it without a load.
template <class C>
__device__ __forceinline__ void cache_install_new(C& c, int lvl, uint32_t ch) {
  CacheEntry* E = centry(c, lvl);
  if constexpr (!kRegLadder<C>) cache_writeback(c, lvl, E);  // register ladder: entry of an empty level is invalid
  const int lane = lane_id();
  if (lane < ME_C) {
    E->qty[lane] = 0;
    E->seq[lane] = 0ull;
  }
  if (lane == 0) E->next = NIL;
  cache_set_state(c, lvl, E, ch, true);
}

// The cached chunk ch of lvl is being freed or unlinked: HBM must hold its final (all-zero)
// quantities before the chunk is reused. Callers pass the chunk the entry holds (the level's
// head, or the chunk a walk just loaded); generic ladders double-check the id.
template <class C>
__device__ __forceinline__ void cache_drop(C& c, int lvl, uint32_t ch) {
  if (!c.cache) return;
  CacheEntry* E = centry(c, lvl);
  if constexpr (kRegLadder<C>) {
    if (!LadderReg::bit_get(c.lad.cv0, c.lad.cv1, lvl)) return;
  } else {
    if (rl32(E->cid, 0) != ch) return;
  }
  cache_writeback(c, lvl, E, ch);
  if constexpr (kRegLadder<C>) {
    LadderReg::bit_clr(c.lad.cv0, c.lad.cv1, lvl);
    LadderReg::bit_clr(c.lad.cd0, c.lad.cd1, lvl);
  } else if (lane_id() == 0) {
    E->cid = NIL;
  }
}

// chdr[ch].next = v, mirrored into the cache entry of lvl when it holds ch.
template <class C>
__device__ __forceinline__ void set_next(C& c, int lvl, uint32_t ch, uint32_t v) {
  const bool mirror = c.cache && cache_holds(c, lvl, ch);
  if (lane_id() == 0) {
    c.bk.chunks[ch].hdr.next = v;
    if (mirror) centry(c, lvl)->next = v;
  }
}

// ---- chunk allocation -------------------------------------------------------------------
// Free-list push: the popped-next is known without a load.
template <class C>
__device__ __forceinline__ void free_chunk(C& c, uint32_t ch) {
  if (lane_id() == 0) c.bk.chunks[ch].hdr.next = c.free_head;
  c.free_next = c.free_head;
  c.free_head = ch;
}

// Issue the load of chdr[free_head].next without waiting for it: the value stays in a VGPR and is
// only read (readlane -> s_waitcnt) by the next pop, usually many records later.
template <class C>
__device__ __forceinline__ void prefetch_free_next(C& c) {
  const bool ok = c.free_head < c.bk.nchunks;
  const uint32_t v = c.bk.chunks[ok ? c.free_head : 0].hdr.next;
  c.free_next = ok ? v : NIL;
}

template <class C>
__device__ __forceinline__ uint32_t alloc_chunk(C& c) {
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
    if (got >= c.bk.nchunks) {
      set_err(c.bk, ERR_CHUNK_OOM);
      return NIL;
    }
    c.bump_cur = got;
    c.bump_end = min(got + BLK, c.bk.nchunks);
  }
  return c.bump_cur++;
}

// Append one fill per lane where e holds, in lane order, to the wave's scratch run.
template <class C>
__device__ __forceinline__ void emit_fills(C& c, bool e, unsigned long long taker, unsigned long long maker,
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

// Consume `take` (> 0, <= level total) from the FIFO of level `lvl`, oldest first. A slot is
// live iff its qty > 0 (consumed, cancelled and unwritten slots hold 0). A chunk's 16 slots are
// ranked with one wave prefix scan; with the cache they come from LDS, otherwise one HBM round
// trip loads header and slots together. Exhausted chunks go back to the free list. Returns the
// new head chunk (NIL: level emptied).
template <class C>
__device__ __forceinline__ uint32_t walk_level(C& c, int lvl, long long take, uint32_t head, uint32_t tail,
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
template <class C>
__device__ __forceinline__ void level_after_take(C& c, int lvl, long long ntot, uint32_t nh, uint32_t tail) {
  Level o;
  o.total = ntot;
  o.head = ntot ? nh : NIL;
  o.tail = ntot ? tail : NIL;
  c.lad.set(lvl, o);
  if (ntot == 0) c.lad.occ_clear(lvl);
}

// Consume `take` at level lvl whose header is (tot, head, tail); returns true if it emptied.
template <class C>
__device__ __forceinline__ bool take_level(C& c, int lvl, long long tot, long long take, uint32_t head,
                                           uint32_t tail, unsigned long long taker) {
  STAMP_ADD(c, PH_SWEEP);
  const uint32_t nh = walk_level(c, lvl, take, head, tail, taker);
  STAMP_ADD(c, PH_WALK);
  level_after_take(c, lvl, tot - take, nh, tail);
  STAMP_ADD(c, PH_SW_UPDATE);
  return tot == take;
}

// Sweep the opposite side for a taker. dir = +1 (BUY: asks upward from best_ask) or -1 (SELL:
// bids downward from best_bid); lim = last level the taker may trade at. Returns qty filled.
// LadderMem: 64-level windows — lanes load consecutive levels, an inclusive scan of their totals
// says how far the taker reaches. LadderReg: one masked scan over the register-resident ladder.
template <class C>
__device__ __forceinline__ long long sweep(C& c, int dir, int lim, long long want, unsigned long long taker, uint32_t& nfill) {
  const int lane = lane_id();
  const int L = (int)c.bk.L;
  long long rem = want;
  int cur = (dir > 0) ? c.ba : c.bb;
  bool emptied = false;
  const unsigned long long w_start = c.wptr;
  nfill = 0;
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
      nfill = (uint32_t)(c.wptr - w_start);
      return want;
    }
  }
  if constexpr (kRegLadder<C>) {
    // level by level from the best: the occupancy bit scan finds the next level in SALU, the
    // level header is a readlane — no scan, no memory round trip
    while (rem > 0 && (dir > 0 ? (cur <= lim && cur < L) : (cur >= lim && cur >= 0))) {
      const Level B = c.lad.get(cur);
      const long long take = B.total < rem ? B.total : rem;
      const bool gone = take_level(c, cur, B.total, take, B.head, B.tail, taker);
      rem -= take;
      if (!gone) break;  // partially consumed: the taker is done
      emptied = true;
      cur = dir > 0 ? c.lad.next_occ(cur + 1) : c.lad.prev_occ(cur - 1);
      STAMP_ADD(c, PH_SW_JUMP);
    }
  } else {
    while (rem > 0) {
      if (dir > 0 ? (cur > lim || cur >= L) : (cur < lim || cur < 0)) break;
      const int lv = cur + dir * lane;
      const bool valid = (dir > 0) ? (lv <= lim && lv < L) : (lv >= lim && lv >= 0);
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
  }
  if (emptied) {
    if (dir > 0)
      c.ba = c.lad.next_occ(c.ba);
    else
      c.bb = c.lad.prev_occ(c.bb);
    STAMP_ADD(c, PH_SW_BEST);
  }
  nfill = (uint32_t)(c.wptr - w_start);
  return want - rem;
}

// Append a resting order at the tail of level lvl's FIFO. The tail fill count lives beside the
// level, so the common case issues no HBM load; a tail that is the cached head is written on chip.
template <class C>
__device__ __forceinline__ bool rest_order(C& c, int lvl, unsigned long long seq, int qty, bool buy) {
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
      h.level = (uint32_t)lvl;
      h.owner = c.s;
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
    if (seq < bk.max_seq) bk.loc[seq] = (uint32_t)g;
  }
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

// Cancel the live resting order `tgt` of this symbol. Returns the removed qty, 0 if not live.
// A chunk left without live orders is unlinked from its FIFO at once (so chunks in use never
// exceed resting orders); a level left empty returns its whole FIFO to the free list.
template <class C>
__device__ __forceinline__ int cancel_order(C& c, unsigned long long tgt) {
  const BookDev& bk = c.bk;
  const int lane = lane_id();
  if (tgt == 0ull || tgt >= bk.max_seq) return 0;
  wave_mem_order();
  const uint32_t g = rl32(bk.loc[tgt], 0);
  if (g == NIL) return 0;
  const uint32_t ch = g / ME_C, slot = g % ME_C;
  if (ch >= bk.nchunks) return 0;
  // one round trip: owner, header, the whole chunk's quantities and the target seq
  const uint32_t owner = rl32(bk.chunks[ch].hdr.owner, 0);
  const ChunkHdr hd = bk.chunks[ch].hdr;
  const bool act = lane < ME_C;
  int qv = act ? cq_at(bk.chunks, (size_t)ch * ME_C + lane) : 0;
  unsigned long long sq = rl64(cs_at(bk.chunks, g), 0);
  if (owner != c.s) return 0;  // another symbol's order: never touch its book
  const int lvl = (int)rl32(hd.level, 0);
  if (lvl < 0 || lvl >= (int)bk.L) {
    set_err(bk, ERR_INCONSISTENT);
    return 0;
  }
  CacheEntry* E = cache_holds(c, lvl, ch) ? centry(c, lvl) : nullptr;
  if (E) {  // the on-chip copy is authoritative
    qv = act ? E->qty[lane] : 0;
    sq = rl64(E->seq[slot], 0);
  }
  const int q = rli32(qv, (int)slot);
  if (sq != tgt || q <= 0) return 0;
  const uint32_t nxt = rl32(hd.next, 0), prv = rl32(hd.prev, 0);
  const uint32_t live_after = (uint32_t)__popcll(__ballot(qv > 0)) - 1;
  Level L = c.lad.get(lvl);
  L.total -= q;
  if (L.tail >= bk.nchunks || L.head >= bk.nchunks) {
    set_err(bk, ERR_INCONSISTENT);
    return q;
  }
  if (E) cache_mark_dirty(c, lvl);
  if (lane == 0) {
    if (E) {
      E->qty[slot] = 0;
    } else {
      cq_at(bk.chunks, g) = 0;
    }
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
  return q;
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
__host__ __device__ constexpr size_t lds_wave_bytes_reg() { return CK_REG * sizeof(CacheEntry); }

// Ladder placement of a k_match instantiation.
enum LadderKind { LAD_HBM = 0, LAD_LDS = 1, LAD_REG = 2 };

// The per-record loop of one symbol, shared by every ladder kind.
template <class C>
__device__ __forceinline__ void match_records(C& c, const BatchDev& bt, uint32_t lo, uint32_t hi) {
  const int lane = lane_id();
  const BookDev& bk = c.bk;
  const long long Lw = (long long)bk.L;
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
      const unsigned long long seq = rl64(oseq, (int)k);
      const long long px = rli64(opx, (int)k);
      const int q = rli32(oq, (int)k);
      const uint32_t kind = rl32(ok_, (int)k);
      c.recs_left = hi - (blk + k);
      const uint32_t side = kind & 3u;
      const bool market = (kind >> 2) & 1u;
      const bool cancel = (kind >> 3) & 1u;
      const unsigned long long fstart = c.wptr;
      if (cancel) {
        const int got = cancel_order(c, (unsigned long long)px);
        STAMP_ADD(c, PH_CANCEL);
        if (got > 0)
          put_result(R, k, 0, got, 0, ME_ST_CANCELED, ME_RJ_NONE, fstart);
        else
          put_result(R, k, 0, 0, 0, ME_ST_REJECTED, ME_RJ_UNKNOWN_ORDER, fstart);
        continue;
      }
      if (q <= 0) {
        put_result(R, k, 0, 0, 0, ME_ST_REJECTED, ME_RJ_BAD_QTY, fstart);
        continue;
      }
      if (side != ME_SIDE_BUY && side != ME_SIDE_SELL) {
        put_result(R, k, 0, q, 0, ME_ST_REJECTED, ME_RJ_BAD_SIDE, fstart);
        continue;
      }
      int li = 0;
      if (!market) {
        if (px < c.base || (unsigned long long)px - (unsigned long long)c.base >= (unsigned long long)Lw) {
          put_result(R, k, 0, q, 0, ME_ST_REJECTED, ME_RJ_OUT_OF_WINDOW, fstart);
          continue;
        }
        li = (int)(px - c.base);
      }
      if (seq == 0ull || seq >= bk.max_seq) {
        put_result(R, k, 0, q, 0, ME_ST_REJECTED, ME_RJ_BAD_SEQ, fstart);
        continue;
      }
      const bool buy = side == ME_SIDE_BUY;
      const int lim = market ? (buy ? (int)Lw - 1 : 0) : li;
      uint32_t nfill = 0;
      const long long got = sweep(c, buy ? 1 : -1, lim, (long long)q, seq, nfill);
      STAMP_ADD(c, PH_SWEEP);
      const int filled = (int)got;
      const int rem = q - filled;
      uint8_t stt;
      if (market) {
        stt = rem == 0 ? ME_ST_FILLED : ME_ST_CANCELED;
      } else {
        const bool failed = rem > 0 && !rest_order(c, li, seq, rem, buy);
        STAMP_ADD(c, PH_REST);
        if (failed) {
          ok = false;  // chunk pool exhausted: the batch fails (sticky error word)
          break;
        }
        stt = rem == 0 ? ME_ST_FILLED : (filled > 0 ? ME_ST_PARTIALLY_FILLED : ME_ST_NEW);
      }
      put_result(R, k, filled, rem, nfill, stt, ME_RJ_NONE, fstart);
    }
    store_results(bt, R, v && (uint32_t)lane < k, oi);
    STAMP_ADD(c, PH_RESULT);
  }
  // return unused bump-reserved chunks to this symbol's free list
  while (c.bump_cur < c.bump_end) free_chunk(c, c.bump_cur++);
}

// Dirty cached head chunks back to HBM: lane = (entry, slot) pairs, 4 entries per pass.
template <class C>
__device__ __forceinline__ void cache_flush_all(C& c, uint32_t entries) {
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

template <class C>
__device__ __forceinline__ bool wave_begin(C& c, const BookDev& bk, const BatchDev& bt, uint32_t s, uint32_t lo, uint32_t hi) {
  const int lane = lane_id();
  c.bk = bk;
  c.s = s;
  c.gs = bk.gsym ? bk.gsym[s] : s;
  const SymState st = bk.sym[s];
  c.base = rli64(st.base, 0);
  c.bb = rli32(st.best_bid, 0);
  c.ba = rli32(st.best_ask, 0);
  c.free_head = rl32(st.free_head, 0);
  prefetch_free_next(c);
  c.bump_cur = c.bump_end = 0;
  c.resting_delta = (int)rl32(st.resting, 0);  // becomes the new resting count
  c.scratch = bt.scratch;
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

template <class C>
__device__ __forceinline__ void wave_end(C& c) {
  if (lane_id() == 0) {
    SymState o;
    o.base = c.base;
    o.best_bid = c.bb;
    o.best_ask = c.ba;
    o.free_head = c.free_head;
    o.resting = (uint32_t)c.resting_delta;
    o.nfree = 0;
    o.pad = 0;
    c.bk.sym[c.s] = o;
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
  const uint32_t lo = wave_lower_bound(bt.skeys, bt.n, s);
  const uint32_t hi = wave_lower_bound(bt.skeys, bt.n, s + 1);
  if (lo >= hi) return;
  if (s == bk.S) {
    reject_bad_symbols(bt, lo, hi);
    return;
  }
  if constexpr (kLad == LAD_HBM) {
    // a busy symbol goes to k_match_hot (LDS window of its ladder), launched right after this
    if (bt.hot_min && hi - lo >= bt.hot_min) {
      uint32_t idx = 0;
      if (lane == 0) idx = atomicAdd(bt.hot, 1u);
      idx = rl32(idx, 0);
      if (idx < HOT_MAX) {
        if (lane == 0) bt.hot[1 + idx] = s;
        return;
      }
    }
  }
  const uint32_t L = bk.L;
  Level* g_lv = bk.levels + (size_t)s * L;
  unsigned long long* g_occ = bk.occ + (size_t)s * bk.Lwords;
  uint8_t* g_tend = bk.tend + (size_t)s * L;
  if constexpr (kLad == LAD_REG) {
    WaveCtx<LadderReg> c;
#ifdef ME_STAMPS
    for (int p = 0; p < PH_N; ++p) c.st[p] = 0;
    STAMP_MARK(c);
#endif
    // levels lane and 64 + lane; the occupancy bitmap is implied by the totals
    Level a = g_lv[lane];
    Level b;
    b.total = 0;
    b.head = b.tail = NIL;
    if (64 + (uint32_t)lane < L) b = g_lv[64 + lane];
    c.lad.t0 = a.total;
    c.lad.h0 = a.head;
    c.lad.l0 = a.tail;
    c.lad.t1 = b.total;
    c.lad.h1 = b.head;
    c.lad.l1 = b.tail;
    c.lad.e0 = g_tend[lane];
    c.lad.e1 = (64 + (uint32_t)lane < L) ? g_tend[64 + lane] : 0u;
    c.lad.L = L;
    c.lad.occ0 = __ballot(a.total > 0);
    c.lad.occ1 = __ballot(b.total > 0);
    c.lad.cv0 = c.lad.cv1 = c.lad.cd0 = c.lad.cd1 = 0ull;
    c.cache = (CacheEntry*)(smem + (size_t)wv * lds_wave_bytes_reg());
    c.cmask = CK_REG - 1;
    if (!wave_begin(c, bk, bt, s, lo, hi)) return;
    STAMP_ADD(c, PH_PROLOGUE);
    match_records(c, bt, lo, hi);
    // dirty cached heads back to HBM (valid entry l holds the head of level l)
    for (int row = 0; row < 2; ++row) {
      unsigned long long d = row ? (c.lad.cd1 & c.lad.cv1) : (c.lad.cd0 & c.lad.cv0);
      while (d) {
        const int j = __builtin_ctzll(d);
        d &= d - 1;
        const uint32_t cid = row ? rl32(c.lad.h1, j) : rl32(c.lad.h0, j);
        const CacheEntry* E = c.cache + row * 64 + j;
        if (lane < ME_C) {
          cq_at(c.bk.chunks, (size_t)cid * ME_C + lane) = E->qty[lane];
          cs_at(c.bk.chunks, (size_t)cid * ME_C + lane) = E->seq[lane];
        }
      }
    }
    g_lv[lane] = Level{c.lad.t0, c.lad.h0, c.lad.l0};
    g_tend[lane] = (uint8_t)c.lad.e0;
    if (64 + (uint32_t)lane < L) {
      g_lv[64 + lane] = Level{c.lad.t1, c.lad.h1, c.lad.l1};
      g_tend[64 + lane] = (uint8_t)c.lad.e1;
    }
    // keep the HBM occupancy bitmap valid for the host-side book dump
    const unsigned long long m0 = __ballot(c.lad.t0 > 0), m1 = __ballot(c.lad.t1 > 0);
    if (lane == 0) {
      g_occ[0] = m0;
      if (bk.Lwords > 1) g_occ[1] = m1;
    }
    wave_end(c);
  } else {
    WaveCtx<LadderMem> c;
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
}


// ---- hot symbols of deep windows (L > LDS_MAX_LEVELS) --------------------------------------
// LDS of one k_match_hot workgroup: occupancy words | window levels | window tail fills | cache.
struct HotLds {
  uint32_t W, occ_off, lv_off, te_off, ck_off, bytes;
  uint32_t cache;  // head-chunk cache on (ME_HOT_CACHE=0 turns it off: A/B runs)
};
__host__ __device__ inline HotLds hot_lds(uint32_t L, uint32_t Lwords, uint32_t budget) {
  HotLds h{};
  h.occ_off = 0;
  const uint32_t fixed = Lwords * 8u + CK_MEM * (uint32_t)sizeof(CacheEntry) + 64u;
  uint32_t W = budget > fixed ? (budget - fixed) / ((uint32_t)sizeof(Level) + 1u) : 0u;
  W &= ~63u;
  if (W > L) W = L;
  h.W = W;
  h.lv_off = (Lwords * 8u + 15u) & ~15u;
  h.te_off = h.lv_off + W * (uint32_t)sizeof(Level);
  h.ck_off = (h.te_off + W + 15u) & ~15u;
  h.bytes = h.ck_off + CK_MEM * (uint32_t)sizeof(CacheEntry);
  h.cache = 1;
  return h;
}

// One workgroup (one wave) per hot symbol, the symbols k_match<LAD_HBM> handed over in bt.hot.
// Same record loop as k_match; the ladder window sits around the symbol's best prices.
__global__ __launch_bounds__(64) void k_match_hot(BookDev bk, BatchDev bt, HotLds hl) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = lane_id();
  const uint32_t cnt = min(rl32(bt.hot[0], 0), HOT_MAX);
  const uint32_t L = bk.L, W = hl.W;
  for (uint32_t i = blockIdx.x; i < cnt; i += gridDim.x) {
    const uint32_t s = rl32(bt.hot[1 + i], 0);
    const uint32_t lo = bt.bin_start ? bt.bin_start[s] : wave_lower_bound(bt.skeys, bt.n, s);
    const uint32_t hi = bt.bin_start ? bt.bin_start[s + 1] : wave_lower_bound(bt.skeys, bt.n, s + 1);
    gptr1<Level> g_lv = (gptr1<Level>)(bk.levels + (size_t)s * L);
    gptr1<unsigned long long> g_occ = (gptr1<unsigned long long>)(bk.occ + (size_t)s * bk.Lwords);
    gptr1<uint8_t> g_tend = (gptr1<uint8_t>)(bk.tend + (size_t)s * L);
    WaveCtx<LadderWin> c;
#ifdef ME_STAMPS
    for (int p = 0; p < PH_N; ++p) c.st[p] = 0;
    STAMP_MARK(c);
#endif
    const SymState st = bk.sym[s];
    const int bb = rli32(st.best_bid, 0), ba = rli32(st.best_ask, 0);
    int center = (int)L / 2;
    if (bb >= 0 && ba < (int)L)
      center = (bb + ba) / 2;
    else if (bb >= 0)
      center = bb;
    else if (ba < (int)L)
      center = ba;
    int wlo = center - (int)(W / 2);
    if (wlo > (int)(L - W)) wlo = (int)(L - W);
    if (wlo < 0) wlo = 0;
    wlo &= ~63;
    c.lad.wl = (lptr<Level>)(smem + hl.lv_off);
    c.lad.wt = (lptr<uint8_t>)(smem + hl.te_off);
    c.lad.occ = (lptr<unsigned long long>)(smem + hl.occ_off);
    c.lad.glv = g_lv;
    c.lad.gtend = g_tend;
    c.lad.L = L;
    c.lad.Lwords = bk.Lwords;
    c.lad.wlo = wlo;
    c.lad.W = W;
    c.cache = hl.cache ? (CacheEntry*)(smem + hl.ck_off) : nullptr;
    c.cmask = hl.cache ? CK_MEM - 1 : 0;
    // stage the window: 8 level loads per lane in flight per step
    for (uint32_t b = 0; b < W; b += 64 * 8) {
      Level r[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t j = b + (uint32_t)k * 64 + (uint32_t)lane;
        r[k] = Level{0, NIL, NIL};
        if (j < W) r[k] = ld_level(g_lv + (wlo + j));
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t j = b + (uint32_t)k * 64 + (uint32_t)lane;
        if (j < W) st_level(c.lad.wl + j, r[k]);
      }
    }
    {
      gptr1<uint32_t> gt4 = (gptr1<uint32_t>)(g_tend + wlo);  // wlo, W multiples of 64
      lptr<uint32_t> wt4 = (lptr<uint32_t>)c.lad.wt;
      for (uint32_t j = lane; j < W / 4; j += 64) wt4[j] = gt4[j];
      for (uint32_t j = lane; j < bk.Lwords; j += 64) c.lad.occ[j] = g_occ[j];
      if (c.cache)
        for (uint32_t j = lane; j < (uint32_t)CK_MEM; j += 64) c.cache[j].cid = NIL;
    }
    wave_mem_order();
    if (!wave_begin(c, bk, bt, s, lo, hi)) return;
    STAMP_ADD(c, PH_PROLOGUE);
    match_records(c, bt, lo, hi);
    if (c.cache) cache_flush_all(c, CK_MEM);
    wave_mem_order();
    for (uint32_t j = lane; j < W; j += 64) st_level(g_lv + (wlo + j), ld_level(c.lad.wl + j));
    {
      gptr1<uint32_t> gt4 = (gptr1<uint32_t>)(g_tend + wlo);
      lptr<uint32_t> wt4 = (lptr<uint32_t>)c.lad.wt;
      for (uint32_t j = lane; j < W / 4; j += 64) gt4[j] = wt4[j];
      for (uint32_t j = lane; j < bk.Lwords; j += 64) g_occ[j] = c.lad.occ[j];
    }
    wave_end(c);
    wave_mem_order();
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
                                                      uint32_t* err) {
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
  for (uint32_t k = tid; k < cnt; k += 256) res[r0 + k].tape_offset = (uint32_t)(base + off[k]);
  __syncthreads();
  if (base + total > tape_cap) {
    if (tid == 0) atomicOr(err, ERR_SCRATCH_OOM);
    return;
  }
  for (uint32_t f = tid; f < total; f += 256) {
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
                            uint32_t zero_words, unsigned long long* scratch_top, uint32_t* bin_start) {
  SortPass p;
  p.shift = (uint32_t)shift;
  p.mask = (1u << dbits) - 1u;
  p.nbins = min(1u << dbits, (clamp_key >> shift) + 1u);
  p.tile = sort_tile(n);
  p.ntiles = (n + p.tile - 1) / p.tile;
  p.clamp = clamp_key;
  hipLaunchKernelGGL(k_sort_hist, dim3(p.ntiles), dim3(256), 0, st, keys_in, n, p, hist, zero_buf, zero_words,
                     scratch_top);
  hipLaunchKernelGGL(k_sort_colscan, dim3((p.nbins + 63) / 64), dim3(64), 0, st, hist, tot, p.nbins, p.ntiles);
  hipLaunchKernelGGL(k_sort_scatter, dim3(p.ntiles), dim3(256), 0, st, keys_in, idx_in, n, p, (uint32_t)dbits, hist,
                     tot, keys_out, idx_out, bin_start);
  return hipGetLastError();
}

hipError_t launch_match_reg(hipStream_t st, const BookDev& bk, const BatchDev* bt, uint32_t ng, const AuxDev& ax,
                            hipEvent_t ev0, hipEvent_t ev1);

// LDS one k_match_hot workgroup may use (the CU's 160 KB, less a margin).
uint32_t hot_lds_budget() { return 160u * 1024u - 1024u; }
static uint32_t g_hot_cache = 1;

// Opt k_match_hot into the large dynamic LDS allocation once per process.
hipError_t prepare_hot(const BookDev& bk) {
  const HotLds hl = hot_lds(bk.L, bk.Lwords, hot_lds_budget());
  if (hl.W < 64) return hipErrorInvalidValue;
  if (const char* v = getenv("ME_HOT_CACHE")) g_hot_cache = (uint32_t)atoi(v);
  return hipFuncSetAttribute((const void*)k_match_hot, hipFuncAttributeMaxDynamicSharedMemorySize, (int)hl.bytes);
}

// ev0 / ev1 (optional, timing): the launch records the kernel's own start and end
// (hipExtLaunchKernelGGL), so timing adds no marker packet — and no gap — to the stream.
hipError_t launch_match(hipStream_t st, const BookDev& bk, const BatchDev& bt, hipEvent_t ev0, hipEvent_t ev1) {
  const uint32_t waves = bk.S + 1;
  const dim3 grid((waves + 3) / 4), block(256);
  if (bk.L <= 128) {
    return launch_match_reg(st, bk, &bt, 1u, AuxDev{}, ev0, ev1);
  } else if (bk.L <= LDS_MAX_LEVELS) {
    hipExtLaunchKernelGGL(k_match<LAD_LDS>, grid, block, 4 * lds_wave_bytes(bk.L), st, ev0, ev1, 0, bk, bt);
  } else if (!bt.hot_min || !bt.hot) {
    hipExtLaunchKernelGGL(k_match<LAD_HBM>, grid, block, 0, st, ev0, ev1, 0, bk, bt);
  } else {
    // deep windows: cold symbols match against the HBM ladder; busy ones are handed to
    // k_match_hot, one workgroup each with an LDS window of the ladder
    HotLds hl = hot_lds(bk.L, bk.Lwords, hot_lds_budget());
    hl.cache = g_hot_cache;
    hipError_t he = hipMemsetAsync(bt.hot, 0, 4, st);
    if (he != hipSuccess) return he;
    hipExtLaunchKernelGGL(k_match<LAD_HBM>, grid, block, 0, st, ev0, nullptr, 0, bk, bt);
    hipExtLaunchKernelGGL(k_match_hot, dim3(HOT_GRID), dim3(64), hl.bytes, st, nullptr, ev1, 0, bk, bt, hl);
  }
  return hipGetLastError();
}

hipError_t launch_tape(hipStream_t st, const BatchDev& bt, me_fill* tape, unsigned long long tape_cap,
                       unsigned long long* tape_count, unsigned long long* fills_acc, uint32_t* err) {
  const uint32_t ntiles = (bt.n + TILE_TAPE - 1) / TILE_TAPE;
  hipLaunchKernelGGL(k_tape_compact, dim3(ntiles), dim3(256), 0, st, bt.tile_sum, ntiles, bt.res, bt.fstart,
                     bt.n, bt.scratch, tape, tape_cap, tape_count, fills_acc, err);
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

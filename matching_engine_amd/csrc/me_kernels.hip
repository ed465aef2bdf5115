// me_kernels.hip — gfx950 kernels of the batched matching core.
//
// One batch (n records, ascending seq) goes through:
//   1. k_sort_hist / k_sort_offsets / k_sort_scatter
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
#include <hip/hip_runtime.h>

#include "me_layout.hpp"

namespace me {

// ------------------------------------------------------------------ wave helpers
__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

__device__ __forceinline__ uint32_t rl32(uint32_t v, int k) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, k);
}
__device__ __forceinline__ int32_t rli32(int32_t v, int k) { return __builtin_amdgcn_readlane(v, k); }
__device__ __forceinline__ unsigned long long rl64(unsigned long long v, int k) {
  uint32_t lo = rl32((uint32_t)v, k), hi = rl32((uint32_t)(v >> 32), k);
  return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ long long rli64(long long v, int k) {
  return (long long)rl64((unsigned long long)v, k);
}
__device__ __forceinline__ unsigned long long lanemask_lt() {
  return (1ull << lane_id()) - 1ull;
}
// DPP row shift / broadcast of a 32-bit value: lanes whose source is outside the pattern get 0.
template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, kRowMask, 0xF, false);
}
template <int kCtrl, int kRowMask>
__device__ __forceinline__ long long dpp64(long long v) {
  const uint32_t lo = dpp32<kCtrl, kRowMask>((uint32_t)v);
  const uint32_t hi = dpp32<kCtrl, kRowMask>((uint32_t)((unsigned long long)v >> 32));
  return (long long)(((unsigned long long)hi << 32) | lo);
}
// Inclusive 64-lane prefix sum of an int64 on the VALU with DPP (no LDS permutes): row_shr
// 1/2/4/8 scans each 16-lane row, row_bcast:15 / row_bcast:31 carry the row totals.
__device__ __forceinline__ long long wave_incl_scan(long long x) {
  x += dpp64<0x111, 0xF>(x);  // row_shr:1
  x += dpp64<0x112, 0xF>(x);  // row_shr:2
  x += dpp64<0x114, 0xF>(x);  // row_shr:4
  x += dpp64<0x118, 0xF>(x);  // row_shr:8
  x += dpp64<0x142, 0xA>(x);  // row_bcast:15 into rows 1, 3
  x += dpp64<0x143, 0xC>(x);  // row_bcast:31 into rows 2, 3
  return x;
}
// Orders the wave's own global stores before its later loads of the same lines (another lane
// may read what this lane wrote). Same-CU ordering: no cache maintenance, a compiler barrier.
__device__ __forceinline__ void wave_mem_order() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

// Diagnostic build only (-DME_STAMPS): per-wave cycle shares of the matching phases, read with
// me_debug_stamps(). The product build compiles every stamp away.
enum { PH_PROLOGUE, PH_FETCH, PH_SWEEP, PH_WALK, PH_REST, PH_CANCEL, PH_RESULT, PH_EPILOGUE,
       PH_SW_WINDOW, PH_SW_UPDATE, PH_SW_JUMP, PH_SW_BEST, PH_N };
#ifdef ME_STAMPS
__device__ __forceinline__ unsigned long long stamp_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define STAMP_MARK(c) (c).st_t = stamp_now()
#define STAMP_ADD(c, ph)                    \
  do {                                      \
    unsigned long long _n = stamp_now();    \
    (c).st[ph] += _n - (c).st_t;            \
    (c).st_t = _n;                          \
  } while (0)
#else
#define STAMP_MARK(c) ((void)0)
#define STAMP_ADD(c, ph) ((void)0)
#endif

// First index p in [0, n) with keys[p] >= key (keys ascending), by a 64-ary search:
// every step the wave samples 64 positions, ballots, and narrows the range 64x.
__device__ uint32_t wave_lower_bound(const uint32_t* keys, uint32_t n, uint32_t key) {
  const int lane = lane_id();
  uint32_t lo = 0, hi = n;  // answer in [lo, hi]
  while (hi - lo > 64) {
    uint32_t step = (hi - lo + 63) / 64;
    uint32_t p = lo + (uint32_t)lane * step;
    bool less = (p < hi) && (keys[p] < key);
    unsigned long long m = __ballot(less);
    uint32_t c = (uint32_t)__popcll(m);  // samples < key form a prefix of the lanes
    if (c == 0) return lo;                // keys[lo] >= key
    uint32_t nlo = lo + (c - 1) * step + 1;
    uint32_t nhi = lo + c * step;
    if (nhi > hi) nhi = hi;
    lo = nlo;
    hi = nhi;
  }
  uint32_t p = lo + (uint32_t)lane;
  bool less = (p < hi) && (keys[p] < key);
  return lo + (uint32_t)__popcll(__ballot(less));
}

// ------------------------------------------------------------------ grouping sort
// One pass of a stable LSD counting sort of the batch by symbol id. digit(key) =
// (min(key, clamp) >> shift) & mask over nbins <= 2048 bins (the last pass uses only the bins that
// occur). Three launches: per-tile histograms -> one-workgroup exclusive scan of the histogram
// matrix in bin-major order (= global start of every (bin, tile) run) -> stable scatter.
struct SortPass {
  uint32_t shift, mask, nbins, tile, ntiles, clamp;
};

__device__ __forceinline__ uint32_t sort_digit(uint32_t k, const SortPass& p) {
  if (k > p.clamp) k = p.clamp;
  return (k >> p.shift) & p.mask;
}

// Per-tile histograms, bin-major [bin][tile].
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
  for (uint32_t b = threadIdx.x; b < p.nbins; b += blockDim.x) hist[(size_t)b * p.ntiles + blockIdx.x] = h[b];
  // Per-batch resets folded into the first kernel of the batch.
  if (zero_buf) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < zero_words; i += gridDim.x * blockDim.x)
      zero_buf[i] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) *scratch_top = 0ull;
  }
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

// In-place exclusive scan of the histogram matrix (count = nbins * ntiles), one workgroup of
// 1024 threads: each thread owns a contiguous run, runs are combined by a wave + LDS scan.
__global__ __launch_bounds__(1024) void k_sort_offsets(uint32_t* __restrict__ hist, uint32_t count) {
  __shared__ uint32_t wsum[16];
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t per = (count + 1023) / 1024;
  const uint32_t b0 = tid * per, b1 = min(count, b0 + per);
  uint32_t local = 0;
  for (uint32_t j = b0; j < b1; ++j) local += hist[j];
  uint32_t x = local;
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t t = __shfl_up(x, d, 64);
    if (lane >= d) x += t;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t run = x - local;
  for (uint32_t k = 0; k < w; ++k) run += wsum[k];
  for (uint32_t j = b0; j < b1; ++j) {
    const uint32_t v = hist[j];
    hist[j] = run;
    run += v;
  }
}

// Stable scatter of one tile: dest = start of this tile's run of its digit (k_sort_offsets) +
// rank among equal digits earlier in the tile. Each wave owns a quarter of the tile and ranks
// 64 records at a time with a ballot multisplit (one ballot per digit bit).
__global__ __launch_bounds__(256) void k_sort_scatter(const uint32_t* __restrict__ keys_in,
                                                      const uint32_t* __restrict__ idx_in, uint32_t n, SortPass p,
                                                      uint32_t dbits, const uint32_t* __restrict__ offsets,
                                                      uint32_t* __restrict__ keys_out,
                                                      uint32_t* __restrict__ idx_out) {
  __shared__ uint32_t wcnt[4][1u << MAX_DIGIT_BITS];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t tile = blockIdx.x;
  for (uint32_t b = tid; b < p.nbins; b += 256) wcnt[0][b] = wcnt[1][b] = wcnt[2][b] = wcnt[3][b] = 0;
  __syncthreads();
  const uint32_t t0 = tile * p.tile, t1 = min(n, t0 + p.tile);
  const uint32_t q = p.tile / 4;
  const uint32_t w0 = min(t1, t0 + w * q), w1 = min(t1, w0 + q);
  for (uint32_t i = w0 + lane; i < w1; i += 64) atomicAdd(&wcnt[w][sort_digit(keys_in[i], p)], 1u);
  __syncthreads();
  // per-bin start of each wave's quarter
  for (uint32_t b = tid; b < p.nbins; b += 256) {
    uint32_t run = offsets[(size_t)b * p.ntiles + tile];
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
    uint32_t k = v ? keys_in[i] : 0u;
    if (k > p.clamp) k = p.clamp;
    const uint32_t val = v ? (idx_in ? idx_in[i] : i) : 0u;
    const uint32_t d = (k >> p.shift) & p.mask;
    unsigned long long peers = __ballot(v);
    for (uint32_t bit = 0; bit < dbits; ++bit) {
      const unsigned long long bb = __ballot((d >> bit) & 1u);
      peers &= ((d >> bit) & 1u) ? bb : ~bb;
    }
    const uint32_t rank = (uint32_t)__popcll(peers & lanemask_lt());
    const uint32_t cnt = (uint32_t)__popcll(peers);
    const uint32_t start = v ? wcnt[w][d] : 0u;
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
// Where a wave's view of its symbol's ladder lives: LDS (L <= LDS_MAX_LEVELS, staged in at
// kernel start and written back at the end) or HBM (deep windows).
struct WaveCtx {
  BookDev bk;
  Level* lv;                 // [L] ladder of this symbol (LDS or HBM)
  unsigned long long* occ;   // [L/64] occupancy bitmap
  uint8_t* tend;             // [L] slots written in each level's tail chunk
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

// Smallest occupied level >= x, or L.
__device__ int next_occ(const WaveCtx& c, int x) {
  const int L = (int)c.bk.L;
  if (x >= L) return L;
  if (x < 0) x = 0;
  const unsigned long long* occ = c.occ;
  int w = x >> 6;
  unsigned long long word = occ[w] & (~0ull << (x & 63));
  if (word) return (w << 6) + __builtin_ctzll(word);
  const int lane = lane_id();
  const int nw = (int)c.bk.Lwords;
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
  return L;
}

// Largest occupied level <= x, or -1.
__device__ int prev_occ(const WaveCtx& c, int x) {
  if (x < 0) return -1;
  if (x >= (int)c.bk.L) x = (int)c.bk.L - 1;
  const unsigned long long* occ = c.occ;
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

__device__ __forceinline__ void occ_set(const WaveCtx& c, int lvl) {
  if (lane_id() == 0) c.occ[lvl >> 6] |= (1ull << (lvl & 63));
}
__device__ __forceinline__ void occ_clear(const WaveCtx& c, int lvl) {
  if (lane_id() == 0) c.occ[lvl >> 6] &= ~(1ull << (lvl & 63));
}

__device__ __forceinline__ void set_err(const BookDev& bk, uint32_t bits) {
  if (lane_id() == 0) atomicOr(bk.err, bits);
}

// Free-list push: the popped-next is known without a load.
__device__ __forceinline__ void free_chunk(WaveCtx& c, uint32_t ch) {
  if (lane_id() == 0) c.bk.chdr[ch].next = c.free_head;
  c.free_next = c.free_head;
  c.free_head = ch;
}

// Issue the load of chdr[free_head].next without waiting for it: the value stays in a VGPR and is
// only read (readlane -> s_waitcnt) by the next pop, usually many records later.
__device__ __forceinline__ void prefetch_free_next(WaveCtx& c) {
  const bool ok = c.free_head < c.bk.nchunks;
  const uint32_t v = c.bk.chdr[ok ? c.free_head : 0].next;
  c.free_next = ok ? v : NIL;
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
__device__ __forceinline__ void emit_fills(WaveCtx& c, bool e, unsigned long long taker,
                                           unsigned long long maker, long long price, int qty) {
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
// live iff its qty > 0 (consumed, cancelled and unwritten slots hold 0), so one round trip loads
// a chunk's header and all ME_C slots together; the slots are ranked with one wave prefix scan.
// Exhausted chunks go back to the free list. Returns the new head chunk (NIL: level emptied).
__device__ uint32_t walk_level(WaveCtx& c, int lvl, long long take, uint32_t head, uint32_t tail,
                               unsigned long long taker) {
  const int lane = lane_id();
  const BookDev& bk = c.bk;
  const long long price = c.base + lvl;
  long long need = take;
  uint32_t ch = head;
  while (need > 0) {
    if (ch >= bk.nchunks) {  // NIL or corrupt: never index with it
      set_err(bk, ERR_INCONSISTENT);
      return NIL;
    }
    // issue every load of the chunk before the first use (one round trip, not two)
    const uint32_t nxt_v = bk.chdr[ch].next;
    const bool act = lane < ME_C;
    const size_t g = (size_t)ch * ME_C + (act ? lane : 0);
    const int qv = act ? bk.cqty[g] : 0;
    const unsigned long long sv = act ? bk.cseq[g] : 0ull;
    const long long inc = wave_incl_scan((long long)qv);
    const long long ex = inc - qv;
    long long f = need - ex;
    if (f < 0) f = 0;
    if (f > qv) f = qv;
    const bool fe = f > 0;
    emit_fills(c, fe, taker, sv, price, (int)f);
    if (fe) bk.cqty[g] = qv - (int)f;
    c.resting_delta -= __popcll(__ballot(fe && f == qv));  // makers filled completely leave the book
    const long long live = rli64(inc, 63);
    need -= (need < live ? need : live);
    const unsigned long long alive = __ballot((qv - f) > 0);
    if (!alive) {  // every slot of the chunk is consumed
      free_chunk(c, ch);
      if (ch == tail) {
        if (need > 0) set_err(bk, ERR_INCONSISTENT);
        return NIL;
      }
      ch = rl32(nxt_v, 0);
    } else if (need > 0) {  // impossible: a live slot remains only once the take is met
      set_err(bk, ERR_INCONSISTENT);
      return ch;
    }
  }
  if (ch != head && ch < bk.nchunks && lane == 0) bk.chdr[ch].prev = NIL;  // new FIFO head
  return ch;
}

// Sweep the opposite side for a taker. dir = +1 (BUY: asks upward from best_ask) or
// -1 (SELL: bids downward from best_bid). lim = last level the taker may trade at.
// Lanes cover 64 consecutive levels; an inclusive scan of their totals gives how far the taker
// reaches; fully consumed levels are emptied, the last one partially.
__device__ long long sweep(WaveCtx& c, int dir, int lim, long long want, unsigned long long taker,
                           uint32_t& nfill) {
  const int lane = lane_id();
  const BookDev& bk = c.bk;
  long long rem = want;
  int cur = (dir > 0) ? c.ba : c.bb;
  bool emptied = false;
  const unsigned long long w_start = c.wptr;
  // fast path: the best level alone fills the taker (no window scan)
  if (dir > 0 ? (cur <= lim && cur < (int)bk.L) : (cur >= lim && cur >= 0)) {
    Level B = c.lv[cur];
    const long long btot = rli64(B.total, 0);
    if (btot >= want) {
      const uint32_t head = rl32(B.head, 0), tail = rl32(B.tail, 0);
      STAMP_ADD(c, PH_SWEEP);
      const uint32_t nh = walk_level(c, cur, want, head, tail, taker);
      STAMP_ADD(c, PH_WALK);
      const long long ntot = btot - want;
      if (lane == 0) {
        Level o;
        o.total = ntot;
        o.head = ntot ? nh : NIL;
        o.tail = ntot ? tail : NIL;
        c.lv[cur] = o;
      }
      if (ntot == 0) {
        occ_clear(c, cur);
        wave_mem_order();
        if (dir > 0)
          c.ba = next_occ(c, cur + 1);
        else
          c.bb = prev_occ(c, cur - 1);
      }
      nfill = (uint32_t)(c.wptr - w_start);
      return want;
    }
  }
  while (rem > 0) {
    if (dir > 0 ? (cur > lim || cur >= (int)bk.L) : (cur < lim || cur < 0)) break;
    const int lv = cur + dir * lane;
    const bool valid = (dir > 0) ? (lv <= lim && lv < (int)bk.L) : (lv >= lim && lv >= 0);
    Level L;
    L.total = 0;
    L.head = NIL;
    L.tail = NIL;
    if (valid) L = c.lv[lv];
    const long long tot = L.total;
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
      const uint32_t head = rl32(L.head, t), tail = rl32(L.tail, t);
      STAMP_ADD(c, PH_SWEEP);
      const uint32_t nh = walk_level(c, lvl, take, head, tail, taker);
      STAMP_ADD(c, PH_WALK);
      rem -= take;
      const long long ntot = ltot - take;
      if (lane == 0) {
        Level o;
        o.total = ntot;
        o.head = ntot ? nh : NIL;
        o.tail = ntot ? tail : NIL;
        c.lv[lvl] = o;
      }
      if (ntot == 0) {
        occ_clear(c, lvl);
        emptied = true;
      }
      STAMP_ADD(c, PH_SW_UPDATE);
    }
    if (rem == 0) break;
    // every valid level of this window is now empty; jump to the next occupied one
    const int nxt = cur + dir * 64;
    wave_mem_order();
    if (dir > 0) {
      if (nxt > lim) break;
      cur = next_occ(c, nxt);
    } else {
      if (nxt < lim) break;
      cur = prev_occ(c, nxt);
    }
    STAMP_ADD(c, PH_SW_JUMP);
  }
  if (emptied) {
    wave_mem_order();
    if (dir > 0)
      c.ba = next_occ(c, c.ba);
    else
      c.bb = prev_occ(c, c.bb);
    STAMP_ADD(c, PH_SW_BEST);
  }
  nfill = (uint32_t)(c.wptr - w_start);
  return want - rem;
}

// Append a resting order at the tail of level lvl's FIFO. With the ladder in LDS the common case
// (room in the tail chunk) issues no HBM load at all: the tail fill count lives beside the level.
__device__ bool rest_order(WaveCtx& c, int lvl, unsigned long long seq, int qty, bool buy) {
  const int lane = lane_id();
  const BookDev& bk = c.bk;
  wave_mem_order();
  Level L = c.lv[lvl];
  L.total = rli64(L.total, 0);
  L.head = rl32(L.head, 0);
  L.tail = rl32(L.tail, 0);
  const uint32_t te = rl32((uint32_t)c.tend[lvl], 0);
  uint32_t ch, slot;
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
      h.pad = 0;
      bk.chdr[ch] = h;
      bk.owner[ch] = c.s;
      if (L.tail != NIL) bk.chdr[L.tail].next = ch;
    }
    if (L.tail == NIL) L.head = ch;
    L.tail = ch;
  } else {
    ch = L.tail;
    slot = te;
  }
  const size_t g = (size_t)ch * ME_C + slot;
  const bool was_empty = (L.total == 0);
  L.total += qty;
  if (lane == 0) {
    bk.cseq[g] = seq;
    bk.cqty[g] = qty;
    c.lv[lvl] = L;
    c.tend[lvl] = (uint8_t)(slot + 1);
    if (seq < bk.max_seq) bk.loc[seq] = (uint32_t)g;
  }
  if (was_empty) occ_set(c, lvl);
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
__device__ int cancel_order(WaveCtx& c, unsigned long long tgt) {
  const BookDev& bk = c.bk;
  const int lane = lane_id();
  if (tgt == 0ull || tgt >= bk.max_seq) return 0;
  wave_mem_order();
  const uint32_t g = rl32(bk.loc[tgt], 0);
  if (g == NIL) return 0;
  const uint32_t ch = g / ME_C, slot = g % ME_C;
  if (ch >= bk.nchunks) return 0;
  // one round trip: owner, header, the whole chunk's quantities and the target seq
  const uint32_t owner = rl32(bk.owner[ch], 0);
  const ChunkHdr hd = bk.chdr[ch];
  const bool act = lane < ME_C;
  const int qv = act ? bk.cqty[(size_t)ch * ME_C + lane] : 0;
  const unsigned long long sq = rl64(bk.cseq[g], 0);
  if (owner != c.s) return 0;  // another symbol's order: never touch its book
  const int q = rli32(qv, (int)slot);
  if (sq != tgt || q <= 0) return 0;
  const int lvl = (int)rl32(hd.level, 0);
  const uint32_t nxt = rl32(hd.next, 0), prv = rl32(hd.prev, 0);
  if (lvl < 0 || lvl >= (int)bk.L) {
    set_err(bk, ERR_INCONSISTENT);
    return 0;
  }
  const uint32_t live_after = (uint32_t)__popcll(__ballot(qv > 0)) - 1;
  Level L = c.lv[lvl];
  L.total = rli64(L.total, 0) - q;
  L.head = rl32(L.head, 0);
  L.tail = rl32(L.tail, 0);
  if (L.tail >= bk.nchunks || L.head >= bk.nchunks) {
    set_err(bk, ERR_INCONSISTENT);
    return q;
  }
  if (lane == 0) bk.cqty[g] = 0;
  if (L.total == 0) {
    // splice the whole (now dead) FIFO onto the free list
    if (lane == 0) bk.chdr[L.tail].next = c.free_head;
    c.free_next = (L.head == L.tail) ? c.free_head : NIL;
    c.free_head = L.head;
    if (L.head != L.tail) prefetch_free_next(c);
    L.head = NIL;
    L.tail = NIL;
    if (lane == 0) c.lv[lvl] = L;
    occ_clear(c, lvl);
    wave_mem_order();
    if (lvl == c.bb) c.bb = prev_occ(c, lvl);
    if (lvl == c.ba) c.ba = next_occ(c, lvl);
  } else if (live_after == 0) {
    // unlink the dead chunk (the level keeps live orders elsewhere, so ch is not both ends)
    uint32_t nh = L.head, nt = L.tail;
    if (ch == L.head) {
      nh = nxt;
      if (lane == 0) bk.chdr[nxt].prev = NIL;
    } else if (ch == L.tail) {
      nt = prv;
      if (lane == 0) {
        bk.chdr[prv].next = NIL;
        c.tend[lvl] = (uint8_t)ME_C;  // a non-tail chunk is always full
      }
    } else if (lane == 0) {
      bk.chdr[prv].next = nxt;
      bk.chdr[nxt].prev = prv;
    }
    L.head = nh;
    L.tail = nt;
    if (lane == 0) c.lv[lvl] = L;
    free_chunk(c, ch);
  } else {
    if (lane == 0) c.lv[lvl] = L;
  }
  c.resting_delta -= 1;
  return q;
}

__device__ __forceinline__ void write_result(const BatchDev& bt, uint32_t i, int filled, int remaining,
                                             uint32_t nfill, uint8_t status, uint8_t reason,
                                             unsigned long long fstart) {
  if (lane_id() == 0) {
    me_order_result r;
    r.filled_qty = filled;
    r.remaining_qty = remaining;
    r.fill_count = nfill;
    r.tape_offset = 0;
    r.status = status;
    r.reason = reason;
    r.pad[0] = 0;
    r.pad[1] = 0;
    bt.res[i] = r;
    bt.fstart[i] = (uint32_t)fstart;
    if (nfill) atomicAdd(&bt.tile_sum[i / TILE_TAPE], nfill);
  }
}

// Bytes of LDS one wave needs to hold its symbol's ladder (levels + occupancy + tail fill).
__host__ __device__ constexpr size_t lds_wave_bytes(uint32_t L) {
  return (size_t)L * sizeof(Level) + (size_t)(L / 64) * 8 + (size_t)L;
}

// One wavefront per symbol (4 per workgroup). Block s/4, wave s%4. Symbol S is the reject bin
// of records whose symbol id is out of range. kLds: the symbol's ladder is staged in LDS.
template <bool kLds>
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
    for (uint32_t j = lo + lane; j < hi; j += 64) {
      uint32_t i = bt.perm[j];
      me_order_result r;
      r.filled_qty = 0;
      r.remaining_qty = 0;
      r.fill_count = 0;
      r.tape_offset = 0;
      r.status = ME_ST_REJECTED;
      r.reason = ME_RJ_BAD_SYMBOL;
      r.pad[0] = r.pad[1] = 0;
      bt.res[i] = r;
      bt.fstart[i] = 0;
    }
    return;
  }
  const uint32_t L = bk.L;
  Level* g_lv = bk.levels + (size_t)s * L;
  unsigned long long* g_occ = bk.occ + (size_t)s * bk.Lwords;
  uint8_t* g_tend = bk.tend + (size_t)s * L;
  WaveCtx c;
#ifdef ME_STAMPS
  for (int p = 0; p < PH_N; ++p) c.st[p] = 0;
  STAMP_MARK(c);
#endif
  c.bk = bk;
  c.s = s;
  if (kLds) {
    unsigned char* base = smem + (size_t)wv * lds_wave_bytes(L);
    c.lv = (Level*)base;
    c.occ = (unsigned long long*)(base + (size_t)L * sizeof(Level));
    c.tend = base + (size_t)L * sizeof(Level) + (size_t)(L / 64) * 8;
    for (uint32_t i = lane; i < L; i += 64) {
      c.lv[i] = g_lv[i];
      c.tend[i] = g_tend[i];
    }
    for (uint32_t i = lane; i < bk.Lwords; i += 64) c.occ[i] = g_occ[i];
    wave_mem_order();
  } else {
    c.lv = g_lv;
    c.occ = g_occ;
    c.tend = g_tend;
  }
  c.gs = bk.gsym ? bk.gsym[s] : s;
  const SymState st = bk.sym[s];
  c.base = rli64(st.base, 0);
  c.bb = rli32(st.best_bid, 0);
  c.ba = rli32(st.best_ask, 0);
  c.free_head = rl32(st.free_head, 0);
  prefetch_free_next(c);
  c.bump_cur = c.bump_end = 0;
  c.resting_delta = 0;
  c.scratch = bt.scratch;
  // scratch run of this wave: fills <= resting makers + 2 * records
  const unsigned long long need = (unsigned long long)rl32(st.resting, 0) + 2ull * (hi - lo);
  unsigned long long w0 = 0;
  if (lane == 0) w0 = atomicAdd(bt.scratch_top, need);
  w0 = rl64(w0, 0);
  if (w0 + need > bt.scratch_cap) {
    set_err(bk, ERR_SCRATCH_OOM);
    return;
  }
  c.wptr = w0;
  STAMP_ADD(c, PH_PROLOGUE);
  const long long Lw = (long long)L;

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
    STAMP_ADD(c, PH_FETCH);
    for (uint32_t k = 0; k < cnt; ++k) {
      const uint32_t i = rl32(oi, (int)k);
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
          write_result(bt, i, 0, got, 0, ME_ST_CANCELED, ME_RJ_NONE, fstart);
        else
          write_result(bt, i, 0, 0, 0, ME_ST_REJECTED, ME_RJ_UNKNOWN_ORDER, fstart);
        continue;
      }
      if (q <= 0) {
        write_result(bt, i, 0, 0, 0, ME_ST_REJECTED, ME_RJ_BAD_QTY, fstart);
        continue;
      }
      if (side != ME_SIDE_BUY && side != ME_SIDE_SELL) {
        write_result(bt, i, 0, q, 0, ME_ST_REJECTED, ME_RJ_BAD_SIDE, fstart);
        continue;
      }
      int li = 0;
      if (!market) {
        if (px < c.base || (unsigned long long)px - (unsigned long long)c.base >= (unsigned long long)Lw) {
          write_result(bt, i, 0, q, 0, ME_ST_REJECTED, ME_RJ_OUT_OF_WINDOW, fstart);
          continue;
        }
        li = (int)(px - c.base);
      }
      if (seq == 0ull || seq >= bk.max_seq) {
        write_result(bt, i, 0, q, 0, ME_ST_REJECTED, ME_RJ_BAD_SEQ, fstart);
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
        const bool rested = rem > 0 && !rest_order(c, li, seq, rem, buy);
        STAMP_ADD(c, PH_REST);
        if (rested) {
          ok = false;  // chunk pool exhausted: the batch fails (sticky error word)
          break;
        }
        stt = rem == 0 ? ME_ST_FILLED : (filled > 0 ? ME_ST_PARTIALLY_FILLED : ME_ST_NEW);
      }
      write_result(bt, i, filled, rem, nfill, stt, ME_RJ_NONE, fstart);
      STAMP_ADD(c, PH_RESULT);
    }
  }
  // return unused bump-reserved chunks to this symbol's free list
  while (c.bump_cur < c.bump_end) free_chunk(c, c.bump_cur++);
  if (kLds) {
    wave_mem_order();
    for (uint32_t i = lane; i < L; i += 64) {
      g_lv[i] = c.lv[i];
      g_tend[i] = c.tend[i];
    }
    for (uint32_t i = lane; i < bk.Lwords; i += 64) g_occ[i] = c.occ[i];
  }
  if (lane == 0) {
    SymState o;
    o.base = c.base;
    o.best_bid = c.bb;
    o.best_ask = c.ba;
    o.free_head = c.free_head;
    o.resting = (uint32_t)((int)st.resting + c.resting_delta);
    o.pad[0] = o.pad[1] = 0;
    bk.sym[s] = o;
  }
#ifdef ME_STAMPS
  STAMP_ADD(c, PH_EPILOGUE);
  if (lane == 0 && bk.dbg)
    for (int p = 0; p < PH_N; ++p) bk.dbg[(size_t)s * 16 + p] = c.st[p];
#endif
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
                            uint32_t clamp_key, int shift, int dbits, uint32_t* hist, uint32_t* keys_out,
                            uint32_t* idx_out, uint32_t* zero_buf, uint32_t zero_words,
                            unsigned long long* scratch_top) {
  SortPass p;
  p.shift = (uint32_t)shift;
  p.mask = (1u << dbits) - 1u;
  p.nbins = min(1u << dbits, (clamp_key >> shift) + 1u);
  p.tile = sort_tile(n);
  p.ntiles = (n + p.tile - 1) / p.tile;
  p.clamp = clamp_key;
  hipLaunchKernelGGL(k_sort_hist, dim3(p.ntiles), dim3(256), 0, st, keys_in, n, p, hist, zero_buf, zero_words,
                     scratch_top);
  hipLaunchKernelGGL(k_sort_offsets, dim3(1), dim3(1024), 0, st, hist, p.nbins * p.ntiles);
  hipLaunchKernelGGL(k_sort_scatter, dim3(p.ntiles), dim3(256), 0, st, keys_in, idx_in, n, p, (uint32_t)dbits, hist,
                     keys_out, idx_out);
  return hipGetLastError();
}

hipError_t launch_match(hipStream_t st, const BookDev& bk, const BatchDev& bt) {
  const uint32_t waves = bk.S + 1;
  const dim3 grid((waves + 3) / 4), block(256);
  if (bk.L <= LDS_MAX_LEVELS) {
    const size_t lds = 4 * lds_wave_bytes(bk.L);
    hipLaunchKernelGGL(k_match<true>, grid, block, lds, st, bk, bt);
  } else {
    hipLaunchKernelGGL(k_match<false>, grid, block, 0, st, bk, bt);
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

hipError_t launch_init_levels(hipStream_t st, Level* levels, size_t count) {
  size_t blocks = (count + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL(k_init_levels, dim3((uint32_t)blocks), dim3(256), 0, st, levels, count);
  return hipGetLastError();
}

}  // namespace me

// me_agg.hip — hot symbols of deep windows in aggregate form (DESIGN.md §4 "k_agg").
//
// A hot symbol (config 4's Zipf head, config 1's single book) is one serial chain of records, so
// whatever one record costs on its wave sets the launch length. Price-time priority splits that cost
// in two parts of very different shape:
//
//   * WHICH levels a taker takes from, how much from the last one, and where a remainder rests
//     depend only on the level TOTALS — a serial chain, but a short one: k_agg_walk runs it on one
//     wave per hot symbol with the top of each side as a 64-lane list of (level, total), no chunk,
//     no FIFO, no fill in the chain. Each record appends "take q from level l" / "rest q at level l"
//     events to a log.
//   * WHICH makers a take consumed is FIFO bookkeeping inside one level: in the level's maker
//     space (the initial FIFO's live orders, then this batch's rests in record order, each an
//     interval of its quantity) the takes of the batch cover [0, C) in order, so the fills are the
//     overlaps of two interval partitions — independent across levels, resolved for all levels at
//     once after the walk (k_agg_levels, k_agg_place), and written where the tape job expects them.
//
// Kernels (the engine's hot stream, after k_hot_pick, beside k_match on the main stream):
//   k_agg_walk    one wave per hot symbol: the level-total chain, the event log, the records' status
//   k_agg_group   one workgroup per hot symbol: a stable counting sort of its log by level -> segments
//   k_agg_sorted  the sorted log entries (every slot over the whole grid)
//   k_agg_levels  one wave per (symbol, level) segment: quantity taken, initial-FIFO walk, consumed
//                 makers, emptied chunks (zeroed), each take's first maker and fill count
//   k_agg_alloc   one wave per hot symbol: chunks for the surviving rests — the symbol's own emptied
//                 chunks first, then its free list, then the bump allocator; the surplus freed
//   k_agg_place   one wave per segment: surviving rests into the level's tail / new chunks, seq ring
//   k_agg_fin     one workgroup per hot symbol: fill offsets (scan over the log), symbol state, the
//                 continuation's scratch position
//   k_agg_out     every take event over the whole grid: the records' fill counts and scratch starts,
//                 the fills into the scratch run, in tape order
// A record the walk does not cover (a cancel, a LIMIT outside the window, a MARKET while far levels
// exist on the side it crosses) hands the symbol's remaining records to k_match_hot_cont, the generic
// record loop, exactly as k_match_hot does; the HBM book is complete before it runs.
// Same semantics and HBM layout as k_match (me_kernels.hip); parity: tests/test_hot_path.py.
#include "me_wave.hpp"
#include "me_far.hpp"  // old_lookup (k_agg_gwalk_cx)

#include <cstdlib>

namespace me {
namespace {

constexpr uint32_t AGG_WORDS = AGG_MAX_L / 64;
#ifndef ME_WALK_PRIO
#define ME_WALK_PRIO 1  // s_setprio(3) on the walking waves (0: off; profiles/r5/prio)
#endif
#ifndef ME_LIST_EMIT
#define ME_LIST_EMIT 0  // the list walk's event staging: 0 LDS (one 16-B lane-0 write per event), 1 VGPR lanes
#endif
// M0 is set only by this file's v_writelane sequences (no LDS-direct, GWS or interpolation use here)
#pragma clang diagnostic ignored "-Winline-asm"

constexpr uint32_t AGG_GCHUNK = 8192;  // log keys k_agg_group stages in LDS per scatter chunk (16 KB)
constexpr int AGG_VMCNT0 = 0x0F70;     // s_waitcnt immediate: vmcnt(0) only (gfx9 encoding)

__device__ __forceinline__ int auni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t auniu(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

__device__ __forceinline__ void a_set_err(const BookDev& bk, uint32_t bits) {
  if (lane_id() == 0) atomicOr(bk.err, bits);
}
// Slots of the launch: every symbol (grouped launches) or k_hot_pick's hot symbols.
__device__ __forceinline__ uint32_t a_nslots(const BookDev& bk, const AggDev& ag) {
  return ag.nslots ? ag.nslots : min(*(volatile uint32_t*)bk.hcount, bk.S);
}

// lane i <- lane i - 1 (gfx9 DPP wave_ror:1): an entry enters mid-list by rotating the ones behind it
__device__ __forceinline__ uint32_t a_up(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x13C, 0xf, 0xf, false);
}
__device__ __forceinline__ long long a_up64(long long v) {
  return (long long)(((unsigned long long)a_up((uint32_t)((unsigned long long)v >> 32)) << 32) |
                     a_up((uint32_t)v));
}
// lane `l` of `old` <- the uniform value v (one compare, shared by the fields written for the same
// lane, and a select per 32 bits; gfx9's v_writelane cannot take both operands from SGPRs)
__device__ __forceinline__ uint32_t a_wlu(uint32_t old, uint32_t v, int l) { return lane_id() == l ? v : old; }
__device__ __forceinline__ int a_wl(int old, int v, int l) { return (int)a_wlu((uint32_t)old, (uint32_t)v, l); }
__device__ __forceinline__ long long a_wl64(long long old, long long v, int l) {
  const uint32_t lo = a_wlu((uint32_t)old, (uint32_t)v, l);
  const uint32_t hi = a_wlu((uint32_t)((unsigned long long)old >> 32), (uint32_t)((unsigned long long)v >> 32), l);
  return (long long)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ void a_drain() {
  __builtin_amdgcn_s_waitcnt(0);
  wave_mem_order();
}

// Diagnostic build (-DME_STAMPS): absolute s_memtime stamps per symbol into bk.dbg[s * 24 + 16 + k]
// (16 walk start, 17 walk end, 18 k_agg_gres start, 19..23 its phases A, B, C, D1, D2 done), read by
// tools/gres_probe.py. The product build compiles them away.
#ifdef ME_STAMPS
#define GR_STAMP(bk, s, k) \
  do { if (threadIdx.x == 0) (bk).dbg[(size_t)(s) * 24u + 16u + (k)] = stamp_now(); } while (0)
// The grouped walk's cycles per symbol by part, accumulated (dbg[s * 24 + 0..3]: batch set-up — bucket
// loads, staging, sort —, block set-up and results, the record loop, records walked)
#define GW_T(k)                                  \
  do {                                           \
    const unsigned long long _n = stamp_now();   \
    gw_t[k] += _n - gw_m;                        \
    gw_m = _n;                                   \
  } while (0)
#else
#define GR_STAMP(bk, s, k) ((void)0)
#define GW_T(k) ((void)0)
#endif

// ------------------------------------------------------------------ the level-total walk
// Top of one side, best first: a ring over the lanes, entry i in lane (f + i) & 63. Side coordinates:
// asks m = level, bids m = L - 1 - level, so "better" is "smaller" on both sides. The list is always
// the exact prefix of the side's occupied window levels (an empty list = an empty side); `more`: there
// may be occupied levels beyond the last entry.
struct AList {
  int m;          // lane: side coordinate of the entry
  long long tot;  // lane: its live quantity (authoritative while listed; HBM's copy is stale)
  int f, n, more; // wave-uniform
};

struct AWalk {
  gptr<Level> lv;
  gptr<unsigned long long> occ;
  gptr<AggEv> ev;
  unsigned long long* locc;  // LDS copy of the occupancy bitmap (both sides)
  uint32_t evp;              // next log index (the slot's log starts 64-aligned)
  int L, W;
#if ME_LIST_EMIT
  // the log's current 64-event block, event i in lane i of three VGPRs (v_writelane, as the ladder walk's
  // LEv): one coalesced 1-KB store per 64 events
  uint32_t vl, vj, vq;
#else
  // the log's current 64-event block, event i in lane i: stored by the whole wave when it fills (one
  // coalesced 1-KB store instead of a lane-0 store per event)
  AggEv* stg;  // LDS [128]: the block's events by log index mod 64, then the other lanes' dummy slots
#endif
};

__device__ __forceinline__ int a_side_lvl(int L, int k, int m) { return k ? m : L - 1 - m; }

#if ME_LIST_EMIT
// Lanes [0, n) of the staged block to log indices [base, base + n).
__device__ __forceinline__ void a_evstore(const AWalk& w, uint32_t base, uint32_t n) {
  AggEv e;
  e.lvl = w.vl;
  e.j = w.vj;
  e.qty = (int)w.vq;
  e.pad = 0u;
  if ((uint32_t)lane_id() < n) w.ev[base + (uint32_t)lane_id()] = e;
}
// The event into lane evp & 63 of the staging VGPRs (three v_writelane, no LDS traffic; the block leaves
// as one coalesced store when it fills). lvl, jt and q are wave-uniform.
__device__ __forceinline__ void a_emit(AWalk& w, int lvl, uint32_t jt, int q) {
  const uint32_t slot = w.evp & 63u;
  asm volatile(
      "s_mov_b32 m0, %3\n\tv_writelane_b32 %0, %4, m0\n\tv_writelane_b32 %1, %5, m0\n\tv_writelane_b32 %2, %6, m0"
      : "+v"(w.vl), "+v"(w.vj), "+v"(w.vq)
      : "s"(slot), "s"(auniu((uint32_t)lvl)), "s"(auniu(jt)), "s"(auniu((uint32_t)q))
      : "m0");
  w.evp += 1;
  if (ME_UNLIKELY(slot == 63u)) a_evstore(w, w.evp - 64u, 64u);
}

#else
// Lanes [0, n) of the staged block to log indices [base, base + n).
__device__ __forceinline__ void a_evstore(const AWalk& w, uint32_t base, uint32_t n) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (a wave's LDS operations complete in order)
  const AggEv e = w.stg[lane_id()];
  if ((uint32_t)lane_id() < n) w.ev[base + (uint32_t)lane_id()] = e;
}
// The event into the LDS block (one 16-B write by lane 0; the other lanes write their dummy slots, so no
// exec change), one coalesced 1-KB store per 64 events.
__device__ __forceinline__ void a_emit(AWalk& w, int lvl, uint32_t jt, int q) {
  const int lane = lane_id();
  AggEv e;
  e.lvl = (uint32_t)lvl;
  e.j = jt;
  e.qty = q;
  e.pad = 0;
  AggEv* p = lane == 0 ? &w.stg[w.evp & 63u] : &w.stg[64 + lane];
  *p = e;
  w.evp += 1;
  if (ME_UNLIKELY((w.evp & 63u) == 0u)) a_evstore(w, w.evp - 64u, 64u);
}

#endif
// Occupancy: non-returning atomics on the LDS copy and on HBM (nothing in the chain waits for them).
__device__ __forceinline__ void a_occ(AWalk& w, int lvl, bool on) {
  const uint32_t wi = (uint32_t)lvl >> 6;
  const unsigned long long bit = 1ull << (lvl & 63);
  if (lane_id() == 0) {
    if (on) {
      __atomic_fetch_or(&w.locc[wi], bit, __ATOMIC_RELAXED);
      __atomic_fetch_or(&w.occ[wi], bit, __ATOMIC_RELAXED);
    } else {
      __atomic_fetch_and(&w.locc[wi], ~bit, __ATOMIC_RELAXED);
      __atomic_fetch_and(&w.occ[wi], ~bit, __ATOMIC_RELAXED);
    }
  }
}

// The r-th (0-based) set bit of w (w has more than r set bits).
__device__ __forceinline__ uint32_t a_nth_set(unsigned long long w, uint32_t r) {
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

// Lanes 0..n-1 <- the first (up to) 64 occupied levels from window level `start` going up (K = 1) or
// down (K = 0), from the LDS occupancy copy; *more: the list filled before the window ended.
template <int K>
__device__ int a_scan(const AWalk& w, int start, int& out_lvl, int& more) {
  const int lane = lane_id();
  out_lvl = -1;
  more = 0;
  if (start < 0 || start >= w.L) return 0;
  int found = 0;
  const int w0 = start >> 6;
  for (int b = 0;; b += 64) {
    const int wi = K ? w0 + b + lane : w0 - b - lane;
    const bool in = wi >= 0 && wi < w.W;
    unsigned long long x = in ? w.locc[wi] : 0ull;
    if (wi == w0) x &= K ? (~0ull << (start & 63)) : (~0ull >> (63 - (start & 63)));
    if (!K) x = __builtin_bitreverse64(x);  // descending: bit 0 = the word's highest level
    const uint32_t c = (uint32_t)__popcll(x);
    const long long inc = wave_incl_scan((long long)c);
    const uint32_t ex = (uint32_t)(inc - c);
    const uint32_t tot = (uint32_t)rli64(inc, 63);
    const int i = lane - found;  // output lane i takes bit (i - ex_j) of the lane j holding it
    int lo = 0;
#pragma unroll
    for (int st = 32; st >= 1; st >>= 1) {
      const uint32_t e = (uint32_t)__shfl((int)ex, min(lo + st, 63), 64);
      if (lo + st < 64 && (int)e <= i) lo += st;
    }
    const unsigned long long wj = (unsigned long long)__shfl((long long)x, lo, 64);
    const uint32_t r = (uint32_t)(i - __shfl((int)ex, lo, 64));
    const uint32_t bpos = a_nth_set(wj, r);
    const int wdx = K ? w0 + b + lo : w0 - b - lo;
    if (i >= 0 && (uint32_t)i < tot) out_lvl = wdx * 64 + (K ? (int)bpos : 63 - (int)bpos);
    found = min(found + (int)tot, 64);
    const bool end = K ? (w0 + b + 64 >= w.W) : (w0 - b - 64 < 0);
    if (found >= 64) {
      more = 1;  // conservative: a later rebuild finds out
      return 64;
    }
    if (end) return found;
  }
}

// Rebuild list S from side coordinate start_m (the best, or a bound no level of either side lies
// inside): occupancy scan in LDS, the totals in one round trip. The caller has flushed the list's own
// totals and waited for every store.
template <int K>
__device__ __forceinline__ void a_rebuild(AWalk& w, AList& S, int start_m) {
  const int lane = lane_id();
  int lvl = -1, more = 0, n = 0;
  if (start_m < w.L) {
    const int sm = start_m < 0 ? 0 : start_m;
    n = a_scan<K>(w, K ? sm : w.L - 1 - sm, lvl, more);
  }
  const bool v = lane < n;
  long long t = 0;
  if (v) t = w.lv[lvl].total;
  // wait here, on the rare path: otherwise the list registers carry a possibly pending load into the
  // record loop, and every read of them there waits vmcnt(0) — which, gfx9 counting loads and stores in
  // one in-order counter, also waits for every store the chain has issued (~1 us per record measured)
  __builtin_amdgcn_s_waitcnt(AGG_VMCNT0);
  S.m = v ? a_side_lvl(w.L, K, lvl) : w.L;
  S.tot = t;
  S.f = 0;
  S.n = auni(n);
  S.more = auni(more);
}

// The listed totals back to HBM (before a rebuild re-reads them, and at the end).
__device__ __forceinline__ void a_flush(AWalk& w, const AList& S, int K) {
  const int rel = (lane_id() - S.f) & 63;
  if (rel < S.n) w.lv[a_side_lvl(w.L, K, S.m)].total = S.tot;
}

// Take up to rem from list O (side K) while its front crosses lim (side coordinates): one event per
// level taken from; a level taken whole leaves the list (the front moves) and the book.
template <int K>
__device__ __forceinline__ void a_take(AWalk& w, AList& O, int lim, uint32_t& rem, uint32_t jt) {
  const int lane = lane_id();
  while (rem && O.n) {
    const int f = O.f;
    const int m0 = rli32(O.m, f);
    if (m0 > lim) break;
    const long long tot = rli64(O.tot, f);
    const int lvl = a_side_lvl(w.L, K, m0);
    if ((long long)rem < tot) {
      O.tot = a_wl64(O.tot, tot - (long long)rem, f);
      a_emit(w, lvl, jt, (int)rem);
      rem = 0;
      break;
    }
    a_emit(w, lvl, jt, (int)tot);
    rem -= (uint32_t)tot;
    if (lane == 0) w.lv[lvl].total = 0;
    a_occ(w, lvl, false);
    O.f = (f + 1) & 63;
    O.n -= 1;
    if (ME_UNLIKELY(!O.n && O.more)) {
      // ran dry with levels beyond it: rebuild now, so that an empty list always means an empty side
      a_drain();
      a_rebuild<K>(w, O, m0 + 1);
    }
  }
}

// Rest q at side coordinate mm (window level lvl) on list M (side K).
template <int K>
__device__ __forceinline__ void a_rest(AWalk& w, AList& M, int mm, int lvl, int q, uint32_t jt) {
  const int lane = lane_id();
  const int rel = (lane - M.f) & 63;
  const bool ent = rel < M.n;
  const int p = __popcll(__ballot(ent && M.m < mm));  // entries better than the level
  if (p < M.n) {
    const int j = (M.f + p) & 63;
    if (rli32(M.m, j) == mm) {  // a listed level: its total grows
      M.tot = a_wl64(M.tot, rli64(M.tot, j) + q, j);
      a_emit(w, lvl, jt, q);
      return;
    }
  }
  if (p < M.n || (!M.more && p < 64)) {
    // an empty level inside the list's span (or past its end when nothing lies beyond): it enters at
    // position p; the entries behind it move one lane up (a full list drops its last entry)
    if (M.n == 64) {
      const int jl = (M.f + 63) & 63;
      if (lane == jl) w.lv[a_side_lvl(w.L, K, M.m)].total = M.tot;
      __builtin_amdgcn_s_waitcnt(0);  // a later rest there is an atomic behind this store
      M.n = 63;
      M.more = 1;
    }
    int j;
    if (p == 0) {  // a new best: the front moves one lane back
      M.f = (M.f - 1) & 63;
      j = M.f;
    } else {
      j = (M.f + p) & 63;
      const bool up = rel > p && rel <= M.n;
      const int um = (int)a_up((uint32_t)M.m);
      const long long ut = a_up64(M.tot);
      M.m = up ? um : M.m;
      M.tot = up ? ut : M.tot;
    }
    M.m = a_wl(M.m, mm, j);
    M.tot = a_wl64(M.tot, (long long)q, j);
    M.n += 1;
    a_occ(w, lvl, true);
  } else {
    // deep (beyond the list's last entry): the HBM total grows by a non-returning atomic
    if (lane == 0) __atomic_fetch_add(&w.lv[lvl].total, (long long)q, __ATOMIC_RELAXED);
    a_occ(w, lvl, true);
    M.more = 1;
  }
  a_emit(w, lvl, jt, q);
}

// The slot's regions of the consumed-maker list and of the chunk-id pool, sized by the slot's fill bound
// (consumed makers <= fills <= resting makers + 2 * records): the per-level kernels then reserve from
// the slot's own cursors (no pool-wide atomic per level). False: the pools are full.
__device__ __forceinline__ bool a_reserve(const AggDev& ag, gptr<AggSlot> slot, uint32_t resting, uint32_t cnt) {
  const unsigned long long mkb = (unsigned long long)resting + 2ull * cnt + 64ull;
  const unsigned long long frb = 2ull * mkb + cnt + 64ull;
  uint32_t mb = 0, fb = 0;
  if (lane_id() == 0) {
    mb = atomicAdd(&ag.ctr[AC_MK], (uint32_t)mkb);
    fb = atomicAdd(&ag.ctr[AC_FR], (uint32_t)frb);
    slot->mk_base = mb;
    slot->mk_cur = 0u;
    slot->fr_base = fb;
    slot->fr_cur = 0u;
  }
  mb = rl32(mb, 0);
  fb = rl32(fb, 0);
  return mb + mkb <= (unsigned long long)ag.mk_cap && fb + frb <= (unsigned long long)ag.fr_cap;
}


// Reject reason (k_match's, in its order; cancels are the generic loop's) and whether the walk covers
// the record: not a cancel, and a LIMIT inside the window or a MARKET while the side it crosses has no
// far levels.
__device__ __forceinline__ bool a_classify(bool v, unsigned long long oseq, long long opx, int oq, uint32_t okd,
                                           long long base, int L, uint32_t nfar0, uint32_t nfar1, uint32_t& rj,
                                           int& olm) {
  const uint32_t side = okd & 3u;
  const bool market = (okd >> 2) & 1u, cancel = (okd >> 3) & 1u;
  rj = oq <= 0                                          ? (uint32_t)ME_RJ_BAD_QTY
       : (side != ME_SIDE_BUY && side != ME_SIDE_SELL) ? (uint32_t)ME_RJ_BAD_SIDE
       : oseq == 0ull                                   ? (uint32_t)ME_RJ_BAD_SEQ
                                                        : 0u;
  const unsigned long long off = (unsigned long long)opx - (unsigned long long)base;
  const bool inw = off < (unsigned long long)L;
  const bool farx = (side == ME_SIDE_BUY ? nfar1 : nfar0) != 0u;
  olm = (int)off;
  return v && !cancel && (rj != 0u || (market ? !farx : inw));
}

// A list running low with levels beyond it is rebuilt at a block start (its totals flushed first).
__device__ __forceinline__ void a_refill(AWalk& w, AList& A, AList& B) {
  if (A.n < 32 && A.more) {
    a_flush(w, A, 1);
    a_drain();
    a_rebuild<1>(w, A, rli32(A.m, A.f));
  }
  if (B.n < 32 && B.more) {
    a_flush(w, B, 0);
    a_drain();
    a_rebuild<0>(w, B, rli32(B.m, B.f));
  }
}

// A record's control word (lw_cw): its level (LIMIT) or last level a taker may trade at (MARKET: the window's
// far end), side, type, reject reason.
constexpr uint32_t LW_BUY = 1u << 15, LW_MKT = 1u << 16, LW_RJ_SHIFT = 17, LW_LIM = 0x7FFFu;

// The serial chain over records [0, cnt) of a block in vector form (lane k = record k: quantity and the
// control word of lw_cw — window level / a taker's last level, side, type, reject reason); record k's log
// id is jb + k. Returns the records it walked (fewer than cnt when record k is one the walk does not cover:
// fastm bit clear); rr lane k = record k's remainder.
__device__ __forceinline__ uint32_t a_block(AWalk& w, AList& A, AList& B, int oq, uint32_t ocw, uint32_t jb,
                                            unsigned long long fastm, uint32_t cnt, int& rr) {
  const int L = w.L;
  uint32_t k = 0;
  for (; k < cnt; ++k) {
    if (ME_UNLIKELY(!((fastm >> k) & 1ull))) break;
    const uint32_t cw = rl32(ocw, (int)k);
    if (ME_UNLIKELY((cw >> LW_RJ_SHIFT) != 0u)) continue;  // rejected: no chain work (a_result: from cw)
    const uint32_t jt = jb + k;
    uint32_t rem = (uint32_t)rli32(oq, (int)k);
    const int lm = (int)(cw & LW_LIM);
    const bool mkt = (cw & LW_MKT) != 0u;
    if (cw & LW_BUY) {
      a_take<1>(w, A, lm, rem, jt | AGG_TAKE);  // (a MARKET's lm is the window's far end)
      if (!mkt && rem) a_rest<0>(w, B, L - 1 - lm, lm, (int)rem, jt);
    } else {
      a_take<0>(w, B, L - 1 - lm, rem, jt | AGG_TAKE);
      if (!mkt && rem) a_rest<1>(w, A, lm, lm, (int)rem, jt);
    }
    asm volatile("s_mov_b32 m0, %1\n\tv_writelane_b32 %0, %2, m0" : "+v"(rr) : "s"(k), "s"(auniu(rem)) : "m0");
  }
  return k;
}

__device__ __forceinline__ void a_walk_init(AWalk& w, const BookDev& bk, const AggDev& ag, uint32_t s, uint32_t eb,
                                            unsigned long long* locc, AggEv* stg) {
  w.lv = (gptr<Level>)vptr(bk.levels + (size_t)s * bk.L);
  w.occ = (gptr<unsigned long long>)vptr(bk.occ + (size_t)s * bk.Lwords);
  w.ev = (gptr<AggEv>)vptr(ag.ev);
  w.locc = locc;
  w.evp = eb;
#if ME_LIST_EMIT
  w.vl = w.vj = w.vq = 0u;
#else
  w.stg = stg;
#endif
  w.L = (int)bk.L;
  w.W = (int)bk.Lwords;
  for (int k = lane_id(); k < w.W; k += 64) locc[k] = w.occ[k];
  wave_mem_order();
}

// The walk's end: the staged log tail and the listed totals to HBM; the best levels.
__device__ __forceinline__ void a_walk_end(AWalk& w, AList& A, AList& B, int& bb, int& ba) {
  if (w.evp & 63u) a_evstore(w, w.evp & ~63u, w.evp & 63u);
  a_flush(w, A, 1);
  a_flush(w, B, 0);
  ba = A.n ? rli32(A.m, A.f) : w.L;
  bb = B.n ? w.L - 1 - rli32(B.m, B.f) : -1;
}

// ------------------------------------------------------------------ the ladder walk
// The level totals live in LDS as 32-bit words indexed by level (128 KB at L = 32,768) and the two best
// levels' totals are cached in SGPRs (their LDS copies are stale while cached). A rest is an LDS add
// (plus a swap of the cached best when it becomes the best); a take compares with an SGPR and only when
// it empties a level scans the LDS totals for the next one. No global memory operation on the chain but
// the log's 1-KB block stores.
//
// 32 bits: SALU has no ordered 64-bit compare (a 64-bit total is compared, and then kept, in VGPRs, with
// copies at every join of the record loop). Exact while the symbol's whole book stays below 2^31: the
// walk starts only if the book's sum is, and adds every block's quantities to that bound before the
// block runs (a block that could cross it goes to the generic loop, from its first record on).
constexpr unsigned long long LW_CAP = 1ull << 31;

struct LWalk {
  uint32_t* tot;     // LDS [L] (empty levels hold 0)
  uint32_t* dummy;   // LDS [64]: the other lanes' targets of a one-lane LDS operation
  uint32_t* occ;     // LDS [L / 32]: occupancy bitmap of the OCC form (bit l: level l's total is nonzero), or null
  int bb, ba;        // best bid (-1: none), best ask (L: none)
  uint32_t cbb, cba; // cached totals of the best levels
  int L;
  unsigned long long ub;  // the book's sum plus the quantities of the blocks walked (< LW_CAP)
};

// smallest occupied level >= x, or L: a scan of the LDS totals. Only levels on the side being searched
// lie there (the other side's cached best, whose LDS copy is stale, is on the other side of x).
// (*tot: its total, read by the scan itself — no second LDS round trip on the chain)
__device__ __forceinline__ uint32_t lw_get(const LWalk& w, int l);
// The OCC form (deep ladders: config 4's hot symbols trade across gaps of hundreds of empty levels): the
// lanes read 64 consecutive 64-bit occupancy words at once, so one LDS read crosses 4,096 levels, and a
// second reads the found level's total.
template <bool OCC = false>
__device__ __forceinline__ int lw_next(const LWalk& w, int x, uint32_t& tot) {
  const int lane = lane_id();
  if constexpr (OCC) {
    const unsigned long long* oc = reinterpret_cast<const unsigned long long*>(w.occ);
    const int nw = w.L >> 6, w0 = x >> 6;
    for (int wb = w0; wb < nw; wb += 64) {
      const int wi = wb + lane;
      unsigned long long m = wi < nw ? oc[wi] : 0ull;
      if (wi == w0) m &= ~0ull << (x & 63);
      const unsigned long long nz = __ballot(m != 0ull);
      if (nz) {
        const int i = __builtin_ctzll(nz);
        const int l = ((wb + i) << 6) + __builtin_ctzll(rl64(m, i));
        tot = lw_get(w, l);
        return l;
      }
    }
    tot = 0u;
    return w.L;
  }
  for (int b = x & ~63; b < w.L; b += 64) {
    const int l = b + lane;
    const uint32_t t = w.tot[l];  // (l < L + 64: beyond L, the dummy slots)
    const unsigned long long m = __ballot(l >= x && l < w.L && t != 0u);
    if (m) {
      const int i = __builtin_ctzll(m);
      tot = rl32(t, i);
      return b + i;
    }
  }
  tot = 0u;
  return w.L;
}
// largest occupied level <= x, or -1
template <bool OCC = false>
__device__ __forceinline__ int lw_prev(const LWalk& w, int x, uint32_t& tot) {
  const int lane = lane_id();
  if constexpr (OCC) {  // lane i reads word w0 - i: the lowest lane with a bit holds the highest level
    const unsigned long long* oc = reinterpret_cast<const unsigned long long*>(w.occ);
    const int w0 = x >> 6;  // (x = -1: -1, no word)
    for (int wb = w0; wb >= 0; wb -= 64) {
      const int wi = wb - lane;
      unsigned long long m = wi >= 0 ? oc[wi] : 0ull;
      if (wi == w0) m &= ~0ull >> (63 - (x & 63));
      const unsigned long long nz = __ballot(m != 0ull);
      if (nz) {
        const int i = __builtin_ctzll(nz);
        const int l = ((wb - i) << 6) + 63 - __builtin_clzll(rl64(m, i));
        tot = lw_get(w, l);
        return l;
      }
    }
    tot = 0u;
    return -1;
  }
  for (int b = x & ~63; b >= 0; b -= 64) {
    const int l = b + lane;
    const uint32_t t = w.tot[l];
    const unsigned long long m = __ballot(l <= x && t != 0u);  // (x < L)
    if (m) {
      const int i = 63 - __builtin_clzll(m);
      tot = rl32(t, i);
      return b + i;
    }
  }
  tot = 0u;
  return -1;
}
// one-lane LDS writes: lane 0 on the level, every other lane on its own dummy slot (no exec change)
__device__ __forceinline__ void lw_add(LWalk& w, int l, uint32_t d) {
  const int lane = lane_id();
  uint32_t* p = lane == 0 ? &w.tot[l] : &w.dummy[lane];
  __hip_atomic_fetch_add(p, d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lw_put(LWalk& w, int l, uint32_t v) {
  const int lane = lane_id();
  uint32_t* p = lane == 0 ? &w.tot[l] : &w.dummy[lane];
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t lw_get(const LWalk& w, int l) {
  return rl32(__hip_atomic_load(&w.tot[l], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP), 0);
}
// The OCC form's bitmap: a level's bit is set by every rest that reaches its LDS total or makes it the best,
// and cleared when a take empties it (non-returning one-lane LDS operations, like lw_add)
template <bool OCC>
__device__ __forceinline__ void lw_occ_set(LWalk& w, int l) {
  if constexpr (OCC) {
    const int lane = lane_id();
    uint32_t* p = lane == 0 ? &w.occ[l >> 5] : &w.dummy[lane];
    __hip_atomic_fetch_or(p, 1u << (l & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}
template <bool OCC>
__device__ __forceinline__ void lw_occ_clr(LWalk& w, int l) {
  if constexpr (OCC) {
    const int lane = lane_id();
    uint32_t* p = lane == 0 ? &w.occ[l >> 5] : &w.dummy[lane];
    __hip_atomic_fetch_and(p, ~(1u << (l & 31)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

// The ladder walk's log staging: event i of the current 64-event block is lane i of three VGPRs, written
// by v_writelane (one instruction per field: no LDS access, no address arithmetic, no lane select), and
// the block leaves as one 16-byte store per lane when it fills.
struct LEv {
  gptr<AggEv> ev;
  uint32_t vl, vj, vq;  // lane i: event i of the block (level, record | AGG_TAKE, quantity)
  uint32_t evp;         // next log index (the slot's log starts 64-aligned)
};
__device__ __forceinline__ void le_store(const LEv& e, uint32_t base, uint32_t n) {
  AggEv x;
  x.lvl = e.vl;
  x.j = e.vj;
  x.qty = (int)e.vq;
  x.pad = 0u;
  if ((uint32_t)lane_id() < n) e.ev[base + (uint32_t)lane_id()] = x;
}
__device__ __forceinline__ void le_emit(LEv& e, uint32_t lvl, uint32_t j, uint32_t q) {
  const uint32_t slot = e.evp & 63u;
  asm volatile(
      "s_mov_b32 m0, %3\n\tv_writelane_b32 %0, %4, m0\n\tv_writelane_b32 %1, %5, m0\n\tv_writelane_b32 %2, %6, m0"
      : "+v"(e.vl), "+v"(e.vj), "+v"(e.vq)
      : "s"(slot), "s"(lvl), "s"(j), "s"(q)
      : "m0");
  e.evp += 1u;
  if (ME_UNLIKELY(slot == 63u)) le_store(e, e.evp - 64u, 64u);
}
__device__ __forceinline__ void le_init(LEv& e, const AggDev& ag, uint32_t eb) {
  e.ev = (gptr<AggEv>)vptr(ag.ev);
  e.vl = e.vj = e.vq = 0u;
  e.evp = eb;
}
__device__ __forceinline__ void le_end(LEv& e) {
  if (e.evp & 63u) le_store(e, e.evp & ~63u, e.evp & 63u);
}
// Grouped launches: 8-B events (AggGEv), two VGPRs — the level and the record number share one word
// (jt already holds record << AGG_GREC_SHIFT | AGG_TAKE), so an event is one SALU or and two v_writelane.
struct LEvG {
  gptr<AggGEv> ev;
  uint32_t vw, vq;
  uint32_t evp;
};
__device__ __forceinline__ void le_store(const LEvG& e, uint32_t base, uint32_t n) {
  AggGEv x;
  x.w = e.vw;
  x.qty = (int)e.vq;
  if ((uint32_t)lane_id() < n) e.ev[base + (uint32_t)lane_id()] = x;
}
__device__ __forceinline__ void le_emit(LEvG& e, uint32_t lvl, uint32_t j, uint32_t q) {
  const uint32_t slot = e.evp & 63u;
  asm volatile("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %3, m0\n\tv_writelane_b32 %1, %4, m0"
               : "+v"(e.vw), "+v"(e.vq)
               : "s"(slot), "s"(lvl | j), "s"(q)
               : "m0");
  e.evp += 1u;
  if (ME_UNLIKELY(slot == 63u)) le_store(e, e.evp - 64u, 64u);
}
// two events, one slot test (the second lands in the same 64-event block unless the first fills it)
__device__ __forceinline__ void le_emit2(LEvG& e, uint32_t lvl, uint32_t j0, uint32_t q0, uint32_t j1, uint32_t q1) {
  const uint32_t slot = e.evp & 63u;
  if (ME_LIKELY(slot < 62u)) {
    asm volatile("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %3, m0\n\tv_writelane_b32 %1, %4, m0\n\t"
                 "s_add_u32 m0, m0, 1\n\tv_writelane_b32 %0, %5, m0\n\tv_writelane_b32 %1, %6, m0"
                 : "+v"(e.vw), "+v"(e.vq)
                 : "s"(slot), "s"(lvl | j0), "s"(q0), "s"(lvl | j1), "s"(q1)
                 : "m0", "scc");
    e.evp += 2u;
  } else {
    le_emit(e, lvl, j0, q0);
    le_emit(e, lvl, j1, q1);
  }
}
__device__ __forceinline__ void le_init(LEvG& e, AggGEv* ev, uint32_t eb) {
  e.ev = (gptr<AggGEv>)vptr(ev);
  e.vw = e.vq = 0u;
  e.evp = eb;
}
__device__ __forceinline__ void le_end(LEvG& e) {
  if (e.evp & 63u) le_store(e, e.evp & ~63u, e.evp & 63u);
}

// A taker's partial take from the best level is the common case and stays out of the loop (no loop
// entry, so none of the loop's register copies); the loop runs only when the best level empties.
template <class LE, bool OCC = false, class W>
__device__ __forceinline__ void lw_take_buy(LE& e, W& w, int lim, uint32_t& rem, uint32_t jt) {
  if (w.ba > lim) return;  // (rem > 0: rejected records never reach the chain)
  if (ME_LIKELY(w.cba > rem)) {
    w.cba -= rem;
    le_emit(e, (uint32_t)w.ba, jt, rem);
    rem = 0;
    return;
  }
  while (true) {  // the best level empties
    le_emit(e, (uint32_t)w.ba, jt, w.cba);
    rem -= w.cba;
    lw_put(w, w.ba, 0u);  // empty levels hold 0 (a rest there adds)
    lw_occ_clr<OCC>(w, w.ba);
    w.ba = lw_next<OCC>(w, w.ba + 1, w.cba);
    if (!rem || w.ba > lim) return;
    if (w.cba > rem) {
      w.cba -= rem;
      le_emit(e, (uint32_t)w.ba, jt, rem);
      rem = 0;
      return;
    }
  }
}
template <class LE, bool OCC = false, class W>
__device__ __forceinline__ void lw_take_sell(LE& e, W& w, int lim, uint32_t& rem, uint32_t jt) {
  if (w.bb < lim) return;
  if (ME_LIKELY(w.cbb > rem)) {
    w.cbb -= rem;
    le_emit(e, (uint32_t)w.bb, jt, rem);
    rem = 0;
    return;
  }
  while (true) {
    le_emit(e, (uint32_t)w.bb, jt, w.cbb);
    rem -= w.cbb;
    lw_put(w, w.bb, 0u);
    lw_occ_clr<OCC>(w, w.bb);
    w.bb = lw_prev<OCC>(w, w.bb - 1, w.cbb);
    if (!rem || w.bb < lim) return;
    if (w.cbb > rem) {
      w.cbb -= rem;
      le_emit(e, (uint32_t)w.bb, jt, rem);
      rem = 0;
      return;
    }
  }
}
// a bid rests at l (< ba: every ask up to the limit was taken)
template <class LE, bool OCC = false, class W>
__device__ __forceinline__ void lw_rest_buy(LE& e, W& w, int l, uint32_t q, uint32_t jt) {
  if (l == w.bb) {
    w.cbb += q;
  } else if (l > w.bb) {  // a new best bid (an empty level)
    if (w.bb >= 0) lw_put(w, w.bb, w.cbb);
    w.bb = l;
    w.cbb = q;
    lw_occ_set<OCC>(w, l);
  } else {
    lw_add(w, l, q);
    lw_occ_set<OCC>(w, l);
  }
  le_emit(e, (uint32_t)l, jt, q);
}
template <class LE, bool OCC = false, class W>
__device__ __forceinline__ void lw_rest_sell(LE& e, W& w, int l, uint32_t q, uint32_t jt) {
  if (l == w.ba) {
    w.cba += q;
  } else if (l < w.ba) {
    if (w.ba < w.L) lw_put(w, w.ba, w.cba);
    w.ba = l;
    w.cba = q;
    lw_occ_set<OCC>(w, l);
  } else {
    lw_add(w, l, q);
    lw_occ_set<OCC>(w, l);
  }
  le_emit(e, (uint32_t)l, jt, q);
}

// The ladder from HBM: 32-bit LDS totals, the cached best totals, the book's sum (false: LW_CAP or more,
// the ladder cannot hold the book)
// (occ: the OCC form's bitmap in LDS, built here from the totals; L a multiple of 64)
__device__ __forceinline__ bool lw_init(LWalk& w, const BookDev& bk, uint32_t s, uint32_t* lds, int bb, int ba,
                                        uint32_t* occ = nullptr) {
  const int lane = lane_id();
  w.L = (int)bk.L;
  w.tot = lds;
  w.dummy = lds + w.L;
  w.occ = occ;
  const Level* lv = bk.levels + (size_t)s * bk.L;
  unsigned long long sum = 0;
  for (int b = 0; b < w.L; b += 16 * 64) {  // sixteen loads in flight per lane
    long long t[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int l = b + u * 64 + lane;
      t[u] = l < w.L ? lv[l].total : 0ll;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int l = b + u * 64 + lane;
      if (l < w.L) w.tot[l] = (uint32_t)t[u];
      sum += (unsigned long long)t[u];
      if (occ) {
        const unsigned long long m = __ballot(l < w.L && t[u] != 0ll);
        if (lane == 0 && b + u * 64 < w.L) reinterpret_cast<unsigned long long*>(occ)[(b + u * 64) >> 6] = m;
      }
    }
  }
  w.ub = (unsigned long long)rli64(wave_incl_scan((long long)sum), 63);  // (DPP: no LDS round trips)
  wave_mem_order();
  w.bb = bb;
  w.ba = ba;
  w.cbb = bb >= 0 ? lw_get(w, bb) : 0u;
  w.cba = ba < w.L ? lw_get(w, ba) : 0u;
  return w.ub < LW_CAP;
}
// The ladder back to HBM (totals, occupancy); the cached totals first. The OCC form writes only the 64-level
// blocks occupied at the start (the book's occupancy words, not yet overwritten) or at the end (its exact
// bitmap): a block empty at both ends holds zeros in HBM already (config 4's seeded books leave ~40 % of a
// 32,768-level window empty).
__device__ __forceinline__ void lw_end(LWalk& w, const BookDev& bk, uint32_t s) {
  const int lane = lane_id();
  if (w.bb >= 0) lw_put(w, w.bb, w.cbb);
  if (w.ba < w.L) lw_put(w, w.ba, w.cba);
  wave_mem_order();
  Level* lv = bk.levels + (size_t)s * bk.L;
  unsigned long long* oc = bk.occ + (size_t)s * bk.Lwords;
  if (w.occ && (w.L >> 6) <= 512 && (int)bk.Lwords == (w.L >> 6)) {
    const int W = w.L >> 6;
    const unsigned long long* eo = reinterpret_cast<const unsigned long long*>(w.occ);
    unsigned long long so[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int b = r * 64 + lane;
      so[r] = b < W ? oc[b] : 0ull;
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      if (r * 64 >= W) break;
      const int b = r * 64 + lane;
      const unsigned long long e = b < W ? eo[b] : 0ull;
      unsigned long long need = __ballot(b < W && (so[r] | e) != 0ull);
      if (b < W && so[r] != e) oc[b] = e;
      while (need) {
        const int bl = r * 64 + __builtin_ctzll(need);
        need &= need - 1ull;
        const int l = bl * 64 + lane;
        lv[l].total = (long long)w.tot[l];
      }
    }
    return;
  }
  for (int b = 0; b < w.L; b += 64) {
    const int l = b + lane;
    const uint32_t t = l < w.L ? w.tot[l] : 0u;
    if (l < w.L) lv[l].total = (long long)t;
    const unsigned long long m = __ballot(t != 0u);
    if (lane == 0 && (b >> 6) < (int)bk.Lwords) oc[b >> 6] = m;
  }
}
// The block's quantities onto the bound; false: the block could take the book to LW_CAP
template <class W>
__device__ __forceinline__ bool lw_admit(W& w, int oq) {
  unsigned long long q = (unsigned long long)(uint32_t)max(oq, 0);
  w.ub += (unsigned long long)rli64(wave_incl_scan((long long)q), 63);
  return w.ub < LW_CAP;
}

// The ladder in registers (windows of L <= 128 levels: the grouped walks): level l's total is lane l & 63
// of VGPR t[l >> 6]. A rest's add is a lane-masked VALU add, a read two v_readlanes and a select, and the
// search for the next occupied level a ballot and a bit scan — no LDS round trip on the chain (the LDS form
// waits on one per emptied level, and config 5's cancels empty a best level 2 times in 3). The best
// levels' totals are cached in SGPRs as in LWalk (their register copies stale while cached); levels >= L
// hold 0.
struct RWalk {
  uint32_t t0, t1;   // VGPRs: levels lane, 64 + lane
  int bb, ba;
  uint32_t cbb, cba;
  int L;
  unsigned long long ub;
};
// (a read takes both VGPRs' lanes and selects the SGPR result: the compiler turned a branch on l's half into
// VALU-materialized conditions; writes branch on the half — same box, k_match per 32 batches: branchless
// writes 460-469 us on config 2, these 450-458, the old read 455-460; config 5 714-734 / 706-712 / 724-731)
__device__ __forceinline__ uint32_t lw_get(const RWalk& w, int l) {
  const uint32_t a = rl32(w.t0, l & 63), b = rl32(w.t1, l & 63);
  return (l & 64) ? b : a;
}
__device__ __forceinline__ void lw_put(RWalk& w, int l, uint32_t v) {
  if (l < 64)
    asm volatile("s_mov_b32 m0, %1\n\tv_writelane_b32 %0, %2, m0" : "+v"(w.t0) : "s"(l), "s"(v) : "m0");
  else
    asm volatile("s_mov_b32 m0, %1\n\tv_writelane_b32 %0, %2, m0" : "+v"(w.t1) : "s"(l - 64), "s"(v) : "m0");
}
__device__ __forceinline__ void lw_add(RWalk& w, int l, uint32_t d) {
  const int lane = lane_id();
  if (l < 64)
    w.t0 += lane == l ? d : 0u;
  else
    w.t1 += lane == l - 64 ? d : 0u;
}
template <bool OCC>
__device__ __forceinline__ void lw_occ_set(RWalk&, int) {}
template <bool OCC>
__device__ __forceinline__ void lw_occ_clr(RWalk&, int) {}
// smallest occupied level >= x (x in [0, 128]), or L
template <bool OCC = false>
__device__ __forceinline__ int lw_next(const RWalk& w, int x, uint32_t& tot) {
  const unsigned long long m0 = __ballot(w.t0 != 0u), m1 = __ballot(w.t1 != 0u);
  if (x < 64) {
    const unsigned long long a = m0 & (~0ull << x);
    if (a) {
      const int l = __builtin_ctzll(a);
      tot = (uint32_t)__builtin_amdgcn_readlane((int)w.t0, l);
      return l;
    }
    x = 64;
  }
  if (x < 128) {
    const unsigned long long a = m1 & (~0ull << (x - 64));
    if (a) {
      const int l = __builtin_ctzll(a);
      tot = (uint32_t)__builtin_amdgcn_readlane((int)w.t1, l);
      return 64 + l;
    }
  }
  tot = 0u;
  return w.L;
}
// largest occupied level <= x (x in [-1, 127]), or -1
template <bool OCC = false>
__device__ __forceinline__ int lw_prev(const RWalk& w, int x, uint32_t& tot) {
  const unsigned long long m0 = __ballot(w.t0 != 0u), m1 = __ballot(w.t1 != 0u);
  if (x >= 64) {
    const unsigned long long a = m1 & (~0ull >> (127 - x));
    if (a) {
      const int l = 63 - __builtin_clzll(a);
      tot = (uint32_t)__builtin_amdgcn_readlane((int)w.t1, l);
      return 64 + l;
    }
    x = 63;
  }
  if (x >= 0) {
    const unsigned long long a = m0 & (~0ull >> (63 - x));
    if (a) {
      const int l = 63 - __builtin_clzll(a);
      tot = (uint32_t)__builtin_amdgcn_readlane((int)w.t0, l);
      return l;
    }
  }
  tot = 0u;
  return -1;
}
// the ladder from HBM (as lw_init: false if the book's sum reaches LW_CAP)
__device__ __forceinline__ bool lw_init(RWalk& w, const BookDev& bk, uint32_t s, int bb, int ba) {
  const int lane = lane_id();
  w.L = (int)bk.L;
  const Level* lv = bk.levels + (size_t)s * bk.L;
  const long long a = lane < w.L ? lv[lane].total : 0ll;
  const long long b = 64 + lane < w.L ? lv[64 + lane].total : 0ll;
  w.t0 = (uint32_t)a;
  w.t1 = (uint32_t)b;
  w.ub = (unsigned long long)rli64(wave_incl_scan(a + b), 63);
  w.bb = bb;
  w.ba = ba;
  w.cbb = bb >= 0 ? lw_get(w, bb) : 0u;
  w.cba = ba < w.L ? lw_get(w, ba) : 0u;
  return w.ub < LW_CAP;
}
// the ladder back to HBM: totals and occupancy words (the cached totals first)
__device__ __forceinline__ void lw_end(RWalk& w, const BookDev& bk, uint32_t s) {
  const int lane = lane_id();
  if (w.bb >= 0) lw_put(w, w.bb, w.cbb);
  if (w.ba < w.L) lw_put(w, w.ba, w.cba);
  Level* lv = bk.levels + (size_t)s * bk.L;
  unsigned long long* oc = bk.occ + (size_t)s * bk.Lwords;
  if (lane < w.L) lv[lane].total = (long long)w.t0;
  if (64 + lane < w.L) lv[64 + lane].total = (long long)w.t1;
  const unsigned long long m0 = __ballot(w.t0 != 0u), m1 = __ballot(w.t1 != 0u);
  if (lane == 0 && bk.Lwords > 0u) oc[0] = m0;
  if (lane == 0 && w.L > 64 && bk.Lwords > 1u) oc[1] = m1;
}

// Control word of a record in vector form: the level a LIMIT rests at / the last level a taker may
// trade at (MARKET: the far end of the window), side, type, reject reason.
__device__ __forceinline__ uint32_t lw_cw(uint32_t okd, int olm, uint32_t rj, int L) {
  const bool buy = (okd & 3u) == ME_SIDE_BUY, mkt = (okd >> 2) & 1u;
  const int lim = mkt ? (buy ? L - 1 : 0) : (olm & (int)LW_LIM);
  return (uint32_t)lim | (buy ? LW_BUY : 0u) | (mkt ? LW_MKT : 0u) | (rj << LW_RJ_SHIFT);
}

// (record r of the block logs its events with jt = (jb + r) << JS: scalar arithmetic, no v_readlane)
template <int JS, class LE, bool OCC = false, class W>
__device__ __forceinline__ uint32_t lw_block(LE& e, W& w, int oq, uint32_t ocw, uint32_t jb,
                                             unsigned long long fastm, uint32_t cnt, int& rr) {
  // the records the walk covers run up to the first it does not (k); rejected ones need no chain work:
  // the loop visits the set bits of `work` (a scalar bit scan, no per-record tests)
  const unsigned long long upto = (cnt >= 64u ? ~0ull : ((1ull << cnt) - 1ull)) & ~fastm;
  const uint32_t k = upto ? (uint32_t)__builtin_ctzll(upto) : cnt;
  const unsigned long long rjm = __ballot((ocw >> LW_RJ_SHIFT) != 0u);
  unsigned long long work = (k >= 64u ? ~0ull : ((1ull << k) - 1ull)) & ~rjm;
  // config 1's walk (JS = 0) reads the next record's control word and quantity one record ahead
  // (v_readlane into SALU waits ~14 cycles; with no record left the lane select is 63, read and unused):
  // 15.13 -> 14.87 ms per batch same box; the grouped walk runs 3 % slower with it (profiles/r4/rl1)
  // (bit 63 set: no zero input, so no undefined count — the compiler keeps the loop's exit test)
  int rn = 0;
  uint32_t cwn = 0, oqn = 0;
  if constexpr (JS == 0) {
    rn = __builtin_ctzll(work | (1ull << 63));
    asm volatile("v_readlane_b32 %0, %2, %4\n\tv_readlane_b32 %1, %3, %4" : "=s"(cwn), "=s"(oqn) : "v"(ocw), "v"(oq), "s"(rn));
  }
  while (work) {
    int r;
    uint32_t cw, rem;
    if constexpr (JS == 0) {
      r = rn;
      asm volatile("s_bitset0_b64 %0, %1" : "+s"(work) : "s"(r));
      cw = cwn;
      rem = oqn;
      rn = __builtin_ctzll(work | (1ull << 63));
      asm volatile("v_readlane_b32 %0, %2, %4\n\tv_readlane_b32 %1, %3, %4" : "=s"(cwn), "=s"(oqn) : "v"(ocw), "v"(oq), "s"(rn));
    } else {
      r = __builtin_ctzll(work);
      asm volatile("s_bitset0_b64 %0, %1" : "+s"(work) : "s"(r));  // (one SALU op; work & (work - 1) is three)
      cw = rl32(ocw, r);
      rem = (uint32_t)rli32(oq, r);
    }
    const uint32_t jt = (jb + (uint32_t)r) << JS;
    const int lim = (int)(cw & LW_LIM);
    // (a MARKET's remainder is dropped: the rest is decided by one integer test — the opaque copy keeps
    // the compiler from re-deriving `!market && rem` as 64-bit boolean masks)
    if (cw & LW_BUY) {
      lw_take_buy<LE, OCC>(e, w, lim, rem, jt | AGG_TAKE);
      uint32_t rq = (cw & LW_MKT) ? 0u : rem;
      asm volatile("" : "+s"(rq));
      if (rq) lw_rest_buy<LE, OCC>(e, w, lim, rq, jt);
    } else {
      lw_take_sell<LE, OCC>(e, w, lim, rem, jt | AGG_TAKE);
      uint32_t rq = (cw & LW_MKT) ? 0u : rem;
      asm volatile("" : "+s"(rq));
      if (rq) lw_rest_sell<LE, OCC>(e, w, lim, rq, jt);
    }
    asm volatile("s_mov_b32 m0, %1\n\tv_writelane_b32 %0, %2, m0" : "+v"(rr) : "s"(r), "s"(auniu(rem)) : "m0");
  }
  return k;
}

// A record's result from its fields and the remainder the chain left (vector form); fill count and
// scratch start come later (k_agg_fin / k_agg_gres, from the log).
__device__ __forceinline__ me_order_result a_result(int oq, uint32_t okd, uint32_t rj, int rem) {
  const bool mkt = (okd >> 2) & 1u;
  const int filled = rj ? 0 : oq - rem;
  me_order_result o;
  o.filled_qty = filled;
  o.remaining_qty = rj ? (rj == ME_RJ_BAD_QTY ? 0 : oq) : rem;
  o.fill_count = 0;
  o.tape_offset = 0;
  o.status = (uint8_t)(rj ? ME_ST_REJECTED
                          : rem == 0 ? ME_ST_FILLED
                          : mkt      ? ME_ST_CANCELED
                          : filled   ? ME_ST_PARTIALLY_FILLED
                                     : ME_ST_NEW);
  o.reason = (uint8_t)rj;
  o.pad[0] = o.pad[1] = 0;
  return o;
}

__device__ void agg_walk_symbol(const BookDev& bk, const BatchDev& bt, const AggDev& ag, uint32_t i, uint32_t s,
                                uint32_t lo, uint32_t hi, unsigned long long* locc, uint32_t* ltot, AggEv* stg) {
  const int lane = lane_id();
  const int L = (int)bk.L;
  const SymState st = bk.sym[s];
  const long long base = rli64(st.base, 0);
  const int bb0 = rli32(st.best_bid, 0), ba0 = rli32(st.best_ask, 0);
  const uint32_t resting = rl32(st.resting, 0), free_head = rl32(st.free_head, 0);
  const uint32_t nfar0 = rl32(st.nfar[0], 0), nfar1 = rl32(st.nfar[1], 0);
  const uint32_t cnt = hi - lo;
  gptr<AggSlot> slot = (gptr<AggSlot>)(ag.slot + i);
  // scratch run of the symbol: fills <= resting makers + 2 * records (k_match's bound)
  const unsigned long long need = (unsigned long long)resting + 2ull * cnt;
  unsigned long long w0 = 0;
  if (lane == 0) w0 = atomicAdd(bt.scratch_top, need);
  w0 = rl64(w0, 0);
  // the log: events <= rests + takes; a take ends its taker or empties a level, and the levels that
  // can empty are the ones occupied at the start (<= min(L, resting)) or created by rests
  const uint32_t evneed = 3u * cnt + min((uint32_t)L, resting) + 64u;
  uint32_t eb = 0;
  if (lane == 0) eb = atomicAdd(&ag.ctr[AC_EV], evneed + 64u);
  eb = (rl32(eb, 0) + 63u) & ~63u;  // 64-aligned: the staged blocks are whole lines of the log
  const bool sok = w0 + need <= bt.scratch_cap;
  const bool eok = (unsigned long long)eb + evneed <= ag.ev_cap;
  if (lane == 0) {
    AggSlot o{};
    o.s = s;
    o.lo = lo;
    o.hi = hi;
    o.pos = sok ? lo : hi;
    o.wbase = w0;
    o.base = base;
    o.ev_base = eb;
    o.free_head = free_head;
    o.resting0 = resting;
    o.bb = bb0;
    o.ba = ba0;
    o.active = 0;
    o.hidx = NIL;
    o.gs = bk.gsym ? bk.gsym[s] : s;
    *slot = o;
  }
  if (!sok) {
    a_set_err(bk, ERR_SCRATCH_OOM);
    return;
  }
  if (!eok || !a_reserve(ag, slot, resting, cnt)) {  // no room in the pools: every record of the symbol
                                                     // goes to the generic loop
    if (lane == 0) {
      const uint32_t idx = atomicAdd(bk.hcount + 1, 1u);
      Handoff ho{};
      ho.s = s;
      ho.pos = lo;
      ho.nsg = hi;
      ho.wptr = (uint32_t)w0;
      ho.wend = (uint32_t)(w0 >> 32);
      bk.hand[bk.S + idx] = ho;
    }
    return;
  }
#ifdef ME_STAMPS
  // the hot walk's cycles by part, accumulated over launches (dbg[s * 24 + 0..4]: set-up, block set-up,
  // record loop, records walked, end), read by tools/hot_probe.py
  unsigned long long gw_t[5] = {0ull, 0ull, 0ull, 0ull, 0ull}, gw_m = stamp_now();
#endif
  AWalk w;
  a_walk_init(w, bk, ag, s, eb, locc, stg);
  // the ladder walk; the top-of-book lists (64-bit totals) for a book the ladder cannot hold, or beyond
  // ag.ladder_max levels
  AList A, B;  // asks (side 1), bids (side 0)
  // (the LDS ladder here: the register form widened to four VGPRs for config 1's 256 levels ran it at
  // 3.9-4.0M against 4.4-4.5M orders/s, same box — its rest-heavy chain prefers the LDS ladder's
  // fire-and-forget adds, and its emptied-level scans are rare; profiles/r6/ab_rw4)
  LWalk lw;
  LEv le;
  le_init(le, ag, eb);
  // the OCC form (next level through an occupancy bitmap in LDS, in locc) for ladders deeper than lw_occ
  const bool occf = ag.lw_occ && L > (int)ag.lw_occ && (L & 63) == 0;
  const bool ladder = L <= (int)ag.ladder_max &&
                      lw_init(lw, bk, s, ltot, bb0, ba0, occf ? reinterpret_cast<uint32_t*>(locc) : nullptr);
  if (!ladder) {
    a_rebuild<1>(w, A, ba0);
    a_rebuild<0>(w, B, L - 1 - bb0);
  }
  GW_T(0);
  uint32_t pos = hi;
  // the blocks' records are gathered ahead of the chain: block b's fields were issued while block b - 1
  // ran, its permutation entries while block b - 2 ran (no HBM round trip between blocks)
  const gptr<const uint32_t> perm = (gptr<const uint32_t>)vptr(bt.perm);
  auto perm_at = [&](uint32_t b) -> uint32_t { return perm[min(b + (uint32_t)lane, hi - 1u)]; };
  uint32_t n_oi = perm_at(lo);
  unsigned long long n_seq = bt.seq[n_oi];
  long long n_px = bt.px[n_oi];
  int n_q = bt.qty[n_oi];
  uint32_t n_kd = bt.kind[n_oi];
  uint32_t nn_oi = perm_at(lo + 64u);
  for (uint32_t blk = lo; blk < hi; blk += 64) {
    const uint32_t j = blk + (uint32_t)lane;
    const bool v = j < hi;
    const uint32_t oi = n_oi;
    const unsigned long long oseq = v ? n_seq : 0ull;
    const long long opx = v ? n_px : 0ll;
    const int oq = v ? n_q : 0;
    const uint32_t okd = v ? n_kd : 0u;
    if (blk + 64u < hi) {  // the next block's fields and the one after's permutation, in flight
      n_oi = nn_oi;
      n_seq = bt.seq[nn_oi];
      n_px = bt.px[nn_oi];
      n_q = bt.qty[nn_oi];
      n_kd = bt.kind[nn_oi];
      nn_oi = perm_at(blk + 128u);
    }
    const uint32_t cntb = min(64u, hi - blk);
    uint32_t rj;
    int olm;
    const unsigned long long fastm = __ballot(a_classify(v, oseq, opx, oq, okd, base, L, nfar0, nfar1, rj, olm));
    int rr = 0;
    uint32_t k;
    if (ladder) {
      const bool adm = lw_admit(lw, v ? oq : 0);  // else: the generic loop from this block on
      GW_T(1);
      k = occf ? lw_block<0, LEv, true>(le, lw, oq, lw_cw(okd, olm, rj, L), blk, adm ? fastm : 0ull, cntb, rr)
               : lw_block<0>(le, lw, oq, lw_cw(okd, olm, rj, L), blk, adm ? fastm : 0ull, cntb, rr);
    } else {
      a_refill(w, A, B);
      GW_T(1);
      k = a_block(w, A, B, oq, lw_cw(okd, olm, rj, L), blk, fastm, cntb, rr);
    }
    GW_T(2);
#ifdef ME_STAMPS
    gw_t[3] += k;
#endif
    if (v && (uint32_t)lane < k) {  // fill count and scratch start: k_agg_out
      bt.res[oi] = a_result(oq, okd, rj, rr);
      bt.fstart[oi] = 0u;
    }
    if (k < cntb) {
      pos = blk + k;  // the generic loop takes over from here (k_match_hot_cont)
      break;
    }
  }
  int bb, ba;
  if (ladder) {
    le_end(le);
    w.evp = le.evp;
    lw_end(lw, bk, s);
    bb = lw.bb;
    ba = lw.ba;
  } else {
    a_walk_end(w, A, B, bb, ba);
  }
  GW_T(4);
#ifdef ME_STAMPS
  if (lane == 0)
    for (int q = 0; q < 5; ++q) bk.dbg[(size_t)s * 24u + q] += gw_t[q];
#endif
  if (lane == 0) {
    slot->pos = pos;
    slot->ev_cnt = w.evp - eb;
    slot->bb = bb;
    slot->ba = ba;
    slot->active = 1;
    if (pos < hi) {
      const uint32_t idx = atomicAdd(bk.hcount + 1, 1u);
      Handoff ho{};
      ho.s = s;
      ho.pos = pos;
      ho.nsg = hi;
      ho.wptr = (uint32_t)w0;  // k_agg_fin moves it past the fills of [lo, pos)
      ho.wend = (uint32_t)(w0 >> 32);
      bk.hand[bk.S + idx] = ho;
      slot->hidx = idx;
    }
  }
}

__global__ __launch_bounds__(64) void k_agg_walk(BookDev bk, BatchDev bt, AggDev ag) {
#if ME_WALK_PRIO
  __builtin_amdgcn_s_setprio(3);  // the serial chain before the short chains of k_match sharing its SIMD
#endif
  __shared__ unsigned long long locc[AGG_WORDS];
  __shared__ AggEv stg[128];  // (the list walk's LDS event staging, ME_LIST_EMIT=0)
  extern __shared__ uint32_t ltot[];  // the ladder walk's totals [L] and dummy slots [64]
  const uint32_t nh = min(*(volatile uint32_t*)bk.hcount, bk.S);
  for (uint32_t i = blockIdx.x; i < nh; i += gridDim.x) {
    const Handoff ho = bk.hand[i];
    agg_walk_symbol(bk, bt, ag, i, auniu(ho.s), auniu(ho.pos), auniu(ho.nsg), locc, ltot, stg);
  }
}

// ------------------------------------------------------------------ grouping the log by level
// One 1024-thread workgroup per hot symbol: level histogram in LDS, segments (one per level with
// events, in level order), then a stable scatter of the log indices (ranks by ballot multisplit over the
// level bits). Windows up to AGG_GW_LMAX levels (config 1's 256): every wave histograms and scatters its
// own contiguous log range (per-wave histograms [16][L] in LDS give each wave its cursors); deeper ones:
// one wave scatters, from log keys staged in LDS chunk by chunk.
constexpr uint32_t AGG_GW_LMAX = 512;
// Deep windows keep one histogram word per level with a pad word after every 32 (level l at l + l / 32): each
// thread owns 32 consecutive levels in the prefix pass, and unpadded, a wave's 64 reads of step k all fell
// in one bank (64-way conflicts, ~60 us of config 4's 188-us launch)
__host__ __device__ constexpr uint32_t agg_gpad(uint32_t l) { return l + (l >> 5); }
__host__ __device__ constexpr size_t agg_group_lds(uint32_t L) {
  return L <= AGG_GW_LMAX ? (size_t)16 * L * 4u : (size_t)agg_gpad(L) * 4u + AGG_GCHUNK * 2u;
}
// The deep path's scatter for logs of up to 16 x 64 x AGG_RX_R events: a stable LSD radix sort of the log by
// level (8-bit digits, two passes), every wave over its own contiguous range held in registers as
// (level << 17 | log index), per-wave digit cursors in LDS (cur [16][256]), the first pass's order through
// the log's evx region (free until k_agg_fin) — instead of one wave ranking the whole log 64 events at a time.
constexpr uint32_t AGG_RX_R = 32;
__device__ __forceinline__ void agg_group_radix(const AggDev& ag, uint32_t eb, uint32_t n, uint32_t nbits,
                                                uint32_t* cur, uint32_t* wtot) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  uint32_t* const tmp = ag.evx + eb;
  const uint32_t per = ((n + 15u) / 16u + 63u) & ~63u;  // <= 64 * AGG_RX_R
  const uint32_t r0 = min(n, (uint32_t)wv * per), r1 = min(n, r0 + per);
  constexpr uint32_t NONE = 0xFFFFFFFFu;  // (no element: level < 2^15, index < 2^17 - 1)
  uint32_t x[AGG_RX_R];
  for (uint32_t pass = 0; pass < 2; ++pass) {
    const uint32_t sh = 17u + (pass ? 8u : 0u), db = pass ? nbits - 8u : 8u;
#pragma unroll
    for (int k = 0; k < (int)AGG_RX_R; ++k) {
      const uint32_t i = r0 + (uint32_t)k * 64u + (uint32_t)lane;
      x[k] = NONE;
      if (i < r1) x[k] = pass ? tmp[i] : ((ag.ev[eb + i].lvl << 17) | i);
    }
    for (uint32_t b = tid; b < 16u * 256u; b += 1024) cur[b] = 0u;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < (int)AGG_RX_R; ++k)
      if (x[k] != NONE) atomicAdd(&cur[wv * 256 + ((x[k] >> sh) & 255u)], 1u);
    __syncthreads();
    // digit-major offsets: digit d of wave w after every smaller digit and after digit d of the earlier waves
    uint32_t c = 0;
    if (tid < 256)
      for (int w = 0; w < 16; ++w) c += cur[w * 256 + tid];
    const uint32_t inc = (uint32_t)wave_incl_scan((long long)c);
    if (lane == 63 && wv < 4) wtot[wv] = inc;
    __syncthreads();
    if (tid < 256) {
      uint32_t base = inc - c;
      for (int w = 0; w < wv; ++w) base += wtot[w];
      for (int w = 0; w < 16; ++w) {
        const uint32_t y = cur[w * 256 + tid];
        cur[w * 256 + tid] = base;
        base += y;
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < (int)AGG_RX_R; ++k) {
      if (r0 + (uint32_t)k * 64u >= r1) break;  // (uniform over the wave)
      const bool v = x[k] != NONE;
      const uint32_t key = v ? (x[k] >> sh) & 255u : 0u;
      unsigned long long peers = __ballot(v);
      for (uint32_t bit = 0; bit < db; ++bit) {
        const unsigned long long bb = __ballot((key >> bit) & 1u);
        peers &= ((key >> bit) & 1u) ? bb : ~bb;
      }
      const uint32_t rank = (uint32_t)__popcll(peers & lanemask_lt());
      const uint32_t cp = (uint32_t)__popcll(peers);
      const uint32_t start = cur[wv * 256 + key];
      if (v) {
        if (pass)
          ag.evs[eb + start + rank] = eb + (x[k] & 0x1FFFFu);
        else
          tmp[start + rank] = x[k];
      }
      __builtin_amdgcn_wave_barrier();
      if (v && rank == 0) cur[wv * 256 + key] = start + cp;
      __builtin_amdgcn_wave_barrier();
    }
    __threadfence();  // the second pass reads the other waves' first-pass writes
    __syncthreads();
  }
}

__global__ __launch_bounds__(1024) void k_agg_group(BookDev bk, AggDev ag) {
  extern __shared__ uint32_t cnt_l[];  // [L], then AGG_GCHUNK 16-bit keys; per-wave: [16][L]
  uint16_t* keys = reinterpret_cast<uint16_t*>(cnt_l + agg_gpad(bk.L));
  __shared__ uint32_t wsum[16], wnz[16], sbase;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t L = bk.L;
  const bool pw = L <= AGG_GW_LMAX;  // (uniform over the launch)
  const uint32_t per = (L + 1023) / 1024;
  uint32_t nbits = 0;
  while ((1u << nbits) < L) ++nbits;
  const uint32_t nh = a_nslots(bk, ag);
  for (uint32_t i = blockIdx.x; i < nh; i += gridDim.x) {
    const AggSlot& sl = ag.slot[i];
    if (!sl.active) continue;  // uniform over the workgroup
    const uint32_t eb = sl.ev_base, n = sl.ev_cnt;
    // per-wave: wave wv's contiguous, 64-aligned log range
    const uint32_t wper = ((n + 15u) / 16u + 63u) & ~63u;
    const uint32_t r0 = min(n, (uint32_t)wv * wper), r1 = min(n, r0 + wper);
    if (pw) {
      for (uint32_t b = tid; b < 16u * L; b += 1024) cnt_l[b] = 0;
      __syncthreads();
      for (uint32_t e = r0 + (uint32_t)lane; e < r1; e += 64) atomicAdd(&cnt_l[(uint32_t)wv * L + ag.ev[eb + e].lvl], 1u);
    } else {
      for (uint32_t b = tid; b < agg_gpad(L); b += 1024) cnt_l[b] = 0;
      __syncthreads();
      for (uint32_t e = tid; e < n; e += 1024) atomicAdd(&cnt_l[agg_gpad(ag.ev[eb + e].lvl)], 1u);
    }
    __syncthreads();
    const uint32_t b0 = tid * per;
    uint32_t lsum = 0, lnz = 0;
    for (uint32_t k = 0; k < per; ++k)
      if (b0 + k < L) {
        uint32_t c = 0;
        if (pw) {
          for (uint32_t w = 0; w < 16; ++w) c += cnt_l[w * L + b0 + k];
        } else {
          c = cnt_l[agg_gpad(b0 + k)];
        }
        lsum += c;
        lnz += c != 0u;
      }
    uint32_t xs = lsum, xn = lnz;  // wave inclusive scans
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t ts = __shfl_up(xs, d, 64), tn = __shfl_up(xn, d, 64);
      if (lane >= d) {
        xs += ts;
        xn += tn;
      }
    }
    if (lane == 63) {
      wsum[wv] = xs;
      wnz[wv] = xn;
    }
    __syncthreads();
    uint32_t ps = 0, pn = 0, tn_all = 0;
    for (int k = 0; k < 16; ++k) {
      if (k < wv) {
        ps += wsum[k];
        pn += wnz[k];
      }
      tn_all += wnz[k];
    }
    if (tid == 0) {
      const uint32_t sb = atomicAdd(&ag.ctr[AC_SEG], tn_all);
      sbase = sb;
      ag.slot[i].seg_base = sb;
      ag.slot[i].nseg = tn_all;
    }
    __syncthreads();
    uint32_t run = ps + xs - lsum, sid = pn + xn - lnz;
    for (uint32_t k = 0; k < per; ++k)
      if (b0 + k < L) {
        const uint32_t l = b0 + k;
        uint32_t c = 0;
        if (pw) {  // each wave's cursor: the level's start plus the earlier waves' events there
          uint32_t r = run;
          for (uint32_t w = 0; w < 16; ++w) {
            const uint32_t x = cnt_l[w * L + l];
            cnt_l[w * L + l] = r;
            r += x;
          }
          c = r - run;
        } else {
          c = cnt_l[agg_gpad(l)];
          cnt_l[agg_gpad(l)] = run;
        }
        if (c) {
          AggSeg g;
          g.slot = i;
          g.lvl = l;
          g.start = eb + run;
          g.cnt = c;
          ag.seg[sbase + sid] = g;
          ++sid;
        }
        run += c;
      }
    __syncthreads();
    if (pw) {  // every wave scatters its range (ranks by ballot multisplit, cursors in its own histogram)
      uint32_t* cur = cnt_l + (uint32_t)wv * L;
      for (uint32_t c0 = r0; c0 < r1; c0 += 64) {
        const uint32_t e = c0 + (uint32_t)lane;
        const bool v = e < r1;
        const uint32_t key = v ? ag.ev[eb + e].lvl : 0u;
        unsigned long long peers = __ballot(v);
        for (uint32_t bit = 0; bit < nbits; ++bit) {
          const unsigned long long bb = __ballot((key >> bit) & 1u);
          peers &= ((key >> bit) & 1u) ? bb : ~bb;
        }
        const uint32_t rank = (uint32_t)__popcll(peers & lanemask_lt());
        const uint32_t cp = (uint32_t)__popcll(peers);
        const uint32_t start = cur[key];
        if (v) ag.evs[eb + start + rank] = eb + e;
        __builtin_amdgcn_wave_barrier();
        if (v && rank == 0) cur[key] = start + cp;
        __builtin_amdgcn_wave_barrier();
      }
      __syncthreads();
    } else if (n <= 16u * 64u * AGG_RX_R && L <= 32768u) {
      agg_group_radix(ag, eb, n, nbits, reinterpret_cast<uint32_t*>(keys), wsum);
    } else {
      // the scatter: chunks of AGG_GCHUNK keys staged in LDS by the whole workgroup (coalesced), then
      // ranked and placed by one wave (its steps read LDS only: no HBM round trip per 64 events)
      for (uint32_t c1 = 0; c1 < n; c1 += AGG_GCHUNK) {
        const uint32_t m = min(AGG_GCHUNK, n - c1);
        for (uint32_t e = tid; e < m; e += 1024) keys[e] = (uint16_t)ag.ev[eb + c1 + e].lvl;
        __syncthreads();
        if (wv == 0) {
          for (uint32_t c0 = 0; c0 < m; c0 += 64) {
            const uint32_t e = c0 + (uint32_t)lane;
            const bool v = e < m;
            const uint32_t key = v ? (uint32_t)keys[e] : 0u;
            unsigned long long peers = __ballot(v);
            for (uint32_t bit = 0; bit < nbits; ++bit) {
              const unsigned long long bb = __ballot((key >> bit) & 1u);
              peers &= ((key >> bit) & 1u) ? bb : ~bb;
            }
            const uint32_t rank = (uint32_t)__popcll(peers & lanemask_lt());
            const uint32_t cp = (uint32_t)__popcll(peers);
            const uint32_t start = cnt_l[agg_gpad(key)];
            if (v) ag.evs[eb + start + rank] = eb + c1 + e;
            __builtin_amdgcn_wave_barrier();
            if (v && rank == 0) cnt_l[agg_gpad(key)] = start + cp;
            __builtin_amdgcn_wave_barrier();
          }
        }
        __syncthreads();
      }
    }
  }
}

// The sorted copies the per-level kernels read (one hop instead of index -> entry), every slot's log over
// the whole grid.
__global__ __launch_bounds__(256) void k_agg_sorted(BookDev bk, AggDev ag) {
  const uint32_t nh = a_nslots(bk, ag);
  const uint32_t T = gridDim.x * blockDim.x;
  for (uint32_t i = 0; i < nh; ++i) {
    const AggSlot& sl = ag.slot[i];
    if (!sl.active) continue;
    const uint32_t eb = sl.ev_base, n = sl.ev_cnt;
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += T) {
      const uint32_t e = ag.evs[eb + p];
      AggEv E = ag.ev[e];
      E.pad = e;
      ag.evq[eb + p] = E;
    }
  }
}

// ------------------------------------------------------------------ per-level FIFO resolution
__device__ __forceinline__ unsigned long long a_seq_of(const BatchDev& bt, uint32_t j) { return bt.seq[bt.perm[j]]; }
__device__ __forceinline__ unsigned long long a_seq_of(const AggSrc& src, uint32_t j) {
  return src.perm ? src.seq[0][src.perm[j]] : src.seq[j >> AGG_GSHIFT][j & AGG_IMASK];
}

// First index in mk[b, b + n) whose end is > x (strict = false: >= x).
__device__ __forceinline__ uint32_t a_search(const AggMk* mk, uint32_t b, uint32_t n, unsigned long long x, bool strict) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    const unsigned long long e = mk[b + mid].end;
    if (strict ? e <= x : e < x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// First index in the LDS maker list m[0, n) whose end is > x (strict = false: >= x).
__device__ __forceinline__ uint32_t a_search_lds(const AggMk* m, uint32_t n, unsigned long long x, bool strict) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    const unsigned long long e = m[mid].end;
    if (strict ? e <= x : e < x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

constexpr uint32_t LV_STAGE = 64;  // consumed makers / emptied chunks a level keeps in LDS (else: HBM)

// One wave per segment (symbol, level): the quantity C the batch took from the level; the initial FIFO
// read once until C is covered — consumed makers (seq, interval end) and emptied chunks staged in LDS —
// and the rests C reaches; then the makers and emptied chunks to HBM, the emptied chunks zeroed, the
// chunk C ends in updated; each take's first maker and fill count (binary search in the staged list);
// what the surviving rests need. A level whose takes consume more than LV_STAGE makers (or empty more
// chunks) reads its FIFO a second time, writing straight into HBM.
template <bool COUNT>
__global__ __launch_bounds__(256) void k_agg_levels(BookDev bk, AggSrc src, AggDev ag) {
  __shared__ AggMk smk[4][LV_STAGE];
  __shared__ uint32_t sfr[4][LV_STAGE];
  const int lane = lane_id();
  const bool act = lane < ME_C;
  const uint32_t wv = threadIdx.x >> 6;
  AggMk* mkl = smk[wv];
  uint32_t* frl = sfr[wv];
  const uint32_t gw = blockIdx.x * 4u + wv, nw = gridDim.x * 4u;
  const uint32_t nseg = min(*(volatile uint32_t*)&ag.ctr[AC_SEG], ag.ev_cap);
  for (uint32_t si = gw; si < nseg; si += nw) {
    const AggSeg sg = ag.seg[si];
    const uint32_t slot_i = auniu(sg.slot), lvl = auniu(sg.lvl), start = auniu(sg.start), cnt = auniu(sg.cnt);
    AggSlot* sl = ag.slot + slot_i;
    const uint32_t s = auniu(sl->s);
    const size_t li = (size_t)s * bk.L + lvl;
    const uint32_t head0 = auniu(bk.levels[li].head);
    const uint32_t te_raw = (uint32_t)bk.tend[li];
    // the first 64 entries stay in registers (most levels have no more)
    AggEv E0{};
    if ((uint32_t)lane < cnt) E0 = ag.evq[start + lane];
    auto entry = [&](uint32_t b) -> AggEv {
      if (b == 0) return E0;
      AggEv E{};
      if (b + (uint32_t)lane < cnt) E = ag.evq[start + b + lane];
      return E;
    };
    // 1. C: the takes' total
    unsigned long long C = 0;
    for (uint32_t b = 0; b < cnt; b += 64) {
      const AggEv E = entry(b);
      const bool v = b + (uint32_t)lane < cnt;
      const bool tk = v && (E.j & AGG_TAKE) != 0u;
      if (!COUNT && v && !tk) ag.evn[E.pad] = 0u;
      C += (unsigned long long)rli64(wave_incl_scan(tk ? (long long)E.qty : 0ll), 63);
    }
    // 2. the initial FIFO, read once: consumed makers and emptied chunks staged in LDS; the chunk C ends
    //    in keeps its quantities and interval ends in registers (pq, pen)
    unsigned long long W = 0;
    uint32_t nmk = 0, nfreed = 0, nfull = 0, newhead = NIL, ch = head0, pch = NIL;
    int pq = 0;
    unsigned long long pen = 0;
    bool exhausted = false;
    for (;;) {
      if (ch == NIL) {
        exhausted = true;
        break;
      }
      if (W >= C) {
        newhead = ch;
        break;
      }
      if (ch >= bk.nchunks) {
        a_set_err(bk, ERR_INCONSISTENT);
        exhausted = true;
        break;
      }
      const int q = act ? bk.chunks[ch].qty[lane] : 0;
      const unsigned long long sq = act ? bk.chunks[ch].seq[lane] : 0ull;
      const uint32_t nx = auniu(bk.chunks[ch].hdr.next);
      const long long inc = wave_incl_scan((long long)q);
      const unsigned long long ex = (unsigned long long)(inc - q), en = W + (unsigned long long)inc;
      const unsigned long long live = (unsigned long long)rli64(inc, 63);
      const bool cons = q > 0 && W + ex < C;
      const unsigned long long cm = __ballot(cons);
      const uint32_t r = nmk + (uint32_t)__popcll(cm & lanemask_lt());
      if (!COUNT && cons && r < LV_STAGE) {
        mkl[r].seq = sq;
        mkl[r].end = en;
      }
      nmk += (uint32_t)__popcll(cm);
      nfull += (uint32_t)__popcll(__ballot(q > 0 && en <= C));
      if (W + live <= C) {  // emptied
        if (!COUNT && lane == 0 && nfreed < LV_STAGE) frl[nfreed] = ch;
        ++nfreed;
        W += live;
        ch = nx;
        continue;
      }
      pch = ch;  // C ends inside this chunk
      pq = q;
      pen = en;
      newhead = ch;
      break;
    }
    const unsigned long long T0 = exhausted ? W : ~0ull;
    const unsigned long long Cr = exhausted && C > W ? C - W : 0ull;  // taken from this batch's rests
    // 3. the rests: those C reaches are makers too (staged after the FIFO's), the others survive
    uint32_t nrc = 0, ks = 0;
    {
      unsigned long long RR = 0;
      for (uint32_t b = 0; b < cnt; b += 64) {
        const AggEv E = entry(b);
        const bool v = b + (uint32_t)lane < cnt;
        const bool rs = v && (E.j & AGG_TAKE) == 0u;
        const long long rq = rs ? (long long)E.qty : 0ll;
        const long long inc = wave_incl_scan(rq);
        const unsigned long long st0 = RR + (unsigned long long)(inc - rq), en = RR + (unsigned long long)inc;
        const bool cons = rs && st0 < Cr;
        const unsigned long long cm = __ballot(cons);
        const uint32_t r = nmk + nrc + (uint32_t)__popcll(cm & lanemask_lt());
        if (!COUNT && cons && r < LV_STAGE) {
          mkl[r].seq = a_seq_of(src, E.j);
          mkl[r].end = T0 + en;
        }
        nrc += (uint32_t)__popcll(cm);
        ks += (uint32_t)__popcll(__ballot(rs && en > Cr));
        RR += (unsigned long long)rli64(inc, 63);
      }
    }
    const uint32_t te0 = newhead != NIL ? auniu(te_raw) : 0u;  // the tail survives iff newhead does
    const uint32_t tailfree = newhead != NIL ? (uint32_t)ME_C - te0 : 0u;
    const uint32_t need = ks > tailfree ? (ks - tailfree + ME_C - 1) / ME_C : 0u;
    const uint32_t own = min(need, nfreed), deficit = need - own;
    const uint32_t nmkt = nmk + nrc;
    if constexpr (COUNT) {  // the counts for k_agg_lvscan (nothing else is written by this pass)
      if (lane == 0) {
        AggSegS o{};
        o.nmk = nmkt;
        o.nfreed = nfreed;
        o.d_off = deficit;
        o.ks = (uint32_t)((int)ks - (int)nfull);
        ag.segs[si] = o;
      }
      continue;
    }
    // the level's regions of the slot's makers / freed chunks and its share of the deficit: k_agg_lvscan's
    // exclusive scans of the counting pass, which ran this same code (a mismatch is an internal error)
    const uint32_t mk_base = auniu(ag.segs[si].mk_base), fr_base = auniu(ag.segs[si].fr_base);
    const uint32_t d_off = auniu(ag.segs[si].d_off);
    if (auniu(ag.segs[si].nmk) != nmkt || auniu(ag.segs[si].nfreed) != nfreed) a_set_err(bk, ERR_INCONSISTENT);
    if (mk_base + nmkt > ag.mk_cap || fr_base + nfreed > ag.fr_cap) {
      a_set_err(bk, ERR_SCRATCH_OOM);  // sized so this cannot happen; leaves the level alone
      for (uint32_t b = lane; b < cnt; b += 64) ag.evn[ag.evq[start + b].pad] = 0u;
      if (lane == 0) {
        AggSegS o{};
        o.T0 = ~0ull;
        o.newhead = head0;
        ag.segs[si] = o;
      }
      continue;
    }
    const bool staged = nmkt <= LV_STAGE && nfreed <= LV_STAGE;
    // 4. makers and emptied chunks to HBM: from LDS, or past LV_STAGE by a second read of the FIFO
    wave_mem_order();
    if (staged) {
      if ((uint32_t)lane < nmkt) ag.mk[mk_base + lane] = mkl[lane];
      if ((uint32_t)lane < nfreed) ag.fr[fr_base + lane] = frl[lane];
    } else {
      unsigned long long Wv = 0;
      uint32_t mi = 0, fi = 0;
      ch = head0;
      while (Wv < C && ch < bk.nchunks) {
        const int q = act ? bk.chunks[ch].qty[lane] : 0;
        const unsigned long long sq = act ? bk.chunks[ch].seq[lane] : 0ull;
        const uint32_t nx = auniu(bk.chunks[ch].hdr.next);
        const long long inc = wave_incl_scan((long long)q);
        const unsigned long long ex = (unsigned long long)(inc - q), en = Wv + (unsigned long long)inc;
        const unsigned long long live = (unsigned long long)rli64(inc, 63);
        const bool cons = q > 0 && Wv + ex < C;
        const unsigned long long cm = __ballot(cons);
        if (cons) {
          AggMk m;
          m.seq = sq;
          m.end = en;
          ag.mk[mk_base + mi + (uint32_t)__popcll(cm & lanemask_lt())] = m;
        }
        mi += (uint32_t)__popcll(cm);
        if (Wv + live > C) break;
        if (lane == 0) ag.fr[fr_base + fi] = ch;
        ++fi;
        Wv += live;
        ch = nx;
      }
      if (Cr) {
        unsigned long long RR = 0;
        for (uint32_t b = 0; b < cnt; b += 64) {
          const AggEv E = entry(b);
          const bool v = b + (uint32_t)lane < cnt;
          const bool rs = v && (E.j & AGG_TAKE) == 0u;
          const long long rq = rs ? (long long)E.qty : 0ll;
          const long long inc = wave_incl_scan(rq);
          const unsigned long long st0 = RR + (unsigned long long)(inc - rq), en = RR + (unsigned long long)inc;
          const bool cons = rs && st0 < Cr;
          const unsigned long long cm = __ballot(cons);
          if (cons) {
            AggMk m;
            m.seq = a_seq_of(src, E.j);
            m.end = T0 + en;
            ag.mk[mk_base + mi + (uint32_t)__popcll(cm & lanemask_lt())] = m;
          }
          mi += (uint32_t)__popcll(cm);
          RR += (unsigned long long)rli64(inc, 63);
        }
      }
    }
    // 5. the FIFO's new state: emptied chunks hold qty 0 (free chunks do), the chunk C ends in keeps
    //    what is left of its makers
    wave_mem_order();
    for (uint32_t f0 = 0; f0 < nfreed; f0 += 4) {
      const uint32_t f = f0 + (uint32_t)lane / ME_C;
      if (f < nfreed) {
        const uint32_t c = staged ? frl[f] : ag.fr[fr_base + f];
        if (c < bk.nchunks) bk.chunks[c].qty[lane % ME_C] = 0;
      }
    }
    if (pch != NIL && act && pq > 0 && pen - (unsigned long long)pq < C)
      bk.chunks[pch].qty[lane] = pen <= C ? 0 : (int)(pen - C);
    // 6. each take: its first maker and its fill count (makers overlapping its interval)
    wave_mem_order();
    {
      unsigned long long A0 = 0;
      for (uint32_t b = 0; b < cnt; b += 64) {
        const AggEv E = entry(b);
        const bool v = b + (uint32_t)lane < cnt;
        const bool tk = v && (E.j & AGG_TAKE) != 0u;
        const long long tq = tk ? (long long)E.qty : 0ll;
        const long long inc = wave_incl_scan(tq);
        if (tk) {
          const unsigned long long a = A0 + (unsigned long long)(inc - tq), z = a + (unsigned long long)E.qty;
          const uint32_t first = staged ? a_search_lds(mkl, nmkt, a, true) : a_search(ag.mk, mk_base, nmkt, a, true);
          const uint32_t last = staged ? a_search_lds(mkl, nmkt, z, false) : a_search(ag.mk, mk_base, nmkt, z, false);
          ag.eva[E.pad] = a;
          ag.evf[E.pad] = mk_base + first;
          ag.evn[E.pad] = last - first + 1u;
        }
        A0 += (unsigned long long)rli64(inc, 63);
      }
    }
    if (lane == 0) {
      AggSegS o;
      o.C = C;
      o.T0 = T0;
      o.newhead = newhead;
      o.mk_base = mk_base;
      o.nmk = nmkt;
      o.fr_base = fr_base;
      o.nfreed = nfreed;
      o.need = need;
      o.d_off = d_off;
      o.ks = ks;
      ag.segs[si] = o;
    }
    wave_mem_order();  // the next segment reuses the staging
  }
}

// The segments' allocations, by scan instead of returning atomics: one workgroup per hot symbol turns the
// counting pass's per-level counts (makers consumed, chunks emptied, chunk deficit, resting change) into
// each level's offsets in the slot's regions of AggDev::mk / ::fr and of its deficit, and sets the slot's
// cursors and totals. (A returning atomic per segment on the slot's cursors serialised config 4's ~7,000
// segments of the hot symbol on one L2 line: k_agg_levels 640-740 us per batch, profiles/r5/occ.)
__global__ __launch_bounds__(1024) void k_agg_lvscan(BookDev bk, AggDev ag) {
  __shared__ long long wsum[3][16];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t nh = a_nslots(bk, ag);
  for (uint32_t i = blockIdx.x; i < nh; i += gridDim.x) {
    AggSlot* sl = ag.slot + i;
    if (!auniu(sl->active)) continue;
    const uint32_t sb = auniu(sl->seg_base), ns = auniu(sl->nseg);
    const uint32_t mb = auniu(sl->mk_base), fb = auniu(sl->fr_base);
    long long c0 = 0, c1 = 0, c2 = 0, cd = 0;  // running totals (every thread keeps them)
    for (uint32_t b = 0; b < ns; b += 1024u) {
      const uint32_t si = sb + b + (uint32_t)tid;
      const bool v = b + (uint32_t)tid < ns;
      long long x0 = 0, x1 = 0, x2 = 0, xd = 0;
      if (v) {
        const AggSegS g = ag.segs[si];
        x0 = g.nmk;
        x1 = g.nfreed;
        x2 = g.d_off;
        xd = (int)g.ks;
      }
      const long long i0 = wave_incl_scan(x0), i1 = wave_incl_scan(x1), i2 = wave_incl_scan(x2);
      const long long id = wave_incl_scan(xd);
      if (lane == 63) {
        wsum[0][wv] = i0;
        wsum[1][wv] = i1;
        wsum[2][wv] = i2;
      }
      __syncthreads();
      long long p0 = 0, p1 = 0, p2 = 0, t0 = 0, t1 = 0, t2 = 0;
      for (int k = 0; k < 16; ++k) {
        if (k < wv) {
          p0 += wsum[0][k];
          p1 += wsum[1][k];
          p2 += wsum[2][k];
        }
        t0 += wsum[0][k];
        t1 += wsum[1][k];
        t2 += wsum[2][k];
      }
      __syncthreads();  // (wsum is rewritten by the next chunk)
      if (v) {
        ag.segs[si].mk_base = mb + (uint32_t)(c0 + p0 + i0 - x0);
        ag.segs[si].fr_base = fb + (uint32_t)(c1 + p1 + i1 - x1);
        ag.segs[si].d_off = (uint32_t)(c2 + p2 + i2 - x2);
      }
      c0 += t0;
      c1 += t1;
      c2 += t2;
      if (lane == 63) cd += id;  // (per wave; summed below by atomics on the slot)
    }
    if (lane == 63 && cd) atomicAdd(&sl->dresting, (int)cd);
    if (tid == 0) {
      sl->mk_cur = (uint32_t)c0;
      sl->fr_cur = (uint32_t)c1;
      sl->deficit = (uint32_t)c2;
    }
    __syncthreads();
  }
}

// One wave per hot symbol: the chunks the surviving rests need beyond their levels' own emptied ones
// (the slot's deficit) come from other levels' surpluses, then the symbol's free list, then the bump
// allocator; surpluses left over join the free list. fr[alloc_base + t], t < deficit: the allocation;
// fr[alloc_base + deficit + u], u < surplus: the surpluses gathered.
__global__ __launch_bounds__(64) void k_agg_alloc(BookDev bk, AggDev ag) {
  const int lane = lane_id();
  const uint32_t nh = a_nslots(bk, ag);
  for (uint32_t i = blockIdx.x; i < nh; i += gridDim.x) {
    AggSlot* sl = ag.slot + i;
    if (!auniu(sl->active)) continue;
    const uint32_t s = auniu(sl->s), sb = auniu(sl->seg_base), ns = auniu(sl->nseg);
    const uint32_t D = auniu(sl->deficit);
    uint32_t fh = auniu(sl->free_head);
    uint32_t Stot = 0;
    for (uint32_t b = 0; b < ns; b += 64) {
      uint32_t sp = 0;
      if (b + lane < ns) {
        const AggSegS& g = ag.segs[sb + b + lane];
        sp = g.nfreed - min(g.need, g.nfreed);
      }
      Stot += (uint32_t)rli64(wave_incl_scan((long long)sp), 63);
    }
    if (!D && !Stot) continue;
    uint32_t ab = 0;
    if (lane == 0) ab = sl->fr_base + atomicAdd(&sl->fr_cur, D + Stot);
    ab = rl32(ab, 0);
    if ((unsigned long long)ab + D + Stot > ag.fr_cap) {
      a_set_err(bk, ERR_SCRATCH_OOM);
      continue;
    }
    // gather the surpluses (level order) into fr[ab + D, ab + D + Stot)
    uint32_t run = 0;
    for (uint32_t b = 0; b < ns; b += 64) {
      uint32_t sp = 0, src = 0;
      if (b + lane < ns) {
        const AggSegS& g = ag.segs[sb + b + lane];
        const uint32_t own = min(g.need, g.nfreed);
        sp = g.nfreed - own;
        src = g.fr_base + own;
      }
      const long long inc = wave_incl_scan((long long)sp);
      const uint32_t ex = run + (uint32_t)(inc - sp);
      for (uint32_t k = 0; k < sp; ++k) ag.fr[ab + D + ex + k] = ag.fr[src + k];
      run += (uint32_t)rli64(inc, 63);
    }
    a_drain();
    const uint32_t k1 = min(D, Stot);
    for (uint32_t t = lane; t < k1; t += 64) ag.fr[ab + t] = ag.fr[ab + D + t];
    if (D > k1) {  // the book grows: the free list, then fresh chunks
      uint32_t t = k1;
      if (lane == 0) {
        while (t < D && fh != NIL && fh < bk.nchunks) {
          ag.fr[ab + t] = fh;
          fh = bk.chunks[fh].hdr.next;
          ++t;
        }
      }
      t = rl32(t, 0);
      fh = rl32(fh, 0);
      if (t < D) {
        const uint32_t left = D - t;
        uint32_t got = 0;
        if (lane == 0) got = atomicAdd(bk.chunk_top, left);
        got = rl32(got, 0);
        const CPool cp = cp_read(bk.cpool);
        if ((unsigned long long)got + left > cp_vcap(cp, bk.nchunks)) {
          a_set_err(bk, ERR_CHUNK_OOM);
          for (uint32_t u = lane; u < left; u += 64) ag.fr[ab + t + u] = 0u;  // never indexed past the pool
        } else {
          for (uint32_t u = lane; u < left; u += 64) {
            const uint32_t id = cp_id(bk.recl, cp, got + u);
            ag.fr[ab + t + u] = id;
            bk.chunks[id].owner = s;  // the symbol's until a reclamation finds the chunk free
          }
        }
      }
    } else if (Stot > D) {  // surpluses left over: linked in front of the free list
      for (uint32_t u = D + lane; u < Stot; u += 64) {
        const uint32_t c = ag.fr[ab + D + u];
        bk.chunks[c].hdr.next = u + 1 < Stot ? ag.fr[ab + D + u + 1] : fh;
      }
      fh = auniu(ag.fr[ab + D + D]);
    }
    if (lane == 0) {
      sl->alloc_base = ab;
      sl->free_head = fh;
    }
  }
}

// One wave per segment: the surviving rests into the level's tail chunk and new chunks (in order),
// the new chunks' headers and links, the seq ring, the level's head / tail / tail fill.
__global__ __launch_bounds__(256) void k_agg_place(BookDev bk, AggSrc src, AggDev ag) {
  const int lane = lane_id();
  const uint32_t gw = blockIdx.x * 4u + (threadIdx.x >> 6), nw = gridDim.x * 4u;
  const uint32_t nseg = min(*(volatile uint32_t*)&ag.ctr[AC_SEG], ag.ev_cap);
  for (uint32_t si = gw; si < nseg; si += nw) {
    const AggSeg sg = ag.seg[si];
    const uint32_t slot_i = auniu(sg.slot), lvl = auniu(sg.lvl), start = auniu(sg.start), cnt = auniu(sg.cnt);
    const AggSlot* sl = ag.slot + slot_i;
    const uint32_t s = auniu(sl->s), alloc_base = auniu(sl->alloc_base);
    const long long base = (long long)rl64((unsigned long long)sl->base, 0);
    const AggSegS g = ag.segs[si];
    const unsigned long long C = rl64(g.C, 0), T0 = rl64(g.T0, 0);
    const uint32_t newhead = auniu(g.newhead), need = auniu(g.need), ks = auniu(g.ks);
    const uint32_t nfreed = auniu(g.nfreed), fr_base = auniu(g.fr_base), d_off = auniu(g.d_off);
    const uint32_t own = min(need, nfreed);
    const size_t li = (size_t)s * bk.L + lvl;
    const uint32_t head0 = auniu(bk.levels[li].head), tail0 = auniu(bk.levels[li].tail);
    const uint32_t te0 = newhead != NIL ? auniu((uint32_t)bk.tend[li]) : 0u;
    const uint32_t tailfree = newhead != NIL ? (uint32_t)ME_C - te0 : 0u;
    auto newchunk = [&](uint32_t c) -> uint32_t {
      return c < own ? ag.fr[fr_base + c] : ag.fr[alloc_base + d_off + (c - own)];
    };
    const bool exhausted = T0 != ~0ull;
    const unsigned long long Cr = exhausted && C > T0 ? C - T0 : 0ull;
    if (ks) {
      unsigned long long RR = 0;
      uint32_t g0 = 0;
      for (uint32_t b = 0; b < cnt; b += 64) {
        const bool v = b + (uint32_t)lane < cnt;
        AggEv E{};
        if (v) E = ag.evq[start + b + lane];
        const bool rs = v && (E.j & AGG_TAKE) == 0u;
        const long long rq = rs ? (long long)E.qty : 0ll;
        const long long inc = wave_incl_scan(rq);
        const unsigned long long st0 = RR + (unsigned long long)(inc - rq), en = RR + (unsigned long long)inc;
        const bool surv = rs && en > Cr;
        const unsigned long long sm = __ballot(surv);
        if (surv) {
          const uint32_t gi = g0 + (uint32_t)__popcll(sm & lanemask_lt());
          uint32_t chk, slt;
          if (gi < tailfree) {
            chk = tail0;
            slt = te0 + gi;
          } else {
            const uint32_t gg = gi - tailfree;
            chk = newchunk(gg / ME_C);
            slt = gg % ME_C;
          }
          const unsigned long long sq = a_seq_of(src, E.j);
          const int left = (int)(en - (st0 > Cr ? st0 : Cr));
          if (chk < bk.nchunks) {
            bk.chunks[chk].qty[slt] = left;
            bk.chunks[chk].seq[slt] = sq;
            bk.loc[sq & bk.ring_mask] = chk * ME_C + slt;
          }
        }
        g0 += (uint32_t)__popcll(sm);
        RR += (unsigned long long)rli64(inc, 63);
      }
    }
    for (uint32_t c = lane; c < need; c += 64) {
      const uint32_t chk = newchunk(c);
      if (chk >= bk.nchunks) continue;
      ChunkHdr h;
      h.next = c + 1 < need ? newchunk(c + 1) : NIL;
      h.prev = c ? newchunk(c - 1) : (newhead != NIL ? tail0 : NIL);
      h.price = base + (long long)lvl;
      bk.chunks[chk].hdr = h;
    }
    const uint32_t first_new = need ? auniu(newchunk(0)) : NIL;
    const uint32_t last_new = need ? auniu(newchunk(need - 1)) : NIL;
    if (lane == 0) {
      if (newhead != NIL && need && tail0 < bk.nchunks) bk.chunks[tail0].hdr.next = first_new;
      if (newhead != NIL && newhead != head0 && newhead < bk.nchunks) bk.chunks[newhead].hdr.prev = NIL;
      const uint32_t hd = newhead != NIL ? newhead : first_new;
      const uint32_t tl = need ? last_new : (newhead != NIL ? tail0 : NIL);
      const uint32_t te = need ? ((ks - tailfree - 1u) % ME_C) + 1u : (newhead != NIL ? te0 + ks : 0u);
      bk.levels[li].head = hd;
      bk.levels[li].tail = tl;
      bk.tend[li] = (uint8_t)te;
    }
  }
}

// One workgroup per hot symbol: the fill offsets (exclusive scan of the events' fill counts in log
// order = tape order), the records' results, the symbol's state, the continuation's scratch position.
__global__ __launch_bounds__(1024) void k_agg_fin(BookDev bk, BatchDev bt, AggDev ag) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t carry_s;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t nh = min(*(volatile uint32_t*)bk.hcount, bk.S);
  constexpr uint32_t PER = 8;
  for (uint32_t i = blockIdx.x; i < nh; i += gridDim.x) {
    const AggSlot sl = ag.slot[i];
    if (!sl.active) continue;
    const uint32_t eb = sl.ev_base, n = sl.ev_cnt;
    uint32_t carry = 0;
    for (uint32_t t0 = 0; t0 < n; t0 += 1024 * PER) {
      const uint32_t b = t0 + (uint32_t)tid * PER;
      uint32_t v[PER], loc = 0;
#pragma unroll
      for (uint32_t k = 0; k < PER; ++k) {
        v[k] = b + k < n ? ag.evn[eb + b + k] : 0u;
        loc += v[k];
      }
      uint32_t x = loc;
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(x, d, 64);
        if (lane >= d) x += t;
      }
      if (lane == 63) wsum[wv] = x;
      __syncthreads();
      uint32_t pre = 0, tot = 0;
      for (int k = 0; k < 16; ++k) {
        if (k < wv) pre += wsum[k];
        tot += wsum[k];
      }
      uint32_t r = carry + pre + x - loc;
#pragma unroll
      for (uint32_t k = 0; k < PER; ++k)
        if (b + k < n) {
          ag.evx[eb + b + k] = r;
          r += v[k];
        }
      carry += tot;
      __syncthreads();
    }
    if (tid == 0) carry_s = carry;
    __syncthreads();
    const uint32_t ftot = carry_s;
    if (tid == 0) {
      ag.evx[eb + n] = ftot;  // (the log's region has room: n < evneed) so evx[e + 1] - evx[e] is e's count

      SymState o = bk.sym[sl.s];
      o.best_bid = sl.bb;
      o.best_ask = sl.ba;
      o.free_head = ag.slot[i].free_head;
      const int dr = ag.slot[i].dresting;
      o.resting = (uint32_t)((int)sl.resting0 + dr);
      bk.sym[sl.s] = o;
      if (dr) atomicAdd(bk.stats + ST_RESTING, (unsigned long long)(long long)dr);
      if (sl.hidx != NIL) {
        const unsigned long long wp = sl.wbase + ftot;
        bk.hand[bk.S + sl.hidx].wptr = (uint32_t)wp;
        bk.hand[bk.S + sl.hidx].wend = (uint32_t)(wp >> 32);
      }
    }
    __syncthreads();
  }
}

// Every take event of every slot over the whole grid (a single hot symbol — config 1 — fills the chip, not
// one workgroup): a record's first take event writes its fill count and scratch start (the walk wrote the
// rest of its result), every take event its fills (the makers overlapping its interval) into the scratch
// run at its tape position. Tape-tile sums are added once per wave and tile. The slots' logs are laid end
// to end (their event counts scanned into LDS by every workgroup), so a thread's events of different slots
// are independent work, not one dependent pass per slot (config 4's ~13 hot symbols: 93 us in 13 passes).
constexpr uint32_t AGG_OUT_FLAT = 256;  // slots the flat form takes (beyond: one pass per slot)
__global__ __launch_bounds__(256) void k_agg_out(BookDev bk, BatchDev bt, AggDev ag) {
  __shared__ uint32_t xoff[AGG_OUT_FLAT + 1];  // exclusive scan of the active slots' event counts
  const uint32_t nh = min(*(volatile uint32_t*)bk.hcount, bk.S);
  const uint32_t T = gridDim.x * blockDim.x;
  const uint32_t gt = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = lane_id();
  const bool flat = nh <= AGG_OUT_FLAT;
  uint32_t ntot = 0;
  if (flat) {
    if (threadIdx.x < 64) {  // wave 0: the scan (an inactive slot counts 0)
      uint32_t run = 0;
      for (uint32_t b = 0; b < nh; b += 64) {
        const uint32_t i = b + (uint32_t)lane;
        const uint32_t c = i < nh && ag.slot[i].active ? ag.slot[i].ev_cnt : 0u;
        const uint32_t inc = (uint32_t)wave_incl_scan((long long)c);
        if (i < nh) xoff[i] = run + inc - c;
        run += rl32(inc, 63);
      }
      if (lane == 0) xoff[nh] = run;
    }
    __syncthreads();
    ntot = xoff[nh];
  }
  for (uint32_t ii = 0; ii < (flat ? 1u : nh); ++ii) {
    uint32_t nall = ntot;
    if (!flat) {
      if (!ag.slot[ii].active) continue;
      nall = ag.slot[ii].ev_cnt;
    }
    for (uint32_t t0 = gt - (uint32_t)lane; t0 < nall; t0 += T) {  // (whole waves: the tile sums below)
      const uint32_t ta = t0 + (uint32_t)lane;
      uint32_t i = ii, t = ta;
      if (flat && ta < nall) {  // the slot holding flat event ta: the last with xoff <= ta
        uint32_t lo = 0, hi = nh;  // xoff[lo] <= ta < xoff[hi]
        while (hi - lo > 1u) {
          const uint32_t mid = (lo + hi) >> 1;
          if (xoff[mid] <= ta) lo = mid; else hi = mid;
        }
        i = lo;
        t = ta - xoff[lo];
      }
      const AggSlot& slr = ag.slot[min(i, nh - 1u)];
      const uint32_t eb = slr.ev_base, n = ta < nall ? (flat ? xoff[i + 1] - xoff[i] : slr.ev_cnt) : 0u;
      const unsigned long long wbase = slr.wbase;
      const long long base = slr.base;
      const uint32_t gs = slr.gs;
      const uint32_t e = eb + t;
      AggEv E{};
      if (t < n) E = ag.ev[e];
      const bool tk = t < n && (E.j & AGG_TAKE) != 0u;
      uint32_t add = 0, tile = 0;
      if (tk) {
        const uint32_t x0 = ag.evx[e];
        if (t == 0 || ag.ev[e - 1].j != E.j) {  // the record's first take event
          uint32_t nte = 1;  // its take events follow each other in the log
          while (t + nte < n && ag.ev[e + nte].j == E.j) ++nte;
          const uint32_t nfill = ag.evx[e + nte] - x0;
          const uint32_t oi = bt.perm[E.j & ~AGG_TAKE];
          bt.res[oi].fill_count = nfill;
          bt.fstart[oi] = (uint32_t)(wbase + x0);
          add = nfill;
          tile = oi / TILE_TAPE;
        }
        const uint32_t nf = ag.evx[e + 1] - x0;
        if (nf) {
          const uint32_t first = ag.evf[e];
          const unsigned long long a = ag.eva[e], z = a + (unsigned long long)E.qty;
          const unsigned long long p = wbase + x0;
          me_fill f;
          f.taker_seq = a_seq_of(bt, E.j & ~AGG_TAKE);
          f.price_q4 = base + (long long)E.lvl;
          f.symbol = gs;
          unsigned long long lo = a;
          for (uint32_t k = 0; k < nf; ++k) {
            const AggMk m = ag.mk[first + k];
            const unsigned long long hi = m.end < z ? m.end : z;
            f.maker_seq = m.seq;
            f.qty = (int)(hi - lo);
            bt.scratch[p + k] = f;
            lo = hi;
          }
        }
      }
      // the wave's tile sums: one atomic per distinct tile (a run of records shares one)
      unsigned long long m = __ballot(add != 0u);
      while (m) {
        const uint32_t t1 = rl32(tile, __builtin_ctzll(m));
        const unsigned long long mm = __ballot(add != 0u && tile == t1);
        const uint32_t sum = (uint32_t)rli64(wave_incl_scan((mm >> lane) & 1ull ? (long long)add : 0ll), 63);
        if (lane == __builtin_ctzll(m)) atomicAdd(&bt.tile_sum[t1], sum);
        m &= ~mm;
      }
    }
  }
}

// ------------------------------------------------------------------ grouped launches (L <= 128)
// The register-window path's groups of up to ME_GMAX bucketed batches, every symbol through the
// aggregate path: k_agg_gwalk (one wave per symbol over its records of every batch of the group, from
// the batches' buckets, in batch order) replaces k_match_reg's serial loop, logging 8-B events (AggGEv);
// k_agg_gres (one workgroup per symbol) resolves every level's FIFO, places each batch's fills in its own
// scratch (the symbol's slab, or the overflow region) and fills in the results the pipeline's tape job
// reads. A record the walk
// does not cover (a cancel, a price outside the window, a bucket past BK_CAP records) hands the symbol's
// rest of the group to k_match_reg's continuation launch (me_match_reg.hip, kSlow).
struct AggGArgs {
  uint32_t* bcnt[ME_GMAX];
  const BkRec* b_rec[ME_GMAX];
  me_order_result* res[ME_GMAX];
  uint32_t* tile_sum[ME_GMAX];
  me_fill* scratch[ME_GMAX];
  unsigned long long* scratch_top[ME_GMAX];
  unsigned long long ovf_base, scratch_cap;
  const uint64_t* seq0;  // the group's first record's seq (k_agg_gres: events carry their seq's offset from it)
  uint32_t slab, ng;
};

// Ascending bitonic sort of 64 (one register) / 128 (two) distinct keys across the wave; partners over
// DPP / permlane swaps (xor_lane, me_wave.hpp), no LDS round trip per step.
template <int J>
__device__ __forceinline__ uint32_t a_bstep(uint32_t v, bool asc) {
  const uint32_t p = xor_lane<J>(v);
  const bool lower = (lane_id() & J) == 0;
  return (lower == asc) ? min(v, p) : max(v, p);
}
template <int K>
__device__ __forceinline__ uint32_t a_bmerge(uint32_t v, bool asc) {
  if constexpr (K >= 64) v = a_bstep<32>(v, asc);
  if constexpr (K >= 32) v = a_bstep<16>(v, asc);
  if constexpr (K >= 16) v = a_bstep<8>(v, asc);
  if constexpr (K >= 8) v = a_bstep<4>(v, asc);
  if constexpr (K >= 4) v = a_bstep<2>(v, asc);
  return a_bstep<1>(v, asc);
}
__device__ __forceinline__ uint32_t a_sort64(uint32_t v, bool desc) {
  const int lane = lane_id();
  v = a_bmerge<2>(v, (lane & 2) == 0);
  v = a_bmerge<4>(v, (lane & 4) == 0);
  v = a_bmerge<8>(v, (lane & 8) == 0);
  v = a_bmerge<16>(v, (lane & 16) == 0);
  v = a_bmerge<32>(v, (lane & 32) == 0);
  return a_bmerge<64>(v, !desc);
}
__device__ __forceinline__ void a_sort128(uint32_t& a, uint32_t& b) {
  a = a_sort64(a, false);
  b = a_sort64(b, true);
  const uint32_t lo = min(a, b), hi = max(a, b);
  a = a_bmerge<64>(lo, true);
  b = a_bmerge<64>(hi, true);
}

struct AStage {  // a symbol's bucket of one batch, staged for the batch-order gather
  unsigned long long seq[BK_CAP];
  long long px[BK_CAP];
  int qty[BK_CAP];
  uint32_t ok[BK_CAP];
};

__device__ __forceinline__ uint32_t* a_gtab(uint32_t* t, uint32_t s, uint32_t g) { return t + (size_t)s * (ME_GMAX + 1) + g; }

// The register-window continuation takes the symbol from record `pos` (in its batch order) of batch g.
__device__ __forceinline__ uint32_t a_ghand(const BookDev& bk, uint32_t s, uint32_t g, uint32_t pos, uint32_t nsg,
                                            uint32_t wptr, uint32_t wend) {
  uint32_t idx = 0;
  if (lane_id() == 0) {
    idx = atomicAdd(bk.hcount, 1u);
    Handoff h{};
    h.s = s;
    h.g = g;
    h.pos = pos;
    h.nsg = nsg;
    h.wptr = wptr;
    h.wend = wend;
    bk.hand[idx] = h;
  }
  return rl32(idx, 0);
}

__global__ __launch_bounds__(64) void k_agg_gwalk(BookDev bk, AggGArgs ga, AggDev ag) {
  __shared__ AStage stg;
  const int lane = lane_id();
  const int L = (int)bk.L;  // <= 128
  const uint32_t ng = ga.ng;
  for (uint32_t s = blockIdx.x; s < bk.S; s += gridDim.x) {
    // lane g < ng: the symbol's records in batch g
    const uint32_t gl = min((uint32_t)lane, ng - 1u);
    const uint32_t nsv = (uint32_t)lane < ng ? ga.bcnt[gl][(size_t)s * BK_CNT_STRIDE] : 0u;
    long long t = (long long)nsv;
    const uint32_t total = (uint32_t)rli64(wave_incl_scan(t), 63);
    const SymState st = bk.sym[s];
    const long long base = rli64(st.base, 0);
    const int bb0 = rli32(st.best_bid, 0), ba0 = rli32(st.best_ask, 0);
    const uint32_t resting = rl32(st.resting, 0);
    const uint32_t nfar0 = rl32(st.nfar[0], 0), nfar1 = rl32(st.nfar[1], 0);
    gptr<AggSlot> slot = (gptr<AggSlot>)(ag.slot + s);
    const uint32_t evneed = 3u * total + min((uint32_t)L, resting) + 64u;
    uint32_t eb = 0;
    if (total && lane == 0) eb = atomicAdd(&ag.ctr[AC_EV], evneed + 64u);
    eb = (rl32(eb, 0) + 63u) & ~63u;
    const bool eok = (unsigned long long)eb + evneed <= ag.ev_cap;
    if (lane == 0) {
      AggSlot o{};
      o.s = s;
      o.base = base;
      o.ev_base = eb;
      o.lo = evneed;  // the region: evneed 8-B events, then the records' seqs and positions [total] each
      o.hi = total;   // (8 evneed + 8 total <= 16 evneed bytes: the region reserved in 16-B units)
      o.free_head = st.free_head;
      o.resting0 = resting;
      o.bb = bb0;
      o.ba = ba0;
      o.active = 0;
      o.hidx = NIL;
      o.gs = bk.gsym ? bk.gsym[s] : s;
      *slot = o;
    }
    if (!total) continue;
    GR_STAMP(bk, s, 0);
#ifdef ME_STAMPS
    unsigned long long gw_t[4] = {0ull, 0ull, 0ull, 0ull}, gw_m = stamp_now();
#endif
    if (!eok || !a_reserve(ag, slot, resting, total)) {  // no room in the pools: the whole group of the
                                                          // symbol goes to the continuation
      const uint32_t g0 = (uint32_t)__builtin_ctzll(__ballot(nsv != 0u));
      a_ghand(bk, s, g0, 0u, rl32(nsv, (int)g0), s * ga.slab, s * ga.slab + ga.slab);
      continue;
    }
    // free chunks k_match_reg parked in fcache[s][0, nfree) join the front of the free list (one header
    // store per lane), so k_agg_gres reuses them before it takes fresh chunks, and writes nfree = 0
    {
      const uint32_t nfc = min(rl32(st.nfree, 0), 64u);
      if (nfc) {
        const uint32_t fc = bk.fcache[(size_t)s * 64u + lane];
        const uint32_t nx = (uint32_t)__shfl((int)fc, min(lane + 1, 63), 64);
        if ((uint32_t)lane < nfc) bk.chunks[fc].hdr.next = (uint32_t)lane + 1u < nfc ? nx : st.free_head;
        if (lane == 0) slot->free_head = fc;
      }
    }
    LEvG w;
    AggGEv* const log8 = reinterpret_cast<AggGEv*>(ag.ev + eb);
    le_init(w, log8, 0u);  // (w.evp: relative to the region)
    // the records' seqs (offset from the group's first) and grouped positions, in walk order
    const gptr<uint32_t> rsq = vptr(reinterpret_cast<uint32_t*>(log8 + evneed));
    const gptr<uint32_t> rjs = rsq + total;
    const unsigned long long gmin = *ga.seq0;
    uint32_t rbase = 0;
    RWalk lw;
    const bool lok = lw_init(lw, bk, s, bb0, ba0);  // else: the continuation from the first record
    uint32_t hidx = NIL, gstop = ng;
    // a batch's bucket is loaded while the batch before it runs (no HBM round trip between batches)
    // (only the lanes of the bucket's records load: a 128-slot bucket holds ~64 at config 2)
    const size_t bko = (size_t)s * BK_CAP;
    BkRec n0{}, n1{};
    auto bload = [&](uint32_t g) {
      const uint32_t c = rl32(nsv, (int)g);
      if ((uint32_t)lane < c) n0 = ga.b_rec[g][bko + lane];
      if (64u + (uint32_t)lane < c) n1 = ga.b_rec[g][bko + 64 + lane];
    };
    bload(0);
    for (uint32_t g = 0; g < ng; ++g) {
      if (lane == 0) *a_gtab(ag.gev, s, g) = eb + w.evp;
      const uint32_t cnt = rl32(nsv, (int)g);
      const BkRec r0 = n0, r1 = n1;
      if (g + 1u < ng) bload(g + 1u);
      if (!cnt) continue;
      if (cnt > (uint32_t)BK_CAP) {  // an overfull bucket: the continuation rescans the batch
        hidx = a_ghand(bk, s, g, 0u, cnt, 0u, 0u);
        gstop = g;
        break;
      }
      if (lane == 0) ga.bcnt[g][(size_t)s * BK_CNT_STRIDE] = 0u;  // ready for a later group's bucket job
      stg.seq[lane] = r0.seq;
      stg.seq[64 + lane] = r1.seq;
      stg.px[lane] = r0.px;
      stg.px[64 + lane] = r1.px;
      stg.qty[lane] = r0.qty;
      stg.qty[64 + lane] = r1.qty;
      stg.ok[lane] = r0.ok;
      stg.ok[64 + lane] = r1.ok;
      uint32_t k0 = (uint32_t)lane < cnt ? ((r0.ok & BK_IDX_MASK) << 7) | (uint32_t)lane : ~0u;
      uint32_t k1 = 64u + (uint32_t)lane < cnt ? ((r1.ok & BK_IDX_MASK) << 7) | (64u + (uint32_t)lane) : ~0u;
      if (cnt > 64u)
        a_sort128(k0, k1);
      else
        k0 = a_sort64(k0, false);
      wave_mem_order();
      me_order_result* res = ga.res[g];
      bool stop = false;
      GW_T(0);
      for (uint32_t blk = 0; blk < cnt; blk += 64) {
        const uint32_t key = blk ? k1 : k0;
        const bool v = blk + (uint32_t)lane < cnt;
        const uint32_t sl = key & (BK_CAP - 1), oi = v ? key >> 7 : 0u;
        const unsigned long long oseq = stg.seq[sl];
        const long long opx = stg.px[sl];
        const int oq = v ? stg.qty[sl] : 0;
        const uint32_t okd = v ? stg.ok[sl] >> BK_KIND_SHIFT : 0u;
        const uint32_t cntb = min(64u, cnt - blk);
        uint32_t rj;
        int olm;
        const unsigned long long fastm = __ballot(a_classify(v, oseq, opx, oq, okd, base, L, nfar0, nfar1, rj, olm));
        int rr = 0;
        const bool adm = lok && lw_admit(lw, v ? oq : 0);
        if (v) {
          rsq[rbase + (uint32_t)lane] = (uint32_t)(oseq - gmin);
          rjs[rbase + (uint32_t)lane] = (g << AGG_GSHIFT) | oi;
        }
        GW_T(1);
        const uint32_t k = lw_block<AGG_GREC_SHIFT>(w, lw, oq, lw_cw(okd, olm, rj, L), rbase, adm ? fastm : 0ull,
                                                     cntb, rr);
        rbase += cntb;
        GW_T(2);
#ifdef ME_STAMPS
        gw_t[3] += k;
#endif
        if (v && (uint32_t)lane < k) res[oi] = a_result(oq, okd, rj, rr);  // fills: k_agg_gres
        if (k < cntb) {
          hidx = a_ghand(bk, s, g, blk + k, cnt, 0u, 0u);  // scratch position: k_agg_gres
          stop = true;
          break;
        }
      }
      if (stop) {
        gstop = g;
        break;
      }
    }
    // the log's end for every batch from the stop on
    for (uint32_t g = (gstop < ng ? gstop + 1u : ng) + (uint32_t)lane; g <= ng; g += 64)
      *a_gtab(ag.gev, s, g) = eb + w.evp;
    if (gstop < ng && lane == 0) *a_gtab(ag.gev, s, gstop + 1u) = eb + w.evp;
    le_end(w);
    if (lok) lw_end(lw, bk, s);  // (else the LDS copy is truncated and nothing was walked)
    const int bb = lw.bb, ba = lw.ba;
    if (lane == 0) {
      slot->ev_cnt = w.evp;
      slot->bb = bb;
      slot->ba = ba;
      slot->active = 1;
      slot->hidx = hidx;
      slot->pos = gstop;  // the batch the continuation starts in (ng: none)
    }
    GR_STAMP(bk, s, 1);
#ifdef ME_STAMPS
    if (lane == 0)
      for (int q = 0; q < 4; ++q) bk.dbg[(size_t)s * 24u + q] = gw_t[q];
#endif
  }
}

// The same walk with its per-batch set-up on a second wave (ME_GW_HELPER, default on). The walker's batch
// set-up — the bucket's load (and, gfx9's single in-order vmcnt, the wait for every store the last batch's
// records issued), its LDS staging, the batch-order sort, the records' classification and control words,
// the admission sums, the records' seq / position arrays — was ~110 of the ~615 cycles a record took on the
// walker's chain (tools/gres_probe.py, profiles/r5/s2). Here wave 1 prepares batch g + 1 into one of two LDS
// buffers while wave 0 walks batch g from the other; one workgroup barrier per batch hands them over. The
// walker keeps what depends on the chain: the log bases, the bucket-count reset (only for batches it walks:
// a hand-off's continuation still reads the later buckets), the walk, the results.
struct GwBuf {
  uint32_t cw[BK_CAP];  // record i of the batch in batch order: control word (lw_cw) ...
  int oq[BK_CAP];       // ... quantity (0: none) ...
  uint32_t oi[BK_CAP];  // ... and index in the batch (the result's position)
  unsigned long long fastm[2];  // per 64-record block: the records the walk covers (a_classify)
  long long qsum[2];            // per block: its quantities (the ladder's admission bound)
};
struct GwShared {
  AStage stg;  // the helper's staging of the raw bucket
  GwBuf buf[2];
  uint32_t go, eb, stop[2];
};

__device__ __forceinline__ void gw_prepare(GwBuf& B, AStage& stg, const AggGArgs& ga, uint32_t g, uint32_t cnt,
                                           size_t bko, long long base, int L, uint32_t nfar0, uint32_t nfar1,
                                           gptr<uint32_t> rsq, gptr<uint32_t> rjs, unsigned long long gmin,
                                           uint32_t& rbase) {
  const int lane = lane_id();
  BkRec r0{}, r1{};
  if ((uint32_t)lane < cnt) r0 = ga.b_rec[g][bko + lane];
  if (64u + (uint32_t)lane < cnt) r1 = ga.b_rec[g][bko + 64 + lane];
  stg.seq[lane] = r0.seq;
  stg.seq[64 + lane] = r1.seq;
  stg.px[lane] = r0.px;
  stg.px[64 + lane] = r1.px;
  stg.qty[lane] = r0.qty;
  stg.qty[64 + lane] = r1.qty;
  stg.ok[lane] = r0.ok;
  stg.ok[64 + lane] = r1.ok;
  uint32_t k0 = (uint32_t)lane < cnt ? ((r0.ok & BK_IDX_MASK) << 7) | (uint32_t)lane : ~0u;
  uint32_t k1 = 64u + (uint32_t)lane < cnt ? ((r1.ok & BK_IDX_MASK) << 7) | (64u + (uint32_t)lane) : ~0u;
  if (cnt > 64u)
    a_sort128(k0, k1);
  else
    k0 = a_sort64(k0, false);
  wave_mem_order();
  for (uint32_t blk = 0; blk < cnt; blk += 64) {
    const uint32_t key = blk ? k1 : k0;
    const bool v = blk + (uint32_t)lane < cnt;
    const uint32_t sl = key & (BK_CAP - 1), oi = v ? key >> 7 : 0u;
    const unsigned long long oseq = stg.seq[sl];
    const long long opx = stg.px[sl];
    const int oq = v ? stg.qty[sl] : 0;
    const uint32_t okd = v ? stg.ok[sl] >> BK_KIND_SHIFT : 0u;
    uint32_t rj;
    int olm;
    const unsigned long long fastm = __ballot(a_classify(v, oseq, opx, oq, okd, base, L, nfar0, nfar1, rj, olm));
    const long long qs = rli64(wave_incl_scan((long long)(uint32_t)max(oq, 0)), 63);
    B.cw[blk + lane] = lw_cw(okd, olm, rj, L);
    B.oq[blk + lane] = oq;
    B.oi[blk + lane] = oi;
    if (lane == 0) {
      B.fastm[blk >> 6] = fastm;
      B.qsum[blk >> 6] = qs;
    }
    if (v) {
      rsq[rbase + (uint32_t)lane] = (uint32_t)(oseq - gmin);
      rjs[rbase + (uint32_t)lane] = (g << AGG_GSHIFT) | oi;
    }
    rbase += min(64u, cnt - blk);
  }
}

__global__ __launch_bounds__(128) void k_agg_gwalk2(BookDev bk, AggGArgs ga, AggDev ag) {
  __shared__ GwShared sh;
  const int lane = lane_id();
  const bool walker = auni((int)(threadIdx.x >> 6)) == 0;
#if ME_WALK_PRIO
  if (walker) __builtin_amdgcn_s_setprio(3);  // the chain before the helper waves sharing its SIMD
#endif
  const int L = (int)bk.L;  // <= 128
  const uint32_t ng = ga.ng;
  for (uint32_t s = blockIdx.x; s < bk.S; s += gridDim.x) {
    const uint32_t gl = min((uint32_t)lane, ng - 1u);
    const uint32_t nsv = (uint32_t)lane < ng ? ga.bcnt[gl][(size_t)s * BK_CNT_STRIDE] : 0u;
    const uint32_t total = (uint32_t)rli64(wave_incl_scan((long long)nsv), 63);
    const SymState st = bk.sym[s];
    const long long base = rli64(st.base, 0);
    const int bb0 = rli32(st.best_bid, 0), ba0 = rli32(st.best_ask, 0);
    const uint32_t resting = rl32(st.resting, 0);
    const uint32_t nfar0 = rl32(st.nfar[0], 0), nfar1 = rl32(st.nfar[1], 0);
    gptr<AggSlot> slot = (gptr<AggSlot>)(ag.slot + s);
    const uint32_t evneed = 3u * total + min((uint32_t)L, resting) + 64u;
    if (walker) {
      uint32_t eb = 0;
      if (total && lane == 0) eb = atomicAdd(&ag.ctr[AC_EV], evneed + 64u);
      eb = (rl32(eb, 0) + 63u) & ~63u;
      const bool eok = (unsigned long long)eb + evneed <= ag.ev_cap;
      if (lane == 0) {
        AggSlot o{};
        o.s = s;
        o.base = base;
        o.ev_base = eb;
        o.lo = evneed;
        o.hi = total;
        o.free_head = st.free_head;
        o.resting0 = resting;
        o.bb = bb0;
        o.ba = ba0;
        o.active = 0;
        o.hidx = NIL;
        o.gs = bk.gsym ? bk.gsym[s] : s;
        *slot = o;
      }
      bool go = total != 0u;
      if (go && (!eok || !a_reserve(ag, slot, resting, total))) {  // no room: the whole group of the symbol
        const uint32_t g0 = (uint32_t)__builtin_ctzll(__ballot(nsv != 0u));  // goes to the continuation
        a_ghand(bk, s, g0, 0u, rl32(nsv, (int)g0), s * ga.slab, s * ga.slab + ga.slab);
        go = false;
      }
      if (lane == 0) {
        sh.go = go ? 1u : 0u;
        sh.eb = eb;
      }
    }
    __syncthreads();
    const bool go = auniu(sh.go) != 0u;
    const uint32_t eb = auniu(sh.eb);
    __syncthreads();  // (the walker's next symbol overwrites go / eb)
    if (!go) continue;
    GR_STAMP(bk, s, 0);
#ifdef ME_STAMPS
    unsigned long long gw_t[4] = {0ull, 0ull, 0ull, 0ull}, gw_m = stamp_now();
#endif
    AggGEv* const log8 = reinterpret_cast<AggGEv*>(ag.ev + eb);
    const gptr<uint32_t> rsq = vptr(reinterpret_cast<uint32_t*>(log8 + evneed));
    const gptr<uint32_t> rjs = rsq + total;
    const size_t bko = (size_t)s * BK_CAP;
    if (walker) {
      const uint32_t nfc = min(rl32(st.nfree, 0), 64u);
      if (nfc) {  // k_match_reg's parked free chunks join the front of the free list (k_agg_gwalk)
        const uint32_t fc = bk.fcache[(size_t)s * 64u + lane];
        const uint32_t nx = (uint32_t)__shfl((int)fc, min(lane + 1, 63), 64);
        if ((uint32_t)lane < nfc) bk.chunks[fc].hdr.next = (uint32_t)lane + 1u < nfc ? nx : st.free_head;
        if (lane == 0) slot->free_head = fc;
      }
    } else {
      uint32_t hrb = 0;
      const unsigned long long gmin = *ga.seq0;
      const uint32_t c0 = rl32(nsv, 0);
      if (c0 && c0 <= (uint32_t)BK_CAP)
        gw_prepare(sh.buf[0], sh.stg, ga, 0u, c0, bko, base, L, nfar0, nfar1, rsq, rjs, gmin, hrb);
      __syncthreads();
      for (uint32_t g = 0; g < ng; ++g) {
        const uint32_t c = g + 1u < ng ? rl32(nsv, (int)(g + 1u)) : 0u;
        if (c && c <= (uint32_t)BK_CAP)
          gw_prepare(sh.buf[(g + 1u) & 1u], sh.stg, ga, g + 1u, c, bko, base, L, nfar0, nfar1, rsq, rjs, gmin, hrb);
        __syncthreads();
        if (auniu(sh.stop[g & 1u])) break;
      }
      continue;
    }
    LEvG w;
    le_init(w, log8, 0u);
    uint32_t rbase = 0;
    RWalk lw;
    const bool lok = lw_init(lw, bk, s, bb0, ba0);
    uint32_t hidx = NIL, gstop = ng;
    __syncthreads();  // batch 0 prepared
    for (uint32_t g = 0; g < ng; ++g) {
      if (lane == 0) *a_gtab(ag.gev, s, g) = eb + w.evp;
      const uint32_t cnt = rl32(nsv, (int)g);
      bool stop = false;
      if (cnt > (uint32_t)BK_CAP) {  // an overfull bucket: the continuation rescans the batch
        hidx = a_ghand(bk, s, g, 0u, cnt, 0u, 0u);
        stop = true;
      } else if (cnt) {
        if (lane == 0) ga.bcnt[g][(size_t)s * BK_CNT_STRIDE] = 0u;  // ready for a later group's bucket job
        const GwBuf& B = sh.buf[g & 1u];
        me_order_result* res = ga.res[g];
        GW_T(0);
        for (uint32_t blk = 0; blk < cnt; blk += 64) {
          const bool v = blk + (uint32_t)lane < cnt;
          const uint32_t ocw = B.cw[blk + lane];
          const int oq = B.oq[blk + lane];
          const uint32_t oi = B.oi[blk + lane];
          const unsigned long long fastm = rl64(B.fastm[blk >> 6], 0);
          const uint32_t cntb = min(64u, cnt - blk);
          int rr = 0;
          bool adm = false;
          if (lok) {
            lw.ub += (unsigned long long)rli64(B.qsum[blk >> 6], 0);
            adm = lw.ub < LW_CAP;
          }
          GW_T(1);
          const uint32_t k = lw_block<AGG_GREC_SHIFT>(w, lw, oq, ocw, rbase, adm ? fastm : 0ull, cntb, rr);
          rbase += cntb;
          GW_T(2);
#ifdef ME_STAMPS
          gw_t[3] += k;
#endif
          if (v && (uint32_t)lane < k)
            res[oi] = a_result(oq, (ocw & LW_MKT) ? 4u : 0u, ocw >> LW_RJ_SHIFT, rr);  // fills: k_agg_gres
          if (k < cntb) {
            hidx = a_ghand(bk, s, g, blk + k, cnt, 0u, 0u);  // scratch position: k_agg_gres
            stop = true;
            break;
          }
        }
      }
      if (lane == 0) sh.stop[g & 1u] = stop ? 1u : 0u;
      __syncthreads();  // batch g + 1 prepared; the helper sees the stop
      if (stop) {
        gstop = g;
        break;
      }
    }
    for (uint32_t g = (gstop < ng ? gstop + 1u : ng) + (uint32_t)lane; g <= ng; g += 64)
      *a_gtab(ag.gev, s, g) = eb + w.evp;
    if (gstop < ng && lane == 0) *a_gtab(ag.gev, s, gstop + 1u) = eb + w.evp;
    le_end(w);
    if (lok) lw_end(lw, bk, s);
    const int bb = lw.bb, ba = lw.ba;
    if (lane == 0) {
      slot->ev_cnt = w.evp;
      slot->bb = bb;
      slot->ba = ba;
      slot->active = 1;
      slot->hidx = hidx;
      slot->pos = gstop;
    }
    GR_STAMP(bk, s, 1);
#ifdef ME_STAMPS
    if (lane == 0)
      for (int q = 0; q < 4; ++q) bk.dbg[(size_t)s * 24u + q] = gw_t[q];
#endif
  }
}

// ------------------------------------------------------------------ the grouped walk with cancels
// k_agg_gwalk_cx: k_agg_gwalk2 for groups that carry cancels (config 5's 60 %), so a cancel no longer hands
// its symbol to k_match_reg's continuation. A cancel of order X at level l removes X's remaining quantity at
// that moment. In the level's maker space (the initial FIFO's live orders, then the group's rests, each an
// interval of its quantity at its FIXED position U: the live quantity ahead of it at the group start, or the
// level's initial total plus the group's earlier rests there) the takes consume from the front, and a cancel
// shortens its maker to the part already consumed. With F_l = T0_l + R_l - X_l - tot_l the quantity the takes
// consumed so far (T0: the initial total, R: the group's rests, X: the quantities the group's cancels removed,
// tot: the live total) and C_X the quantities cancelled ahead of X (makers with U < U_X), X has consumed
// clamp(F_l - (U_X - C_X), 0, q_X) and the cancel removes the rest. X's start U_X - C_X lies between
// max(F at its rest, U_X - X_l) and U_X, so the bounds decide most cancels (untouched since it rested, or
// consumed whole); the rest take the exact C_X from the level's list of the group's cancels {U, removed} in
// LDS (its first GW_CXL; a level with more hands the symbol off when it needs the exact start). The walk logs
// a cancel as two 8-B events {removed} {U}; the resolve shortens that maker to its consumed part, so its
// interval overlaps stay exact (k_agg_gres).
// Targets: the helper wave finds every cancel's target while preparing its batch — an order of this group
// through a tagged seq-ring entry (it writes TAG | record for the group's LIMITs first; the record's seq
// confirms it), an older one through the ring / old-order table and a walk of its level's initial FIFO (its
// live quantity ahead). A rest's {U, qty | level, F} is kept in a 256-record LDS ring (the batch being walked
// and the one before) and in the symbol's HBM region, from which the helper fetches it for older records.
// Only a far level's order, one behind more than 64 chunks, a level past GW_CXN cancels in one group or past
// GW_CXP older-order cancels hands the symbol to the continuation.
constexpr uint32_t GW_CXL = 20;      // cancels a level lists per group (p99 11 on config 5's 20-batch groups)
constexpr uint32_t GW_CXN = 64;      // cancels a level takes per group (k_agg_gres stages them in lanes)
constexpr uint32_t GW_CXP = 64;      // cancels of orders from before the group per symbol and group
constexpr uint32_t GW_RING = 256;    // records of the rest ring (two batches of BK_CAP)
constexpr uint32_t CT_PRE = 1u << 31;  // target descriptor: an order from before the group (level, qty, U)
constexpr uint32_t CT_RING = 1u << 30; // ... a record of the batch being walked or the one before: the ring
constexpr uint32_t CX_TAG = 1u << 31;  // seq-ring entry of one of this group's LIMITs: TAG | its record number
constexpr uint32_t LW_CX = 1u << 30;   // control word: a cancel (lw_cw's reject reason stays below it)
constexpr uint32_t LW_RJ_MASK = 0x1FFFu;
// record-field flags of the two events of a cancel (log word bits 7 + x; k_agg_gres's sorted entries bits 16 + x)
constexpr uint32_t AGG_CXF = 1u << 14, AGG_CXU = 1u << 13, AGG_CXP = 1u << 12;
constexpr uint32_t RI_BIG = 0xFFFFFFFFu;  // rest info of a rest too large to pack (>= 2^25): its cancel hands off

struct alignas(16) GwRi {  // a LIMIT's rest: maker position U, qty << 7 | level (0: none), F at the rest
  uint32_t u, lq, f, pad;
};
struct GwCx {
  uint32_t ct0[2][BK_CAP], ct1[2][BK_CAP], ct2[2][BK_CAP], ct3[2][BK_CAP];  // per batch buffer: each cancel's
                                            // target {CT_PRE | level << 24 | qty, U, -, -} or {record | level << 16
                                            // | CT_RING, -, -, -} or {record | level << 16, U, lq, F} (from HBM)
  uint2 ent[128 * GW_CXL];                  // per level: its first GW_CXL cancels {maker position, removed}
  uint2 edum[64];                           // the other lanes' targets of a one-lane list write (and the
                                            // writes of a level's cancels past its first GW_CXL)
  GwRi ring[GW_RING];                       // the rests of the batch being walked and the one before
  // (the helper's) targets of the group's cancels so far: a second cancel of one is UNKNOWN — the first left
  // the order dead, whether it removed anything or found it consumed
  uint32_t tbit[ME_GMAX * BK_CAP / 32];     // per record of the group
  uint32_t npre, preu[GW_CXP], prel[GW_CXP];  // orders from before the group {position, level}
};

__device__ __forceinline__ uint32_t a_ldg(const uint32_t* p) {  // (past the L1: another wave's recent store)
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t a_wsum(uint32_t v) { return (uint32_t)rli64(wave_incl_scan((long long)v), 63); }

// An order from before the group (uniform seq T < gmin): live at the group start in this symbol's window?
// Ring entry, else the old-order table (seq below the horizon); then its live quantity ahead in its level's
// FIFO. d0 / d1: the descriptor; returns 0 live, 1 unknown (not live), 2 hand off.
__device__ __forceinline__ uint32_t gw_pre_target(const BookDev& bk, uint32_t s, unsigned long long T, long long base,
                                                  uint32_t& d0, uint32_t& d1) {
  const int lane = lane_id();
  const SeqState sqs = bk.sq[bk.sq_idx];
  auto live = [&](uint32_t g) -> bool {
    if (g == NIL || g / ME_C >= bk.nchunks) return false;
    const Chunk* c = bk.chunks + g / ME_C;
    return auniu(c->owner) == s && (unsigned long long)rl64(c->seq[g % ME_C], 0) == T && (int)auniu((uint32_t)c->qty[g % ME_C]) > 0;
  };
  uint32_t g = auniu(a_ldg(bk.loc + (T & bk.ring_mask)));
  if (!live(g)) {
    if (T >= sqs.horizon) return 1u;
    g = old_lookup((gptr<const OldEnt>)bk.old, bk.old_mask, sqs.epoch, T);
    if (!live(g)) return 1u;
  }
  const uint32_t cx = g / ME_C, sx = g % ME_C;
  const long long px = rli64(bk.chunks[cx].hdr.price, 0);
  const unsigned long long off = (unsigned long long)px - (unsigned long long)base;
  if (off >= (unsigned long long)bk.L) return 2u;  // a far level: the continuation
  const uint32_t q = auniu((uint32_t)bk.chunks[cx].qty[sx]);
  if (q >= (1u << 24)) return 2u;
  unsigned long long U = 0;
  uint32_t ch = auniu(bk.levels[(size_t)s * bk.L + off].head);
  for (uint32_t steps = 0; ch != cx; ++steps) {
    if (ch >= bk.nchunks || steps >= 64u) return 2u;
    const int qv = lane < ME_C ? bk.chunks[ch].qty[lane] : 0;
    U += a_wsum((uint32_t)max(qv, 0));
    ch = auniu(bk.chunks[ch].hdr.next);
  }
  const int qv = lane < (int)sx ? bk.chunks[cx].qty[lane] : 0;
  U += a_wsum((uint32_t)max(qv, 0));
  if (U >= (1ull << 31)) return 2u;
  d0 = CT_PRE | ((uint32_t)off << 24) | q;
  d1 = (uint32_t)U;
  return 0u;
}

// The symbol's per-record rest info in HBM (beside rsq / rjs in its log region): U, qty << 7 | level, F.
struct GwRest {
  gptr<GwRi> r;  // [total] (16-B aligned: the log region starts 64-event aligned)
};

// gw_prepare with cancels: the same batch set-up, the group's LIMITs tagged in the seq ring (and their rest
// info cleared), then every cancel's target classified (cw: unknown -> ME_RJ_UNKNOWN_ORDER; fastm: hand-offs
// cleared; the descriptor). cut: the first record of the batch the walker walks now (older ones: from HBM);
// Bp: that batch's buffer (the targets' levels in their control words).
__device__ __forceinline__ void gw_prepare_cx(GwBuf& B, const GwBuf& Bp, GwCx& X, uint32_t bsel, AStage& stg,
                                              const AggGArgs& ga, const BookDev& bk, uint32_t s, uint32_t g,
                                              uint32_t cnt, size_t bko, long long base, int L, uint32_t nfar0,
                                              uint32_t nfar1, gptr<uint32_t> rsq, gptr<uint32_t> rjs,
                                              const GwRest& ri, unsigned long long gmin, uint32_t& rbase,
                                              uint32_t cut) {
  const int lane = lane_id();
  BkRec r0{}, r1{};
  if ((uint32_t)lane < cnt) r0 = ga.b_rec[g][bko + lane];
  if (64u + (uint32_t)lane < cnt) r1 = ga.b_rec[g][bko + 64 + lane];
  stg.seq[lane] = r0.seq;
  stg.seq[64 + lane] = r1.seq;
  stg.px[lane] = r0.px;
  stg.px[64 + lane] = r1.px;
  stg.qty[lane] = r0.qty;
  stg.qty[64 + lane] = r1.qty;
  stg.ok[lane] = r0.ok;
  stg.ok[64 + lane] = r1.ok;
  uint32_t k0 = (uint32_t)lane < cnt ? ((r0.ok & BK_IDX_MASK) << 7) | (uint32_t)lane : ~0u;
  uint32_t k1 = 64u + (uint32_t)lane < cnt ? ((r1.ok & BK_IDX_MASK) << 7) | (64u + (uint32_t)lane) : ~0u;
  if (cnt > 64u)
    a_sort128(k0, k1);
  else
    k0 = a_sort64(k0, false);
  wave_mem_order();
  const uint32_t rb0 = rbase;
  long long tgt[2] = {0ll, 0ll};
  bool isc[2] = {false, false};
  for (uint32_t blk = 0; blk < cnt; blk += 64) {
    const uint32_t key = blk ? k1 : k0;
    const bool v = blk + (uint32_t)lane < cnt;
    const uint32_t sl = key & (BK_CAP - 1), oi = v ? key >> 7 : 0u;
    const unsigned long long oseq = stg.seq[sl];
    const long long opx = stg.px[sl];
    const int oq = v ? stg.qty[sl] : 0;
    const uint32_t okd = v ? stg.ok[sl] >> BK_KIND_SHIFT : 0u;
    const bool cancel = v && ((okd >> 3) & 1u);
    uint32_t rj;
    int olm;
    const bool cov = a_classify(v, oseq, opx, oq, okd, base, L, nfar0, nfar1, rj, olm);
    const unsigned long long fastm = __ballot(cov || cancel);
    const long long qs = rli64(wave_incl_scan(cancel ? 0ll : (long long)(uint32_t)max(oq, 0)), 63);
    B.cw[blk + lane] = cancel ? LW_CX : lw_cw(okd, olm, rj, L);
    B.oq[blk + lane] = cancel ? 0 : oq;
    B.oi[blk + lane] = oi;
    if (lane == 0) {
      B.fastm[blk >> 6] = fastm;
      B.qsum[blk >> 6] = qs;
    }
    const uint32_t j = rbase + (uint32_t)lane;
    if (v) {
      rsq[j] = (uint32_t)(oseq - gmin);
      rjs[j] = (g << AGG_GSHIFT) | oi;
      // a LIMIT of this group the walk may rest: its ring entry names its record until k_agg_gres places it
      // (and its rest info reads "none" until the walker writes it)
      if (!cancel && !((okd >> 2) & 1u) && cov && rj == 0u) {
        bk.loc[oseq & bk.ring_mask] = CX_TAG | j;
        ri.r[j].lq = 0u;
      }
    }
    tgt[blk >> 6] = opx;
    isc[blk >> 6] = cancel;
    rbase += min(64u, cnt - blk);
  }
  if (!__ballot(isc[0] || isc[1])) return;
  a_drain();  // the tags and record seqs above, before the lookups below read them
  for (uint32_t blk = 0; blk < cnt; blk += 64) {
    const bool c = isc[blk >> 6];
    const unsigned long long T = (unsigned long long)tgt[blk >> 6];
    const uint32_t jself = rb0 + blk + (uint32_t)lane;
    uint32_t d0 = 0, d1 = 0, d2 = 0, d3 = 0, cls = 1;  // 0 live, 1 unknown, 2 hand off
    if (c && T >= gmin && T - gmin < (1ull << 32)) {  // this group's order: its tagged ring entry, confirmed by its seq
      const uint32_t e = a_ldg(bk.loc + (T & bk.ring_mask));
      const uint32_t jj = e & ~CX_TAG;
      if ((e & CX_TAG) && jj < jself && a_ldg((const uint32_t*)&rsq[jj]) == (uint32_t)(T - gmin)) {
        cls = 0u;
        if (jj >= cut) {  // walked in this batch or the one before: the walker reads the ring; its level now
          const uint32_t cwt = jj >= rb0 ? B.cw[jj - rb0] : Bp.cw[jj - cut];
          d0 = jj | ((cwt & 127u) << 16) | CT_RING;
        } else {  // walked before: its rest info from HBM now
          const GwRi q = ri.r[jj];
          d0 = jj | ((q.lq & 127u) << 16);
          d1 = q.u;
          d2 = q.lq;
          d3 = q.f;
        }
      }
    }
    unsigned long long pm = __ballot(c && T < gmin);
    while (pm) {  // orders from before the group: one at a time (~0.6 per symbol and group at config 5)
      const int i = __builtin_ctzll(pm);
      pm &= pm - 1ull;
      uint32_t e0 = 0, e1 = 0;
      const uint32_t r = gw_pre_target(bk, s, rl64(T, i), base, e0, e1);
      if (lane == i) {
        cls = r;
        d0 = e0;
        d1 = e1;
      }
    }
    // a target some earlier cancel of the group named is dead: UNKNOWN (records in order, lane by lane)
    for (unsigned long long m = __ballot(c && cls == 0u); m; m &= m - 1ull) {
      const int i = __builtin_ctzll(m);
      const uint32_t e0 = rl32(d0, i);
      uint32_t r = 0;  // 0 first, 1 seen, 2 no room
      if (e0 & CT_PRE) {
        const uint32_t pu = rl32(d1, i), pl = (e0 >> 24) & 127u, np = auniu(X.npre);
        const bool vp = (uint32_t)lane < np;
        if (__ballot(vp && X.preu[vp ? lane : 0] == pu && X.prel[vp ? lane : 0] == pl)) {
          r = 1u;
        } else if (np >= GW_CXP) {
          r = 2u;
        } else if (lane == 0) {
          X.preu[np] = pu;
          X.prel[np] = pl;
          X.npre = np + 1u;
        }
      } else {
        static_assert(ME_GMAX * BK_CAP <= 4096, "a group's record numbers fit the descriptor's 12-bit mask");
        const uint32_t jj = e0 & 0xFFFu, wd = auniu(X.tbit[jj >> 5]);
        if ((wd >> (jj & 31u)) & 1u)
          r = 1u;
        else if (lane == 0)
          X.tbit[jj >> 5] = wd | (1u << (jj & 31u));
      }
      if (lane == i && r) cls = r;
    }
    if (c) {
      X.ct0[bsel][blk + lane] = d0;
      X.ct1[bsel][blk + lane] = d1;
      X.ct2[bsel][blk + lane] = d2;
      X.ct3[bsel][blk + lane] = d3;
      if (cls == 1u) B.cw[blk + lane] = LW_CX | ((uint32_t)ME_RJ_UNKNOWN_ORDER << LW_RJ_SHIFT);
    }
    const unsigned long long ho = __ballot(c && cls == 2u);
    if (ho && lane == 0) B.fastm[blk >> 6] &= ~ho;
  }
}

// The group's per-level state in registers (level l: lane l & 63 of [l >> 6]), beside the ladder's totals:
// initial total, the group's rests, its cancels, the quantity they removed. Reads are v_readlane, writes
// v_writelane — no LDS round trip on the chain.
struct GwLvR {
  uint32_t t0[2], rl[2], n[2], xl[2];
};
__device__ __forceinline__ uint32_t gv_get(const uint32_t (&v)[2], uint32_t l) {  // (as lw_get)
  const uint32_t a = rl32(v[0], (int)(l & 63u)), b = rl32(v[1], (int)(l & 63u));
  return (l & 64u) ? b : a;
}
__device__ __forceinline__ void gv_put(uint32_t (&v)[2], uint32_t l, uint32_t x) {
  const int lane = lane_id();
  v[0] = lane == (int)l ? x : v[0];
  v[1] = lane == (int)l - 64 ? x : v[1];
}

// The chain of a block with cancels (lw_block's loop; a LIMIT also records its rest info, cancels as above).
// Returns the records walked: fewer than cnt at the first one the walk does not cover.
// Rest info: record r of the block keeps its {U, qty << 7 | level, F} in lane r of three VGPRs (a cancel of
// it later in the block reads them there); at the block's end the lanes store them to the LDS ring and, for
// rests, to HBM. A cancel of a record from an earlier block has its target's rest info loaded at the block's
// start, one vector LDS read for the block, so the chain reads it with v_readlane too.
__device__ __forceinline__ uint32_t lw_block_cx(LEvG& e, RWalk& w, GwLvR& V, GwCx& X, const GwRest& ri, int oq,
                                                uint32_t ocw, uint32_t c0v, uint32_t c1v, uint32_t c2v, uint32_t c3v,
                                                uint32_t jb, unsigned long long fastm, uint32_t cnt, int& rr,
                                                unsigned long long* rt) {
  const int lane = lane_id();
  const unsigned long long upto = (cnt >= 64u ? ~0ull : ((1ull << cnt) - 1ull)) & ~fastm;
  uint32_t k = upto ? (uint32_t)__builtin_ctzll(upto) : cnt;
  const unsigned long long rjm = __ballot(((ocw >> LW_RJ_SHIFT) & LW_RJ_MASK) != 0u);
  // the cancels' targets: {U, lq, F} per cancel lane (older orders: from the descriptor; earlier records:
  // HBM's from the helper, or the ring's now); a target earlier in this block: its lane of bu / blq / bf
  // (a PRE descriptor's level spans bits 24-30, CT_RING's bit among them: test CT_RING only without CT_PRE)
  const bool isx = (uint32_t)lane < cnt && (ocw & LW_CX) != 0u;
  const bool xpre = isx && (c0v & CT_PRE) != 0u;
  const bool xring = isx && (c0v & (CT_PRE | CT_RING)) == CT_RING;
  const uint32_t xj = c0v & 0xFFFFu;
  const unsigned long long samem = __ballot(xring && xj >= jb), prem = __ballot(xpre);
  const uint32_t tlv = xpre ? (c0v >> 24) & 127u : (c0v >> 16) & 127u;  // the target's level
  uint32_t su = xring && xj >= jb ? xj - jb : c1v, slq = c2v, sf = c3v;  // (same block: the target's lane)
  if (xring && xj < jb) {
    const GwRi R = X.ring[xj & (GW_RING - 1u)];
    su = R.u;
    slq = R.lq;
    sf = R.f;
  }
  if (xpre) {
    slq = ((c0v & 0xFFFFFFu) << 7) | ((c0v >> 24) & 127u);
    sf = 0u;  // (nothing consumed at the group start)
  }
  uint32_t bu = 0u, blq = 0u, bf = 0u;
#ifdef ME_STAMPS
  // (the stamps build: cycles by record kind — cancels the bounds decide, LIMITs, MARKETs, cancels that read
  // the level's list — in rt[0..3], counts in rt[4..7]; rt[8]: cancels that emptied a best level, rt[9]: of
  // orders from before the group)
  unsigned long long rt_m = stamp_now();
  int rt_k = -1;
#define RT_MARK(kind)                            \
  do {                                           \
    const unsigned long long _n = stamp_now();   \
    if (rt_k >= 0) {                             \
      rt[rt_k] += _n - rt_m;                     \
      rt[rt_k + 4] += 1ull;                      \
    }                                            \
    rt_m = _n;                                   \
    rt_k = (kind);                               \
  } while (0)
#else
#define RT_MARK(kind) ((void)0)
#endif
  unsigned long long work = (k >= 64u ? ~0ull : ((1ull << k) - 1ull)) & ~rjm;
  while (work) {
    const int r = __builtin_ctzll(work);
    asm volatile("s_bitset0_b64 %0, %1" : "+s"(work) : "s"(r));
    const uint32_t cw = rl32(ocw, r);
    const uint32_t jr = jb + (uint32_t)r;
    RT_MARK((cw & LW_CX) ? 0 : (cw & LW_MKT) ? 2 : 1);
    if (cw & LW_CX) {
      const bool pre = (prem >> r) & 1ull;
      const uint32_t l = rl32(tlv, r);
      uint32_t U, lq, Fr;
      if ((samem >> r) & 1ull) {
        const int x = (int)rl32(su, r);
        U = rl32(bu, x);
        lq = rl32(blq, x);
        Fr = rl32(bf, x);
      } else {
        U = rl32(su, r);
        lq = rl32(slq, r);
        Fr = rl32(sf, r);
      }
      if (lq == RI_BIG) {  // (before anything changed: the continuation from here)
        k = (uint32_t)r;
        break;
      }
      const uint32_t q = lq >> 7;  // (0: never rested — a LIMIT filled at once)
      const uint32_t tot = (int)l == w.bb ? w.cbb : (int)l == w.ba ? w.cba : lw_get(w, (int)l);
      const uint32_t n = gv_get(V.n, l), xr = gv_get(V.xl, l), t0 = gv_get(V.t0, l);
      const uint32_t F = t0 + gv_get(V.rl, l) - xr - tot;  // consumed by the group's takes
      const uint32_t lo = max(Fr, U > xr ? U - xr : 0u);    // X's start is at least this, and at most U
      uint32_t cons = F <= lo ? 0u : q;
      if (ME_UNLIKELY(F > lo && F < U + q)) {  // the bounds do not decide: the exact start from the list
        if (n > GW_CXL) {                      // it no longer holds every cancel: the continuation
          k = (uint32_t)r;
          break;
        }
#ifdef ME_STAMPS
        rt_k = 3;
#endif
        const bool vl = (uint32_t)lane < n;
        const uint2 ce = vl ? X.ent[l * GW_CXL + lane] : make_uint2(0u, 0u);
        const uint32_t st = U - a_wsum(vl && ce.x < U ? ce.y : 0u);
        cons = F > st ? min(F - st, q) : 0u;
      }
      const uint32_t rem = q - cons;
      if (rem) {
        if (n + 1u >= GW_CXN) {
          k = (uint32_t)r;
          break;
        }
        {  // (one-lane write without an exec change: the other lanes, and a full list, write dummy slots)
          uint2* ep = lane == 0 && n < GW_CXL ? &X.ent[l * GW_CXL + n] : &X.edum[lane];
          *ep = make_uint2(U, rem);
        }
        gv_put(V.n, l, n + 1u);
        gv_put(V.xl, l, xr + rem);
        if ((int)l == w.bb) {
          w.cbb -= rem;
          if (!w.cbb) {
#ifdef ME_STAMPS
            rt[8] += 1ull;
#endif
            lw_put(w, w.bb, 0u);
            w.bb = lw_prev(w, w.bb - 1, w.cbb);
          }
        } else if ((int)l == w.ba) {
          w.cba -= rem;
          if (!w.cba) {
#ifdef ME_STAMPS
            rt[8] += 1ull;
#endif
            lw_put(w, w.ba, 0u);
            w.ba = lw_next(w, w.ba + 1, w.cba);
          }
        } else {
          lw_add(w, (int)l, 0u - rem);
        }
#ifdef ME_STAMPS
        if (pre) rt[9] += 1ull;
#endif
        const uint32_t flg = pre ? AGG_CXF | AGG_CXP : AGG_CXF;
        le_emit2(e, l, (jr | flg) << AGG_GREC_SHIFT, rem, (jr | flg | AGG_CXU) << AGG_GREC_SHIFT,
                 pre ? U : U - t0);  // the FIFO's / the rests' position
      }
      asm volatile("s_mov_b32 m0, %1\n\tv_writelane_b32 %0, %2, m0" : "+v"(rr) : "s"(r), "s"(rem) : "m0");
      continue;
    }
    uint32_t rem = (uint32_t)rli32(oq, r);
    const uint32_t jt = jr << AGG_GREC_SHIFT;
    const int lim = (int)(cw & LW_LIM);
    uint32_t rq;
    if (cw & LW_BUY) {
      lw_take_buy<LEvG>(e, w, lim, rem, jt | AGG_TAKE);
      rq = (cw & LW_MKT) ? 0u : rem;
      asm volatile("" : "+s"(rq));
      if (rq) lw_rest_buy<LEvG>(e, w, lim, rq, jt);
    } else {
      lw_take_sell<LEvG>(e, w, lim, rem, jt | AGG_TAKE);
      rq = (cw & LW_MKT) ? 0u : rem;
      asm volatile("" : "+s"(rq));
      if (rq) lw_rest_sell<LEvG>(e, w, lim, rq, jt);
    }
    // a rest's info: its maker position and what the level's takes had consumed when it rested (a lower
    // bound on its start ever after); a LIMIT that did not rest keeps lq 0 ("none")
    if (rq) {
      const uint32_t rl = gv_get(V.rl, (uint32_t)lim);
      const uint32_t tot = lim == w.bb ? w.cbb : lim == w.ba ? w.cba : lw_get(w, lim);
      const uint32_t ou = gv_get(V.t0, (uint32_t)lim) + rl;
      const uint32_t of = ou + rq - gv_get(V.xl, (uint32_t)lim) - tot;
      const uint32_t olq = rq < (1u << 25) ? (rq << 7) | (uint32_t)lim : RI_BIG;
      gv_put(V.rl, (uint32_t)lim, rl + rq);
      asm volatile("s_mov_b32 m0, %3\n\tv_writelane_b32 %0, %4, m0\n\tv_writelane_b32 %1, %5, m0\n\tv_writelane_b32 %2, %6, m0"
                   : "+v"(bu), "+v"(blq), "+v"(bf)
                   : "s"(r), "s"(ou), "s"(olq), "s"(of)
                   : "m0");
    }
    asm volatile("s_mov_b32 m0, %1\n\tv_writelane_b32 %0, %2, m0" : "+v"(rr) : "s"(r), "s"(auniu(rem)) : "m0");
  }
  RT_MARK(-1);
#undef RT_MARK
  // the block's rest info: the ring (cancels in later blocks of this batch and the next) and, for rests, HBM
  // (the helper's, for cancels in later batches)
  if ((uint32_t)lane < k) {
    GwRi o;
    o.u = bu;
    o.lq = blq;
    o.f = bf;
    o.pad = 0u;
    X.ring[(jb + (uint32_t)lane) & (GW_RING - 1u)] = o;
    if (blq) ri.r[jb + (uint32_t)lane] = o;
  }
  return k;
}

// A cancel's result: CANCELED with the quantity removed, or REJECTED / UNKNOWN_ORDER (the oracle's order of
// checks: a cancel is never rejected for its quantity, side or seq).
__device__ __forceinline__ me_order_result a_result_cx(uint32_t rj, int rem) {
  me_order_result o;
  const bool ok = rj == 0u && rem > 0;
  o.filled_qty = 0;
  o.remaining_qty = ok ? rem : 0;
  o.fill_count = 0;
  o.tape_offset = 0;
  o.status = (uint8_t)(ok ? ME_ST_CANCELED : ME_ST_REJECTED);
  o.reason = (uint8_t)(ok ? ME_RJ_NONE : ME_RJ_UNKNOWN_ORDER);
  o.pad[0] = o.pad[1] = 0;
  return o;
}

__global__ __launch_bounds__(128) void k_agg_gwalk_cx(BookDev bk, AggGArgs ga, AggDev ag) {
  __shared__ GwShared sh;
  __shared__ GwCx cx;
  const int lane = lane_id();
  const bool walker = auni((int)(threadIdx.x >> 6)) == 0;
#if ME_WALK_PRIO
  if (walker) __builtin_amdgcn_s_setprio(3);
#endif
  const int L = (int)bk.L;  // <= 128
  const uint32_t ng = ga.ng;
  for (uint32_t s = blockIdx.x; s < bk.S; s += gridDim.x) {
    const uint32_t gl = min((uint32_t)lane, ng - 1u);
    const uint32_t nsv = (uint32_t)lane < ng ? ga.bcnt[gl][(size_t)s * BK_CNT_STRIDE] : 0u;
    const uint32_t total = (uint32_t)rli64(wave_incl_scan((long long)nsv), 63);
    const SymState st = bk.sym[s];
    const long long base = rli64(st.base, 0);
    const int bb0 = rli32(st.best_bid, 0), ba0 = rli32(st.best_ask, 0);
    const uint32_t resting = rl32(st.resting, 0);
    const uint32_t nfar0 = rl32(st.nfar[0], 0), nfar1 = rl32(st.nfar[1], 0);
    gptr<AggSlot> slot = (gptr<AggSlot>)(ag.slot + s);
    const uint32_t evneed = 3u * total + min((uint32_t)L, resting) + 64u;
    if (walker) {
      uint32_t eb = 0;
      if (total && lane == 0) eb = atomicAdd(&ag.ctr[AC_EV], evneed + 64u);
      eb = (rl32(eb, 0) + 63u) & ~63u;
      const bool eok = (unsigned long long)eb + evneed <= ag.ev_cap;
      if (lane == 0) {
        AggSlot o{};
        o.s = s;
        o.base = base;
        o.ev_base = eb;
        o.lo = evneed;
        o.hi = total;
        o.free_head = st.free_head;
        o.resting0 = resting;
        o.bb = bb0;
        o.ba = ba0;
        o.active = 0;
        o.hidx = NIL;
        o.gs = bk.gsym ? bk.gsym[s] : s;
        *slot = o;
      }
      bool go = total != 0u;
      if (go && (!eok || !a_reserve(ag, slot, resting, total))) {
        const uint32_t g0 = (uint32_t)__builtin_ctzll(__ballot(nsv != 0u));
        a_ghand(bk, s, g0, 0u, rl32(nsv, (int)g0), s * ga.slab, s * ga.slab + ga.slab);
        go = false;
      }
      if (lane == 0) {
        sh.go = go ? 1u : 0u;
        sh.eb = eb;
      }
    }
    __syncthreads();
    const bool go = auniu(sh.go) != 0u;
    const uint32_t eb = auniu(sh.eb);
    __syncthreads();
    if (!go) continue;
    AggGEv* const log8 = reinterpret_cast<AggGEv*>(ag.ev + eb);
    // the region: evneed 8-B events, then the records' seqs and positions [total] each, then (16-B aligned)
    // their rest info [total] (8 evneed + 24 total + 16 <= 16 evneed bytes: evneed >= 3 total + 64)
    const gptr<uint32_t> rsq = vptr(reinterpret_cast<uint32_t*>(log8 + evneed));
    const gptr<uint32_t> rjs = rsq + total;
    GwRest ri;
    ri.r = vptr(reinterpret_cast<GwRi*>((reinterpret_cast<uintptr_t>(log8 + evneed) + 8ull * total + 15ull) & ~15ull));
    const size_t bko = (size_t)s * BK_CAP;
    if (walker) {
      const uint32_t nfc = min(rl32(st.nfree, 0), 64u);
      if (nfc) {
        const uint32_t fc = bk.fcache[(size_t)s * 64u + lane];
        const uint32_t nx = (uint32_t)__shfl((int)fc, min(lane + 1, 63), 64);
        if ((uint32_t)lane < nfc) bk.chunks[fc].hdr.next = (uint32_t)lane + 1u < nfc ? nx : st.free_head;
        if (lane == 0) slot->free_head = fc;
      }
    } else {
      uint32_t hrb = 0;
      const unsigned long long gmin = *ga.seq0;
      const uint32_t c0 = rl32(nsv, 0);
      for (uint32_t j = (uint32_t)lane; j < ME_GMAX * BK_CAP / 32; j += 64) cx.tbit[j] = 0u;
      if (lane == 0) cx.npre = 0u;
      wave_mem_order();
#ifdef ME_STAMPS
      unsigned long long h_t = 0, h_m = stamp_now();
#endif
      if (c0 && c0 <= (uint32_t)BK_CAP)
        gw_prepare_cx(sh.buf[0], sh.buf[1], cx, 0u, sh.stg, ga, bk, s, 0u, c0, bko, base, L, nfar0, nfar1, rsq, rjs,
                      ri, gmin, hrb, 0u);
#ifdef ME_STAMPS
      h_t += stamp_now() - h_m;
#endif
      __syncthreads();
      for (uint32_t g = 0; g < ng; ++g) {
        const uint32_t c = g + 1u < ng ? rl32(nsv, (int)(g + 1u)) : 0u;
        // batch g's first record: when batch g + 1 is walked the ring holds batches g and g + 1
        const uint32_t cg = rl32(nsv, (int)g);
        const uint32_t cut = hrb - (cg <= (uint32_t)BK_CAP ? cg : 0u);
#ifdef ME_STAMPS
        h_m = stamp_now();
#endif
        if (c && c <= (uint32_t)BK_CAP)
          gw_prepare_cx(sh.buf[(g + 1u) & 1u], sh.buf[g & 1u], cx, (g + 1u) & 1u, sh.stg, ga, bk, s, g + 1u, c, bko,
                        base, L, nfar0, nfar1, rsq, rjs, ri, gmin, hrb, cut);
#ifdef ME_STAMPS
        h_t += stamp_now() - h_m;
#endif
        __syncthreads();
        if (auniu(sh.stop[g & 1u])) break;
      }
#ifdef ME_STAMPS
      if (lane == 0) bk.dbg[(size_t)s * 24u + 5u] = h_t;
#endif
      continue;
    }
    GR_STAMP(bk, s, 0);
#ifdef ME_STAMPS
    unsigned long long gw_t[4] = {0ull, 0ull, 0ull, 0ull}, gw_m = stamp_now();
    unsigned long long gw_rt[10] = {0ull, 0ull, 0ull, 0ull, 0ull, 0ull, 0ull, 0ull, 0ull, 0ull};
#else
    unsigned long long* const gw_rt = nullptr;
#endif
    LEvG w;
    le_init(w, log8, 0u);
    uint32_t rbase = 0;
    RWalk lw;
    const bool lok = lw_init(lw, bk, s, bb0, ba0);
    GwLvR lv;  // the levels' initial totals (the ladder's, exact at its start), no rests or cancels yet
    lv.t0[0] = lw.t0;
    lv.t0[1] = lw.t1;
    lv.rl[0] = lv.rl[1] = lv.n[0] = lv.n[1] = lv.xl[0] = lv.xl[1] = 0u;
    uint32_t hidx = NIL, gstop = ng;
    GW_T(1);
    __syncthreads();  // batch 0 prepared
    GW_T(0);
    for (uint32_t g = 0; g < ng; ++g) {
      if (lane == 0) *a_gtab(ag.gev, s, g) = eb + w.evp;
      const uint32_t cnt = rl32(nsv, (int)g);
      bool stop = false;
      if (cnt > (uint32_t)BK_CAP) {
        hidx = a_ghand(bk, s, g, 0u, cnt, 0u, 0u);
        stop = true;
      } else if (cnt) {
        if (lane == 0) ga.bcnt[g][(size_t)s * BK_CNT_STRIDE] = 0u;
        const GwBuf& B = sh.buf[g & 1u];
        me_order_result* res = ga.res[g];
        for (uint32_t blk = 0; blk < cnt; blk += 64) {
          const bool v = blk + (uint32_t)lane < cnt;
          const uint32_t ocw = B.cw[blk + lane];
          const int oq = B.oq[blk + lane];
          const uint32_t oi = B.oi[blk + lane];
          const uint32_t b2 = g & 1u;
          const uint32_t c0v = cx.ct0[b2][blk + lane], c1v = cx.ct1[b2][blk + lane];
          const uint32_t c2v = cx.ct2[b2][blk + lane], c3v = cx.ct3[b2][blk + lane];
          const unsigned long long fastm = rl64(B.fastm[blk >> 6], 0);
          const uint32_t cntb = min(64u, cnt - blk);
          int rr = 0;
          bool adm = false;
          if (lok) {
            lw.ub += (unsigned long long)rli64(B.qsum[blk >> 6], 0);
            adm = lw.ub < LW_CAP;
          }
          GW_T(1);
          const uint32_t k = lw_block_cx(w, lw, lv, cx, ri, oq, ocw, c0v, c1v, c2v, c3v, rbase, adm ? fastm : 0ull, cntb, rr,
                                         gw_rt);
          GW_T(2);
#ifdef ME_STAMPS
          gw_t[3] += k;
#endif
          rbase += cntb;
          if (v && (uint32_t)lane < k) {
            const uint32_t rj = (ocw >> LW_RJ_SHIFT) & LW_RJ_MASK;
            res[oi] = (ocw & LW_CX) ? a_result_cx(rj, rr) : a_result(oq, (ocw & LW_MKT) ? 4u : 0u, rj, rr);
          }
          if (k < cntb) {
            hidx = a_ghand(bk, s, g, blk + k, cnt, 0u, 0u);
            stop = true;
            break;
          }
        }
      }
      if (lane == 0) sh.stop[g & 1u] = stop ? 1u : 0u;
      GW_T(1);
      __syncthreads();
      GW_T(0);
      if (stop) {
        gstop = g;
        break;
      }
    }
    for (uint32_t g = (gstop < ng ? gstop + 1u : ng) + (uint32_t)lane; g <= ng; g += 64)
      *a_gtab(ag.gev, s, g) = eb + w.evp;
    if (gstop < ng && lane == 0) *a_gtab(ag.gev, s, gstop + 1u) = eb + w.evp;
    le_end(w);
    if (lok) lw_end(lw, bk, s);
    const int bb = lw.bb, ba = lw.ba;
    if (lane == 0) {
      slot->ev_cnt = w.evp;
      slot->bb = bb;
      slot->ba = ba;
      slot->active = 1;
      slot->hidx = hidx;
      slot->pos = gstop;
    }
    GR_STAMP(bk, s, 1);
#ifdef ME_STAMPS
    if (lane == 0)
      for (int q = 0; q < 4; ++q) bk.dbg[(size_t)s * 24u + q] = gw_t[q];
    if (lane == 0)
      for (int q = 0; q < 10; ++q) bk.dbg[(size_t)s * 24u + 6u + q] = gw_rt[q];
#endif
  }
}

// ------------------------------------------------------------------ grouped launches: one workgroup per symbol
// k_agg_gres does the work of the hot path's k_agg_group ... k_agg_out for a grouped launch in ONE launch,
// one 512-thread workgroup per symbol (the walk's workgroup of the same symbol ran on the same XCD,
// blockIdx = symbol):
//   A  the symbol's log sorted by level (per-wave histograms of contiguous log ranges in LDS, a stable
//      ballot-multisplit scatter of 8-B entries {log index | record, qty} into the slot's region of
//      AggDev::evq), so phases B and D read each level's events as one contiguous run instead of gathering
//      them from the log line by line; a seq is read from the symbol's own record array beside its log;
//   B  its levels resolved by the waves (a level per wave, taken from an LDS counter): the initial FIFO
//      walked until the group's takes are covered, consumed makers, emptied chunks, each take's fill count
//      into an LDS array indexed by log position; the slot's cursors are LDS atomics, not pool-wide ones;
//   C  the fill offsets (exclusive scan of the fill counts in log order = tape order, in place, each wave
//      over its log range), each batch's scratch base, the records' fill counts and scratch starts;
//   D  the chunk allocation (wave 0), then per level in one pass over its events: the fills of its takes and
//      the surviving rests placed into the level's tail and new chunks.
// The per-event LDS array (fill counts) holds `ne` events (the launch sizes it from the group's mean records
// per symbol); a symbol with a longer log keeps it in the log's own HBM region (AggDev::evn) instead.
// ~16 KB of static LDS and a register budget of GR_WPE waves per SIMD.
#ifndef GR_WAVES
#define GR_WAVES 8  // waves per workgroup (same-box A/B)
#endif
constexpr uint32_t GR_THREADS = GR_WAVES * 64;
#ifndef GR_WPE
#define GR_WPE 8  // waves per SIMD the register budget is cut for: 8 puts all four workgroups of a CU (1,024
                  // symbols) in one round (same-box A/B, profiles/r4/g2: 640 steps 2,300 -> 2,515M, the group
                  // launch 588 -> 560 us at the driver shape; 6 was the round-3 choice)
#endif
constexpr uint64_t GR_FOUR_BELOW = 512;  // records per symbol per group below which the resolve runs 4 waves
constexpr uint32_t GR_STAGE = 48;  // consumed makers / emptied chunks a level stages in LDS (else: HBM)

struct GrLevel {  // what phase B found for one level
  unsigned long long C, T0;
  uint32_t newhead, mk_base, nmk, fr_base, nfreed, need, d_off, ks;
};
struct GrStage {  // a wave's maker / emptied-chunk staging (phases B and D)
  AggMk mk[GR_STAGE];
  uint32_t fr[GR_STAGE];
};
struct GrCxStage {  // (walks with cancels) a wave's staging of its level's cancels (the walk takes <= GW_CXN)
  uint32_t cxu[64], cxr[64], cxp[64];
};
// the cancel events' flags in the sorted entries (k_agg_gwalk_cx's AGG_CX* record-field flags << 16)
constexpr uint32_t GR_CXF = AGG_CXF << 16, GR_CXU = AGG_CXU << 16, GR_CXP = AGG_CXP << 16;
template <int NW>
struct GrShared {
  union {
    uint32_t wh[NW][128];  // phase A: per-wave level histograms, then scatter cursors
    GrStage st[NW];
  } u;
  GrLevel lv[128];
  uint32_t lstart[129];
  uint32_t lhead[128], ltail[128];
  uint32_t lvlist[128];
  uint32_t gev[ME_GMAX + 1], gex[ME_GMAX + 1], gbase[ME_GMAX + 1];
  uint32_t wsum[NW];
  uint32_t nlv, next, next2, cur_mk, cur_fr, deficit, alloc_base;
  int dresting;
  uint8_t ltend[128];
};

// Level work items of phases B and D: lane 0 takes the next from an LDS counter.
__device__ __forceinline__ uint32_t gr_take(uint32_t* ctr) {
  uint32_t i = 0;
  if (lane_id() == 0) i = atomicAdd(ctr, 1u);
  return rl32(i, 0);
}

template <int NW, bool kLds, bool CX>
__device__ __forceinline__ void gres_symbol(const BookDev& bk, const AggGArgs& ga, const AggSrc& src, const AggDev& ag,
                                            uint32_t s, const AggSlot& sl, GrShared<NW>& sh, uint32_t* nf,
                                            GrCxStage* cxs) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t L = bk.L;  // <= 128
  const uint32_t eb = sl.ev_base, n = sl.ev_cnt, ng = ga.ng;
  const AggGEv* ev = reinterpret_cast<const AggGEv*>(ag.ev + eb);
  const uint32_t* rsq = reinterpret_cast<const uint32_t*>(ev + sl.lo);  // the records' seq offsets ...
  const uint32_t* rjs = rsq + sl.hi;                                    // ... and grouped positions
  // the log sorted by level (phase A), read by phases B and D one level segment at a time (coalesced):
  // entry w = log index | record << 16 | AGG_TAKE (the level is the segment's)
  AggGEv* const srt = reinterpret_cast<AggGEv*>(ag.evq + eb);
  auto srec = [](uint32_t w) -> uint32_t { return (w >> 16) & 0x7FFFu; };
  const size_t lo_l = (size_t)s * L;
  // every seq of the group lies in [gmin, gmin + seq_ring) (k_seq_sweep's check; seq_ring <= 2^32 here)
  const unsigned long long gmin = *ga.seq0;
  GR_STAMP(bk, s, 2);
  // ---- A: level heads (one coalesced load), the batches' log boundaries, the scalars
  if ((uint32_t)tid < L) {
    const Level v = bk.levels[lo_l + tid];
    sh.lhead[tid] = v.head;
    sh.ltail[tid] = v.tail;
    sh.ltend[tid] = bk.tend[lo_l + tid];
  }
  if ((uint32_t)tid <= ng) sh.gev[tid] = *a_gtab(ag.gev, s, (uint32_t)tid) - eb;
  if (tid == 0) {
    sh.next = sh.next2 = 0u;
    sh.cur_mk = sh.cur_fr = sh.deficit = 0u;
    sh.dresting = 0;
  }
  sh.u.wh[wv][lane] = 0u;
  sh.u.wh[wv][64 + lane] = 0u;
  wave_mem_order();
  // each wave owns a contiguous 64-aligned log range: its level histogram, then a stable scatter of the
  // same range
  const uint32_t per = ((n + NW - 1u) / NW + 63u) & ~63u;
  const uint32_t r0 = min(n, (uint32_t)wv * per), r1 = min(n, r0 + per);
#pragma unroll 4
  for (uint32_t b = r0; b < r1; b += 64) {
    const uint32_t e = b + (uint32_t)lane;
    if (e < r1) atomicAdd(&sh.u.wh[wv][ev[e].w & AGG_GLVL_MASK], 1u);
  }
  __syncthreads();
  if (wv == 0) {
    uint32_t c0 = 0, c1 = 0;
    for (int w = 0; w < NW; ++w) {
      c0 += sh.u.wh[w][lane];
      c1 += sh.u.wh[w][64 + lane];
    }
    const uint32_t i0 = (uint32_t)wave_incl_scan((long long)c0), t0 = rl32(i0, 63);
    const uint32_t i1 = (uint32_t)wave_incl_scan((long long)c1);
    uint32_t a0 = i0 - c0, a1 = t0 + i1 - c1;
    sh.lstart[lane] = a0;
    sh.lstart[64 + lane] = a1;
    if (lane == 0) sh.lstart[128] = n;
    const unsigned long long m0 = __ballot(c0 != 0u), m1 = __ballot(c1 != 0u);
    if (c0) sh.lvlist[__popcll(m0 & lanemask_lt())] = (uint32_t)lane;
    if (c1) sh.lvlist[__popcll(m0) + __popcll(m1 & lanemask_lt())] = 64u + (uint32_t)lane;
    if (lane == 0) sh.nlv = (uint32_t)(__popcll(m0) + __popcll(m1));
    for (int w = 0; w < NW; ++w) {  // wave w's events of level l start at its running base
      const uint32_t x0 = sh.u.wh[w][lane], x1 = sh.u.wh[w][64 + lane];
      sh.u.wh[w][lane] = a0;
      sh.u.wh[w][64 + lane] = a1;
      a0 += x0;
      a1 += x1;
    }
  }
  __syncthreads();
  for (uint32_t b = r0; b < r1; b += 64) {
    const uint32_t e = b + (uint32_t)lane;
    const bool v = e < r1;
    AggGEv E{};
    if (v) E = ev[e];
    const uint32_t key = v ? (E.w & AGG_GLVL_MASK) : 0u;
    unsigned long long peers = __ballot(v);
#pragma unroll
    for (uint32_t bit = 0; bit < 7; ++bit) {
      const unsigned long long bb = __ballot((key >> bit) & 1u);
      peers &= ((key >> bit) & 1u) ? bb : ~bb;
    }
    const uint32_t rank = (uint32_t)__popcll(peers & lanemask_lt());
    const uint32_t start = sh.u.wh[wv][key];
    if (v) {
      AggGEv S;
      S.w = e | (((E.w & ~AGG_TAKE) >> AGG_GREC_SHIFT) << 16) | (E.w & AGG_TAKE);
      S.qty = E.qty;
      srt[start + rank] = S;
    }
    wave_mem_order();
    if (v && rank == 0) sh.u.wh[wv][key] = start + (uint32_t)__popcll(peers);
    wave_mem_order();
  }
  __syncthreads();
  GR_STAMP(bk, s, 3);
  // ---- B: the levels
  const uint32_t nlv = sh.nlv;
  const bool act = lane < ME_C;
  AggMk* mkl = sh.u.st[wv].mk;
  uint32_t* frl = sh.u.st[wv].fr;
  auto entry = [&](uint32_t start, uint32_t cnt, uint32_t b, uint32_t& er) -> AggGEv {
    AggGEv E{};
    er = 0;
    if (b + (uint32_t)lane < cnt) {
      E = srt[start + b + lane];
      er = E.w & 0xFFFFu;
    }
    return E;
  };
  for (uint32_t it = gr_take(&sh.next); it < nlv; it = gr_take(&sh.next)) {
    const uint32_t lvl = __builtin_amdgcn_readfirstlane(sh.lvlist[it]);
    const uint32_t start = __builtin_amdgcn_readfirstlane(sh.lstart[lvl]);
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(sh.lstart[lvl + 1]) - start;
    const uint32_t head0 = __builtin_amdgcn_readfirstlane(sh.lhead[lvl]);
    const uint32_t te_raw = sh.ltend[lvl];
    uint32_t er0;
    const AggGEv E0 = entry(start, cnt, 0, er0);  // the first 64 entries stay in registers
    auto ent = [&](uint32_t b, uint32_t& er) -> AggGEv {
      if (b == 0) {
        er = er0;
        return E0;
      }
      return entry(start, cnt, b, er);
    };
    // 0. (CX) the level's cancels: pairs {removed} {maker position} into lanes (lane k: entry k, in log order).
    //    An in-group target's position is its offset in the group's rests (R before it), an older order's its
    //    live quantity ahead in the initial FIFO (flag AGG_CXP).
    uint32_t ncx = 0, tu = 0, tr = 0, tpv = 0, npre = 0;
    bool hasin = false;
    unsigned long long umax = 0;
    if constexpr (CX) {
      GrCxStage& X = cxs[wv];
      for (uint32_t b = 0; b < cnt; b += 64) {
        uint32_t er;
        const AggGEv E = ent(b, er);
        const bool v = b + (uint32_t)lane < cnt;
        const bool cu = v && (E.w & (GR_CXF | GR_CXU)) == (GR_CXF | GR_CXU);
        const unsigned long long m = __ballot(cu);
        if (!m) continue;
        const uint32_t k = ncx + (uint32_t)__popcll(m & lanemask_lt());
        if (cu && k < 64u) {
          X.cxu[k] = (uint32_t)E.qty;
          X.cxr[k] = (uint32_t)srt[start + b + lane - 1].qty;  // its first event, just before it
          X.cxp[k] = (E.w & GR_CXP) ? 1u : 0u;
        }
        ncx += (uint32_t)__popcll(m);
      }
      if (ncx > 64u) {  // (the walk takes at most GW_CXN per level and group)
        a_set_err(bk, ERR_INCONSISTENT);
        ncx = 64u;
      }
      wave_mem_order();
      if ((uint32_t)lane < ncx) {
        tu = X.cxu[lane];
        tr = X.cxr[lane];
        tpv = X.cxp[lane];
      }
      const unsigned long long pm = __ballot((uint32_t)lane < ncx && tpv);
      npre = (uint32_t)__popcll(pm);
      hasin = __ballot((uint32_t)lane < ncx && !tpv) != 0ull;
      for (unsigned long long m = pm; m; m &= m - 1ull) {
        const unsigned long long uk = rl32(tu, __builtin_ctzll(m));
        umax = uk > umax ? uk : umax;
      }
    }
    // (CX) a rest's effective quantity: its full quantity less what a cancel removed (ru: its offset in the
    // group's rests at the level, RU the running offset)
    auto reff = [&](bool rs, long long rqf, unsigned long long& RU) -> long long {
      if constexpr (!CX) {
        return rqf;
      } else {
        if (!hasin) return rqf;
        const long long incu = wave_incl_scan(rqf);
        const unsigned long long ru = RU + (unsigned long long)(incu - rqf);
        RU += (unsigned long long)rli64(incu, 63);
        uint32_t dec = 0;
        for (uint32_t k = 0; k < ncx; ++k) {
          const uint32_t uk = rl32(tu, (int)k), rk = rl32(tr, (int)k), pk = rl32(tpv, (int)k);
          if (!pk && rs && ru == (unsigned long long)uk) dec = rk;
        }
        return rqf - (long long)dec;
      }
    };
    auto is_rest = [&](bool v, const AggGEv& E) -> bool {
      if constexpr (CX)
        return v && (E.w & (AGG_TAKE | GR_CXF)) == 0u;
      else
        return v && (E.w & AGG_TAKE) == 0u;
    };
    // 1. C: the takes' total
    unsigned long long C = 0;
    for (uint32_t b = 0; b < cnt; b += 64) {
      uint32_t er;
      const AggGEv E = ent(b, er);
      const bool v = b + (uint32_t)lane < cnt;
      const bool tk = v && (E.w & AGG_TAKE) != 0u;
      if (v && !tk) nf[er] = 0u;
      C += (unsigned long long)rli64(wave_incl_scan(tk ? (long long)E.qty : 0ll), 63);
    }
    // 2. the initial FIFO, read once
    unsigned long long W = 0;
    uint32_t nmk = 0, nfreed = 0, nfull = 0, newhead = NIL, ch = head0, pch = NIL;
    int pq = 0;
    unsigned long long pen = 0;
    bool exhausted = false;
    uint32_t ntail = NIL, nte = 0;  // (CX slow path) the FIFO's tail and its fill after the group
    const bool slow = CX && npre != 0u;
    // (CX) the slow path — cancels of orders from before the group at this level: one FIFO chunk as the
    // maker space sees it (per slot: its effective quantity after a cancel, where it starts and ends, what
    // is left of it after the group)
    struct SlowChunk {
      uint32_t uq, qe, nq, nx;
      unsigned long long cs, ce, sq, iu, ic;
    };
    auto slow_chunk = [&](uint32_t c, unsigned long long Wu, unsigned long long Wc) -> SlowChunk {
      SlowChunk o;
      const int q = act ? bk.chunks[c].qty[lane] : 0;
      o.sq = act ? bk.chunks[c].seq[lane] : 0ull;
      o.nx = auniu(bk.chunks[c].hdr.next);
      o.uq = (uint32_t)max(q, 0);
      const long long iu = wave_incl_scan((long long)o.uq);
      const unsigned long long us = Wu + (unsigned long long)(iu - (long long)o.uq);
      uint32_t dec = 0;
      for (uint32_t k = 0; k < ncx; ++k) {
        const uint32_t uk = rl32(tu, (int)k), rk = rl32(tr, (int)k), pk = rl32(tpv, (int)k);
        if (pk && o.uq && us == (unsigned long long)uk) dec = rk;
      }
      o.qe = o.uq - dec;
      const long long ic = wave_incl_scan((long long)o.qe);
      o.cs = Wc + (unsigned long long)(ic - (long long)o.qe);
      o.ce = Wc + (unsigned long long)ic;
      o.nq = !o.uq ? 0u : dec ? 0u : o.ce <= C ? 0u : o.cs >= C ? o.uq : (uint32_t)(o.ce - C);
      o.iu = (unsigned long long)rli64(iu, 63);
      o.ic = (unsigned long long)rli64(ic, 63);
      return o;
    };
    if (slow) {
      // pass 1 (counts): up to the first chunk the group leaves untouched (the takes covered and every
      // cancelled order passed), or the FIFO's end
      unsigned long long Wu = 0;
      uint32_t lastkept = NIL;
      bool reached_end = false;
      for (uint32_t guard = 0;; ++guard) {
        if (ch == NIL) {
          reached_end = true;
          break;
        }
        if (W >= C && Wu > umax) break;
        if (guard > bk.nchunks) {  // (a cycle in the chain: corrupt)
          a_set_err(bk, ERR_INCONSISTENT);
          reached_end = true;
          ch = NIL;
          break;
        }
        if (ch >= bk.nchunks) {
          a_set_err(bk, ERR_INCONSISTENT);
          reached_end = true;
          ch = NIL;
          break;
        }
        const SlowChunk o = slow_chunk(ch, Wu, W);
        nmk += (uint32_t)__popcll(__ballot(o.qe > 0u && o.cs < C));
        nfull += (uint32_t)__popcll(__ballot(o.uq > 0u && o.nq == 0u));  // initial orders leaving the book
        if (__ballot(o.nq > 0u) == 0ull) {
          ++nfreed;
        } else {
          if (newhead == NIL) newhead = ch;
          lastkept = ch;
        }
        Wu += o.iu;
        W += o.ic;
        ch = o.nx;
      }
      if (newhead == NIL) newhead = reached_end ? NIL : ch;
      exhausted = reached_end && W <= C;
      ntail = reached_end ? lastkept : auniu(sh.ltail[lvl]);
      nte = !reached_end ? auniu(te_raw) : lastkept == NIL ? 0u : lastkept == auniu(sh.ltail[lvl]) ? auniu(te_raw) : (uint32_t)ME_C;
    } else {
      for (;;) {
        if (ch == NIL) {
          exhausted = true;
          break;
        }
        if (W >= C) {
          newhead = ch;
          break;
        }
        if (ch >= bk.nchunks) {
          a_set_err(bk, ERR_INCONSISTENT);
          exhausted = true;
          break;
        }
        const int q = act ? bk.chunks[ch].qty[lane] : 0;
        const unsigned long long sq = act ? bk.chunks[ch].seq[lane] : 0ull;
        const uint32_t nx = auniu(bk.chunks[ch].hdr.next);
        const long long inc = wave_incl_scan((long long)q);
        const unsigned long long ex = (unsigned long long)(inc - q), en = W + (unsigned long long)inc;
        const unsigned long long live = (unsigned long long)rli64(inc, 63);
        const bool cons = q > 0 && W + ex < C;
        const unsigned long long cm = __ballot(cons);
        const uint32_t r = nmk + (uint32_t)__popcll(cm & lanemask_lt());
        if (cons && r < GR_STAGE) {
          mkl[r].seq = sq;
          mkl[r].end = en;
        }
        nmk += (uint32_t)__popcll(cm);
        nfull += (uint32_t)__popcll(__ballot(q > 0 && en <= C));
        if (W + live <= C) {  // emptied
          if (lane == 0 && nfreed < GR_STAGE) frl[nfreed] = ch;
          ++nfreed;
          W += live;
          ch = nx;
          continue;
        }
        pch = ch;  // C ends inside this chunk
        pq = q;
        pen = en;
        newhead = ch;
        break;
      }
      if (newhead != NIL) {
        ntail = auniu(sh.ltail[lvl]);
        nte = auniu(te_raw);
      }
    }
    const unsigned long long T0 = exhausted ? W : ~0ull;
    const unsigned long long Cr = exhausted && C > W ? C - W : 0ull;  // taken from this group's rests
    // 3. the rests: those C reaches are makers too (after the FIFO's), the others survive
    uint32_t nrc = 0, ks = 0;
    {
      unsigned long long RR = 0, RU = 0;
      for (uint32_t b = 0; b < cnt; b += 64) {
        uint32_t er;
        const AggGEv E = ent(b, er);
        const bool v = b + (uint32_t)lane < cnt;
        const bool rs = is_rest(v, E);
        const long long rq = reff(rs, rs ? (long long)E.qty : 0ll, RU);
        const long long inc = wave_incl_scan(rq);
        const unsigned long long st0 = RR + (unsigned long long)(inc - rq), en = RR + (unsigned long long)inc;
        const bool cons = rs && rq > 0 && st0 < Cr;
        const unsigned long long cm = __ballot(cons);
        const uint32_t r = nmk + nrc + (uint32_t)__popcll(cm & lanemask_lt());
        if (cons && r < GR_STAGE) {
          mkl[r].seq = gmin + rsq[srec(E.w)];
          mkl[r].end = T0 + en;
        }
        nrc += (uint32_t)__popcll(cm);
        ks += (uint32_t)__popcll(__ballot(rs && rq > 0 && en > Cr));
        RR += (unsigned long long)rli64(inc, 63);
      }
    }
    const uint32_t te0 = newhead != NIL ? nte : 0u;  // the FIFO's tail fill, if anything of it survives
    const uint32_t tailfree = newhead != NIL ? (uint32_t)ME_C - te0 : 0u;
    const uint32_t need = ks > tailfree ? (ks - tailfree + ME_C - 1) / ME_C : 0u;
    const uint32_t own = min(need, nfreed), deficit = need - own;
    const uint32_t nmkt = nmk + nrc;
    uint32_t mk_base = 0, fr_base = 0, d_off = 0;
    if (lane == 0) {
      mk_base = sl.mk_base + atomicAdd(&sh.cur_mk, nmkt);
      fr_base = sl.fr_base + atomicAdd(&sh.cur_fr, nfreed);
      if (deficit) d_off = atomicAdd(&sh.deficit, deficit);
      const int dr = (int)ks - (int)nfull;
      if (dr) atomicAdd(&sh.dresting, dr);
    }
    mk_base = rl32(mk_base, 0);
    fr_base = rl32(fr_base, 0);
    d_off = rl32(d_off, 0);
    if (mk_base + nmkt > ag.mk_cap || fr_base + nfreed > ag.fr_cap) {
      a_set_err(bk, ERR_SCRATCH_OOM);  // sized so this cannot happen; leaves the level alone
      for (uint32_t b = 0; b < cnt; b += 64) {
        uint32_t er;
        (void)ent(b, er);
        if (b + (uint32_t)lane < cnt) nf[er] = 0u;
      }
      if (lane == 0) {
        GrLevel o{};
        o.T0 = ~0ull;
        o.newhead = head0;
        sh.lv[lvl] = o;
      }
      wave_mem_order();
      continue;
    }
    const bool staged = !slow && nmkt <= GR_STAGE && nfreed <= GR_STAGE;
    // 4. makers and emptied chunks to HBM: from LDS, or past GR_STAGE by a second read of the FIFO
    wave_mem_order();
    if (staged) {
      if ((uint32_t)lane < nmkt) ag.mk[mk_base + lane] = mkl[lane];
      if ((uint32_t)lane < nfreed) ag.fr[fr_base + lane] = frl[lane];
    } else {
      unsigned long long Wv = 0;
      uint32_t mi = 0, fi = 0;
      ch = head0;
      if (slow) {
        // pass 2 (writes): the same chunks; consumed makers, freed chunks, the slots' new quantities, and the
        // surviving chunks linked to each other (a chunk a cancel left without live orders leaves the FIFO)
        unsigned long long Wu = 0;
        uint32_t pk = NIL;
        for (uint32_t guard = 0;; ++guard) {
          if (ch == NIL || (Wv >= C && Wu > umax) || ch >= bk.nchunks || guard > bk.nchunks) break;
          const SlowChunk o = slow_chunk(ch, Wu, Wv);
          const bool cons = o.qe > 0u && o.cs < C;
          const unsigned long long cm = __ballot(cons);
          if (cons) {
            AggMk m;
            m.seq = o.sq;
            m.end = o.ce;
            ag.mk[mk_base + mi + (uint32_t)__popcll(cm & lanemask_lt())] = m;
          }
          mi += (uint32_t)__popcll(cm);
          if (act && o.nq != o.uq) bk.chunks[ch].qty[lane] = (int)o.nq;
          if (__ballot(o.nq > 0u) == 0ull) {
            if (lane == 0) ag.fr[fr_base + fi] = ch;
            ++fi;
          } else {
            if (lane == 0) {
              bk.chunks[ch].hdr.prev = pk;
              if (pk != NIL) bk.chunks[pk].hdr.next = ch;
            }
            pk = ch;
          }
          Wu += o.iu;
          Wv += o.ic;
          ch = o.nx;
        }
        if (lane == 0) {
          const uint32_t stop = ch < bk.nchunks ? ch : NIL;  // the first chunk the group left alone
          if (pk != NIL) bk.chunks[pk].hdr.next = stop;
          if (stop != NIL) bk.chunks[stop].hdr.prev = pk;
        }
      } else {
        while (Wv < C && ch < bk.nchunks) {
          const int q = act ? bk.chunks[ch].qty[lane] : 0;
          const unsigned long long sq = act ? bk.chunks[ch].seq[lane] : 0ull;
          const uint32_t nx = auniu(bk.chunks[ch].hdr.next);
          const long long inc = wave_incl_scan((long long)q);
          const unsigned long long ex = (unsigned long long)(inc - q), en = Wv + (unsigned long long)inc;
          const unsigned long long live = (unsigned long long)rli64(inc, 63);
          const bool cons = q > 0 && Wv + ex < C;
          const unsigned long long cm = __ballot(cons);
          if (cons) {
            AggMk m;
            m.seq = sq;
            m.end = en;
            ag.mk[mk_base + mi + (uint32_t)__popcll(cm & lanemask_lt())] = m;
          }
          mi += (uint32_t)__popcll(cm);
          if (Wv + live > C) break;
          if (lane == 0) ag.fr[fr_base + fi] = ch;
          ++fi;
          Wv += live;
          ch = nx;
        }
      }
      if (Cr) {
        unsigned long long RR = 0, RU = 0;
        for (uint32_t b = 0; b < cnt; b += 64) {
          uint32_t er;
          const AggGEv E = ent(b, er);
          const bool v = b + (uint32_t)lane < cnt;
          const bool rs = is_rest(v, E);
          const long long rq = reff(rs, rs ? (long long)E.qty : 0ll, RU);
          const long long inc = wave_incl_scan(rq);
          const unsigned long long st0 = RR + (unsigned long long)(inc - rq), en = RR + (unsigned long long)inc;
          const bool cons = rs && rq > 0 && st0 < Cr;
          const unsigned long long cm = __ballot(cons);
          if (cons) {
            AggMk m;
            m.seq = gmin + rsq[srec(E.w)];
            m.end = T0 + en;
            ag.mk[mk_base + mi + (uint32_t)__popcll(cm & lanemask_lt())] = m;
          }
          mi += (uint32_t)__popcll(cm);
          RR += (unsigned long long)rli64(inc, 63);
        }
      }
    }
    // 5. the FIFO's new state: emptied chunks hold qty 0, the chunk C ends in keeps what is left (the slow
    //    path wrote its chunks in pass 2)
    wave_mem_order();
    if (!slow) {
      for (uint32_t f0 = 0; f0 < nfreed; f0 += 4) {
        const uint32_t f = f0 + (uint32_t)lane / ME_C;
        if (f < nfreed) {
          const uint32_t c = staged ? frl[f] : ag.fr[fr_base + f];
          if (c < bk.nchunks) bk.chunks[c].qty[lane % ME_C] = 0;
        }
      }
      if (pch != NIL && act && pq > 0 && pen - (unsigned long long)pq < C)
        bk.chunks[pch].qty[lane] = pen <= C ? 0 : (int)(pen - C);
    }
    // 6. each take's fill count: the makers overlapping its interval of the level's maker space
    wave_mem_order();
    {
      unsigned long long A0 = 0;
      for (uint32_t b = 0; b < cnt; b += 64) {
        uint32_t er;
        const AggGEv E = ent(b, er);
        const bool v = b + (uint32_t)lane < cnt;
        const bool tk = v && (E.w & AGG_TAKE) != 0u;
        const long long tq = tk ? (long long)E.qty : 0ll;
        const long long inc = wave_incl_scan(tq);
        if (tk) {
          const unsigned long long a = A0 + (unsigned long long)(inc - tq), z = a + (unsigned long long)E.qty;
          const uint32_t first = staged ? a_search_lds(mkl, nmkt, a, true) : a_search(ag.mk, mk_base, nmkt, a, true);
          const uint32_t last = staged ? a_search_lds(mkl, nmkt, z, false) : a_search(ag.mk, mk_base, nmkt, z, false);
          nf[er] = last - first + 1u;
        }
        A0 += (unsigned long long)rli64(inc, 63);
      }
    }
    if (lane == 0) {
      GrLevel o;
      o.C = C;
      o.T0 = T0;
      o.newhead = newhead;
      o.mk_base = mk_base;
      o.nmk = nmkt;
      o.fr_base = fr_base;
      o.nfreed = nfreed;
      o.need = need;
      o.d_off = d_off;
      o.ks = ks;
      sh.lv[lvl] = o;
      // (CX) the FIFO's tail after the group for phase D (a cancel may have taken the old tail chunk out)
      if constexpr (CX) {
        sh.ltail[lvl] = newhead != NIL ? ntail : NIL;
        sh.ltend[lvl] = (uint8_t)te0;
      }
    }
    wave_mem_order();  // the next level reuses the staging
  }
  __syncthreads();
  GR_STAMP(bk, s, 4);
  // ---- C: fill offsets in log order (exclusive scan of nf in place, each wave over its log range)
  {
    uint32_t sum = 0;
    for (uint32_t b = r0; b < r1; b += 64) {
      const uint32_t e = b + (uint32_t)lane;
      sum += e < r1 ? nf[e] : 0u;
    }
    sum = (uint32_t)rli64(wave_incl_scan((long long)sum), 63);
    if (lane == 0) sh.wsum[wv] = sum;
  }
  __syncthreads();
  uint32_t ftot = 0, base = 0;
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const uint32_t w = sh.wsum[k];
    base += k < wv ? w : 0u;
    ftot += w;
  }
  for (uint32_t b = r0; b < r1; b += 64) {
    const uint32_t e = b + (uint32_t)lane;
    const uint32_t c = e < r1 ? nf[e] : 0u;
    const uint32_t inc = (uint32_t)wave_incl_scan((long long)c);
    if (e < r1) nf[e] = base + inc - c;
    base += rl32(inc, 63);
  }
  __syncthreads();
  auto EX = [&](uint32_t e) -> uint32_t { return e < n ? nf[e] : ftot; };
  if ((uint32_t)tid < ng) {  // each batch's fills: the symbol's slab of that batch if they fit, else overflow
    const uint32_t g = (uint32_t)tid;
    const uint32_t x0 = EX(sh.gev[g]), x1 = EX(sh.gev[g + 1]);
    const uint32_t f = x1 - x0;
    unsigned long long b0 = (unsigned long long)s * ga.slab;
    if (f > ga.slab) {
      b0 = ga.ovf_base + atomicAdd(ga.scratch_top[g], (unsigned long long)f);
      if (b0 + f > ga.scratch_cap) {
        atomicOr(bk.err, ERR_SCRATCH_OOM);
        b0 = 0;
      }
    }
    sh.gex[g] = x0;
    sh.gbase[g] = (uint32_t)b0;
  }
  __syncthreads();
  // the first take event of each record (the records' events are consecutive in the log): its fill count
  // and scratch start; each wave over its log range, 64 events at a time
  {
    uint32_t prevj = r0 > 0 && r0 < r1 ? auniu(ev[r0 - 1].w >> AGG_GREC_SHIFT) : NIL;
    for (uint32_t b = r0; b < r1; b += 64) {
      const uint32_t e = b + (uint32_t)lane;
      const bool v = e < r1;
      const uint32_t j = v ? ev[e].w >> AGG_GREC_SHIFT : NIL;  // record | take (the level shifted out)
      uint32_t pj = (uint32_t)__shfl_up((int)j, 1, 64);
      pj = lane == 0 ? prevj : pj;
      uint32_t nj = (uint32_t)__shfl_down((int)j, 1, 64);
      nj = lane == 63 ? NIL : nj;
      const unsigned long long same = __ballot(v && nj == j);  // bit k: event k + 1 continues k's run
      prevj = rl32(j, 63);
      if (v && (j & (AGG_TAKE >> AGG_GREC_SHIFT)) && pj != j) {
        // the record's take events: the run of j from here (lane 63's bit is clear)
        uint32_t nte = (uint32_t)__builtin_ctzll(~(same >> lane)) + 1u;
        if (lane + (int)nte == 64)
          while (e + nte < n && (ev[e + nte].w >> AGG_GREC_SHIFT) == j) ++nte;  // the run goes past this block
        const uint32_t gp = rjs[j & ~(AGG_TAKE >> AGG_GREC_SHIFT)];
        const uint32_t g = gp >> AGG_GSHIFT, oi = gp & AGG_IMASK;
        const uint32_t x0 = EX(e), nfill = EX(e + nte) - x0;
        me_order_result* res = ga.res[g];
        res[oi].fill_count = nfill;
        res[oi].tape_offset = sh.gbase[g] + (x0 - sh.gex[g]);
#ifndef ME_AB_NO_TILESUM  // (measurement-only switch: the tape's tile sums left out, tapes wrong)
        if (nfill) atomicAdd(&ga.tile_sum[g][oi / TILE_TAPE], nfill);
#endif
      }
    }
  }
  if (tid == 0 && sl.hidx != NIL) {  // the continuation goes on behind the walk's fills of its batch
    const uint32_t g = sl.pos;
    const uint32_t f = EX(sh.gev[g + 1]) - sh.gex[g];
    const uint32_t b0 = sh.gbase[g];
    bk.hand[sl.hidx].wptr = b0 + f;
    bk.hand[sl.hidx].wend = f <= ga.slab ? s * ga.slab + ga.slab : b0 + f;
  }
  GR_STAMP(bk, s, 5);
  // ---- D: chunk allocation (wave 0); the symbol's state
  if (wv == 0) {
    uint32_t D = sh.deficit, fh = sl.free_head;
    uint32_t Stot = 0;
    for (uint32_t b = 0; b < nlv; b += 64) {
      uint32_t sp = 0;
      if (b + lane < nlv) {
        const GrLevel& g = sh.lv[sh.lvlist[b + lane]];
        sp = g.nfreed - min(g.need, g.nfreed);
      }
      Stot += (uint32_t)rli64(wave_incl_scan((long long)sp), 63);
    }
    uint32_t ab = 0;
    bool ok = true;
    if (D || Stot) {
      ab = sl.fr_base + sh.cur_fr;  // (no other wave reserves any more)
      if ((unsigned long long)ab + D + Stot > ag.fr_cap) {
        a_set_err(bk, ERR_SCRATCH_OOM);
        ok = false;
      }
    }
    if ((D || Stot) && ok) {
      uint32_t run = 0;  // the surpluses (level order) into fr[ab + D, ab + D + Stot)
      for (uint32_t b = 0; b < nlv; b += 64) {
        uint32_t sp = 0, srcf = 0;
        if (b + lane < nlv) {
          const GrLevel& g = sh.lv[sh.lvlist[b + lane]];
          const uint32_t own = min(g.need, g.nfreed);
          sp = g.nfreed - own;
          srcf = g.fr_base + own;
        }
        const long long inc = wave_incl_scan((long long)sp);
        const uint32_t ex = run + (uint32_t)(inc - sp);
        for (uint32_t k = 0; k < sp; ++k) ag.fr[ab + D + ex + k] = ag.fr[srcf + k];
        run += (uint32_t)rli64(inc, 63);
      }
      a_drain();
      const uint32_t k1 = min(D, Stot);
      for (uint32_t t = lane; t < k1; t += 64) ag.fr[ab + t] = ag.fr[ab + D + t];
      if (D > k1) {  // the book grows: the free list, then fresh chunks
        uint32_t t = k1;
        if (lane == 0) {
          while (t < D && fh != NIL && fh < bk.nchunks) {
            ag.fr[ab + t] = fh;
            fh = bk.chunks[fh].hdr.next;
            ++t;
          }
        }
        t = rl32(t, 0);
        fh = rl32(fh, 0);
        if (t < D) {
          const uint32_t left = D - t;
          uint32_t got = 0;
          if (lane == 0) got = atomicAdd(bk.chunk_top, left);
          got = rl32(got, 0);
          const CPool cp = cp_read(bk.cpool);
          if ((unsigned long long)got + left > cp_vcap(cp, bk.nchunks)) {
            a_set_err(bk, ERR_CHUNK_OOM);
            for (uint32_t u = lane; u < left; u += 64) ag.fr[ab + t + u] = 0u;  // never indexed past the pool
          } else {
            for (uint32_t u = lane; u < left; u += 64) {
              const uint32_t id = cp_id(bk.recl, cp, got + u);
              ag.fr[ab + t + u] = id;
              bk.chunks[id].owner = s;  // the symbol's until a reclamation finds the chunk free
            }
          }
        }
      } else if (Stot > D) {  // surpluses left over: linked in front of the free list
        for (uint32_t u = D + lane; u < Stot; u += 64) {
          const uint32_t c = ag.fr[ab + D + u];
          bk.chunks[c].hdr.next = u + 1 < Stot ? ag.fr[ab + D + u + 1] : fh;
        }
        fh = auniu(ag.fr[ab + D + D]);
      }
    }
    if (lane == 0) {
      sh.alloc_base = ab;
      SymState o = bk.sym[s];
      o.best_bid = sl.bb;
      o.best_ask = sl.ba;
      o.free_head = fh;
      o.nfree = 0;  // the walk linked the parked chunks into the free list
      const int dr = sh.dresting;
      o.resting = (uint32_t)((int)sl.resting0 + dr);
      bk.sym[s] = o;
      if (dr) atomicAdd(bk.stats + ST_RESTING, (unsigned long long)(long long)dr);
    }
  }
  __syncthreads();
  GR_STAMP(bk, s, 6);
  // ---- D: per level, one pass over its events: the fills of its takes (makers overlapping each take's
  //      interval, at the record's scratch position) and its surviving rests into the tail chunk and new
  //      chunks; the new chunks' headers, the level's head / tail / tail fill
  const uint32_t alloc_base = sh.alloc_base;
  for (uint32_t it = gr_take(&sh.next2); it < nlv; it = gr_take(&sh.next2)) {
    const uint32_t lvl = __builtin_amdgcn_readfirstlane(sh.lvlist[it]);
    const uint32_t start = __builtin_amdgcn_readfirstlane(sh.lstart[lvl]);
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(sh.lstart[lvl + 1]) - start;
    const GrLevel& gl = sh.lv[lvl];
    const unsigned long long C = rl64(gl.C, 0), T0 = rl64(gl.T0, 0);
    const uint32_t newhead = auniu(gl.newhead), need = auniu(gl.need), ks = auniu(gl.ks);
    const uint32_t nfreed = auniu(gl.nfreed), fr_base = auniu(gl.fr_base), d_off = auniu(gl.d_off);
    const uint32_t nmk = auniu(gl.nmk), mk_base = auniu(gl.mk_base);
    const uint32_t own = min(need, nfreed);
    const size_t li = lo_l + lvl;
    const uint32_t head0 = auniu(sh.lhead[lvl]), tail0 = auniu(sh.ltail[lvl]);
    const uint32_t te0 = newhead != NIL ? auniu((uint32_t)sh.ltend[lvl]) : 0u;
    const uint32_t tailfree = newhead != NIL ? (uint32_t)ME_C - te0 : 0u;
    // (CX) the level's cancels of this group's rests: {offset in the rests, removed} in lanes
    uint32_t ncx = 0, tu = 0, tr = 0;
    if constexpr (CX) {
      GrCxStage& X = cxs[wv];
      for (uint32_t b = 0; b < cnt; b += 64) {
        uint32_t er;
        const AggGEv E = entry(start, cnt, b, er);
        const bool v = b + (uint32_t)lane < cnt;
        const bool cu = v && (E.w & (GR_CXF | GR_CXU | GR_CXP)) == (GR_CXF | GR_CXU);
        const unsigned long long m = __ballot(cu);
        if (!m) continue;
        const uint32_t k = ncx + (uint32_t)__popcll(m & lanemask_lt());
        if (cu && k < 64u) {
          X.cxu[k] = (uint32_t)E.qty;
          X.cxr[k] = (uint32_t)srt[start + b + lane - 1].qty;
        }
        ncx += (uint32_t)__popcll(m);
      }
      ncx = min(ncx, 64u);
      wave_mem_order();
      if ((uint32_t)lane < ncx) {
        tu = X.cxu[lane];
        tr = X.cxr[lane];
      }
    }
    auto newchunk = [&](uint32_t c) -> uint32_t {
      return c < own ? ag.fr[fr_base + c] : ag.fr[alloc_base + d_off + (c - own)];
    };
    const bool exhausted = T0 != ~0ull;
    const unsigned long long Cr = exhausted && C > T0 ? C - T0 : 0ull;
    const bool staged = nmk <= GR_STAGE;
    if (nmk && staged && (uint32_t)lane < nmk) mkl[lane] = ag.mk[mk_base + lane];
    wave_mem_order();
    const long long price = sl.base + (long long)lvl;
    unsigned long long A0 = 0, RR = 0, RU = 0;
    uint32_t g0 = 0;
    for (uint32_t b = 0; b < cnt; b += 64) {
      uint32_t er;
      const AggGEv E = entry(start, cnt, b, er);
      const bool v = b + (uint32_t)lane < cnt;
      const bool tk = v && (E.w & AGG_TAKE) != 0u;
      const bool rs = CX ? v && (E.w & (AGG_TAKE | GR_CXF)) == 0u : v && !tk;
      const long long tq = tk ? (long long)E.qty : 0ll;
      long long rq = rs ? (long long)E.qty : 0ll;
      if (CX && ncx) {  // a rest a cancel shortened keeps its consumed part only
        const long long incu = wave_incl_scan(rq);
        const unsigned long long ru = RU + (unsigned long long)(incu - rq);
        RU += (unsigned long long)rli64(incu, 63);
        uint32_t dec = 0;
        for (uint32_t k = 0; k < ncx; ++k) {
          const uint32_t uk = rl32(tu, (int)k), rk = rl32(tr, (int)k);
          if (rs && ru == (unsigned long long)uk) dec = rk;
        }
        rq -= (long long)dec;
      }
      const long long tinc = wave_incl_scan(tq), rinc = wave_incl_scan(rq);
      const unsigned long long sq = gmin + rsq[(tk || rs) ? srec(E.w) : 0u];
      if (tk && nmk) {  // fills
        const uint32_t x0 = nf[er], nfl = EX(er + 1) - x0;
        if (nfl) {
          const unsigned long long a = A0 + (unsigned long long)(tinc - tq), z = a + (unsigned long long)E.qty;
          const uint32_t first = staged ? a_search_lds(mkl, nmk, a, true) : a_search(ag.mk, mk_base, nmk, a, true);
          const uint32_t g = rjs[srec(E.w)] >> AGG_GSHIFT;
          const uint32_t p = sh.gbase[g] + (x0 - sh.gex[g]);
          me_fill f;
          f.taker_seq = sq;
          f.price_q4 = price;
          f.symbol = sl.gs;
          me_fill* sc = ga.scratch[g];
          unsigned long long lo = a;
          for (uint32_t k = 0; k < nfl; ++k) {
            const AggMk m = staged ? mkl[first + k] : ag.mk[mk_base + first + k];
            const unsigned long long hi = m.end < z ? m.end : z;
            f.maker_seq = m.seq;
            f.qty = (int)(hi - lo);
            sc[p + k] = f;
            lo = hi;
          }
        }
      }
      // surviving rests
      const unsigned long long st0 = RR + (unsigned long long)(rinc - rq), en = RR + (unsigned long long)rinc;
      const bool surv = rs && rq > 0 && en > Cr;
      const unsigned long long sm = __ballot(surv);
      if (surv) {
        const uint32_t gi = g0 + (uint32_t)__popcll(sm & lanemask_lt());
        uint32_t chk, slt;
        if (gi < tailfree) {
          chk = tail0;
          slt = te0 + gi;
        } else {
          const uint32_t gg = gi - tailfree;
          chk = newchunk(gg / ME_C);
          slt = gg % ME_C;
        }
        const int left = (int)(en - (st0 > Cr ? st0 : Cr));
        if (chk < bk.nchunks) {
          bk.chunks[chk].qty[slt] = left;
          bk.chunks[chk].seq[slt] = sq;
          bk.loc[sq & bk.ring_mask] = chk * ME_C + slt;
        }
      }
      g0 += (uint32_t)__popcll(sm);
      A0 += (unsigned long long)rli64(tinc, 63);
      RR += (unsigned long long)rli64(rinc, 63);
    }
    for (uint32_t c = lane; c < need; c += 64) {
      const uint32_t chk = newchunk(c);
      if (chk >= bk.nchunks) continue;
      ChunkHdr h;
      h.next = c + 1 < need ? newchunk(c + 1) : NIL;
      h.prev = c ? newchunk(c - 1) : (newhead != NIL ? tail0 : NIL);
      h.price = price;
      bk.chunks[chk].hdr = h;
    }
    const uint32_t first_new = need ? auniu(newchunk(0)) : NIL;
    const uint32_t last_new = need ? auniu(newchunk(need - 1)) : NIL;
    if (lane == 0) {
      if (newhead != NIL && need && tail0 < bk.nchunks) bk.chunks[tail0].hdr.next = first_new;
      if (newhead != NIL && newhead != head0 && newhead < bk.nchunks) bk.chunks[newhead].hdr.prev = NIL;
      const uint32_t hd = newhead != NIL ? newhead : first_new;
      const uint32_t tl = need ? last_new : (newhead != NIL ? tail0 : NIL);
      const uint32_t te = need ? ((ks - tailfree - 1u) % ME_C) + 1u : (newhead != NIL ? te0 + ks : 0u);
      bk.levels[li].head = hd;
      bk.levels[li].tail = tl;
      bk.tend[li] = (uint8_t)te;
    }
    wave_mem_order();  // the next level reuses the staging
  }
  __syncthreads();
  GR_STAMP(bk, s, 7);
}

template <int NW, bool CX>
__global__ __launch_bounds__(NW * 64, GR_WPE) void k_agg_gres(BookDev bk, AggGArgs ga, AggSrc src, AggDev ag,
                                                       uint32_t ne) {
  __shared__ GrShared<NW> sh;
  __shared__ GrCxStage cxs[CX ? NW : 1];
  extern __shared__ uint32_t gr_dyn[];  // [ne] fill counts / offsets
  for (uint32_t s = blockIdx.x; s < bk.S; s += gridDim.x) {
    const AggSlot sl = ag.slot[s];
    if (!sl.active) continue;  // (uniform over the workgroup)
    if (sl.ev_cnt >= 65536u) {  // 16-bit log indices in the sorted entries: a grouped log is at most 3 x 32 x BK_CAP + L + 64 long
      if (threadIdx.x == 0) atomicOr(bk.err, ERR_INCONSISTENT);
      continue;
    }
    if (sl.ev_cnt <= ne)
      gres_symbol<NW, true, CX>(bk, ga, src, ag, s, sl, sh, gr_dyn, cxs);
    else
      gres_symbol<NW, false, CX>(bk, ga, src, ag, s, sl, sh, ag.evn + sl.ev_base, cxs);
    __syncthreads();
  }
}

}  // namespace

hipError_t launch_agg(hipStream_t hs, const BookDev& bk, const BatchDev& bt, const AggDev& ag0) {
  AggDev ag = ag0;
  ag.nslots = 0;  // k_hot_pick's hot symbols
  AggSrc src{};
  src.perm = bt.perm;
  src.seq[0] = bt.seq;
  const size_t lwb = bk.L <= ag.ladder_max ? ((size_t)bk.L + 64u) * 4u : 0u;
  hipLaunchKernelGGL(k_agg_walk, dim3(64), dim3(64), lwb, hs, bk, bt, ag);
  hipLaunchKernelGGL(k_agg_group, dim3(64), dim3(1024), agg_group_lds(bk.L), hs, bk, ag);
  hipLaunchKernelGGL(k_agg_sorted, dim3(1024), dim3(256), 0, hs, bk, ag);
  hipLaunchKernelGGL(k_agg_levels<true>, dim3(1024), dim3(256), 0, hs, bk, src, ag);
  hipLaunchKernelGGL(k_agg_lvscan, dim3(64), dim3(1024), 0, hs, bk, ag);
  hipLaunchKernelGGL(k_agg_levels<false>, dim3(1024), dim3(256), 0, hs, bk, src, ag);
  hipLaunchKernelGGL(k_agg_alloc, dim3(64), dim3(64), 0, hs, bk, ag);
  hipLaunchKernelGGL(k_agg_place, dim3(1024), dim3(256), 0, hs, bk, src, ag);
  hipLaunchKernelGGL(k_agg_fin, dim3(64), dim3(1024), 0, hs, bk, bt, ag);
  hipLaunchKernelGGL(k_agg_out, dim3(1024), dim3(256), 0, hs, bk, bt, ag);
  return hipGetLastError();
}

}  // namespace me

namespace me {
// A grouped register-window launch through the aggregate path (batches bt[0, ng), all bucketed): the
// walk, the per-level kernels, the fills; the continuation launch follows (me_kernels.hip).
hipError_t launch_agg_group(hipStream_t st, const BookDev& bk, const BatchDev* bt, uint32_t ng, const AggDev& ag0) {
  if (!ng || ng > (uint32_t)ME_GMAX || bk.L > 128u) return hipErrorInvalidValue;
  AggDev ag = ag0;
  ag.nslots = bk.S;
  AggGArgs ga{};
  AggSrc src{};
  for (uint32_t g = 0; g < ng; ++g) {
    if (!bt[g].bcnt) return hipErrorInvalidValue;
    ga.bcnt[g] = bt[g].bcnt;
    ga.b_rec[g] = bt[g].b_rec;
    ga.res[g] = bt[g].res;
    ga.tile_sum[g] = bt[g].tile_sum;
    ga.scratch[g] = bt[g].scratch;
    ga.scratch_top[g] = bt[g].scratch_top;
    src.seq[g] = bt[g].seq;
  }
  ga.ovf_base = bt[0].ovf_base;
  ga.scratch_cap = bt[0].scratch_cap;
  ga.seq0 = bt[0].seq;
  ga.slab = bt[0].slab;
  ga.ng = ng;
  // one workgroup per symbol up to the grid cap, then symbols striding over the grid (blockIdx = symbol mod
  // grid: a symbol's walk and resolve run on the same XCD either way)
  static const uint32_t gcap = [] {
    const char* e = getenv("ME_AGG_GRID");
    return e && atoi(e) > 0 ? (uint32_t)atoi(e) : 65536u;
  }();
  const uint32_t grid = bk.S < gcap ? bk.S : gcap;
  static const bool helper = [] {
    const char* e = getenv("ME_GW_HELPER");
    return !e || atoi(e) != 0;
  }();
  const bool cx = ag.gw_cx != 0u;  // groups with cancels: the walk that covers them, and its resolve
  if (cx)
    hipLaunchKernelGGL(k_agg_gwalk_cx, dim3(grid), dim3(128), 0, st, bk, ga, ag);
  else if (helper)
    hipLaunchKernelGGL(k_agg_gwalk2, dim3(grid), dim3(128), 0, st, bk, ga, ag);
  else
    hipLaunchKernelGGL(k_agg_gwalk, dim3(grid), dim3(64), 0, st, bk, ga, ag);
  // the per-event LDS array (fill counts, 4 B per event) sized for 1.75 events per record of the group's
  // mean symbol plus slack; a longer log keeps it in HBM. Capped so the workgroup's LDS stays within 64 KB.
  uint64_t recs = 0;
  for (uint32_t g = 0; g < ng; ++g) recs += bt[g].n;
  uint64_t ne = (recs * 7u / 4u) / (bk.S ? bk.S : 1u) + 256u;  // (config 2: 1.4 events per record)
  ne = (ne + 63u) & ~63ull;
  // resolve workgroups of 8 waves, or of 4 for groups with few records per symbol (config 3's ~210: twice
  // the workgroups in flight); ME_GRES_WAVES=4/8 forces either
  static const int gw_env = [] {
    const char* e = getenv("ME_GRES_WAVES");
    return e ? atoi(e) : 0;
  }();
  const uint64_t per_sym = recs / (bk.S ? bk.S : 1u);
  int nw = gw_env == 2 || gw_env == 4 || gw_env == 8 ? gw_env : per_sym < GR_FOUR_BELOW ? 4 : 8;
  if (cx && nw == 2) nw = 4;  // (the 2-wave form is a measurement switch; the resolve with cancels has 4 or 8)
  const size_t shb = nw == 2 ? sizeof(GrShared<2>) : nw == 4 ? sizeof(GrShared<4>) : sizeof(GrShared<GR_WAVES>);
  const uint64_t ne_cap = ((64u << 10) - shb) / 4u & ~63ull;
  if (ne > ne_cap) ne = ne_cap;
  if (nw == 2) {
    hipLaunchKernelGGL((k_agg_gres<2, false>), dim3(grid), dim3(128), (size_t)ne * 4u, st, bk, ga, src, ag, (uint32_t)ne);
  } else if (nw == 4) {
    if (cx)
      hipLaunchKernelGGL((k_agg_gres<4, true>), dim3(grid), dim3(256), (size_t)ne * 4u, st, bk, ga, src, ag, (uint32_t)ne);
    else
      hipLaunchKernelGGL((k_agg_gres<4, false>), dim3(grid), dim3(256), (size_t)ne * 4u, st, bk, ga, src, ag, (uint32_t)ne);
  } else {
    if (cx)
      hipLaunchKernelGGL((k_agg_gres<GR_WAVES, true>), dim3(grid), dim3(GR_THREADS), (size_t)ne * 4u, st, bk, ga, src,
                         ag, (uint32_t)ne);
    else
      hipLaunchKernelGGL((k_agg_gres<GR_WAVES, false>), dim3(grid), dim3(GR_THREADS), (size_t)ne * 4u, st, bk, ga, src,
                         ag, (uint32_t)ne);
  }
  return hipGetLastError();
}
}  // namespace me

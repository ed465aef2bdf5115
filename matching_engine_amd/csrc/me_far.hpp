// me_far.hpp — price levels outside a symbol's window, shared by both matching kernels.
//
// The reference accepts any LIMIT with a positive raw price (src/server/matching_engine_service.cpp:
// 78-83) at any int64 Q4 (include/domain/price.hpp:15-29), so a fixed-depth window cannot be the whole
// book. Levels outside it live in two sorted arrays per symbol (BookDev::far):
//   side 0: bids below the window, ascending price (best = last entry),
//   side 1: asks above the window, descending price (best = last entry),
// with the same FIFO chunks as window levels. Invariant I: no bid rests above the window and no ask
// below it, so window levels are always better than far levels of the same side, a taker walks
// the window first and then pops far levels from the best end, and a rest that would break I
// re-centres the window first (the kernels' recentre routines). Far levels are the rare path: no
// caching, plain HBM round trips, wave-uniform control flow.
//
// The arrays are unbounded (round 5; before, `far_levels` per side was a hard cap whose overflow failed
// the engine). Each (symbol, side) owns a region of the far arena named by fdir[s][k] = {off, cap}:
// first its inline region of `far_levels` entries; a rest or re-centre that finds the region full moves
// the side to a region twice as large taken from the active half of the arena (far_grow: one atomic
// add on that half's top, a copy, the new fdir entry). Abandoned regions are reclaimed by a copying
// collection in k_seq_sweep (me_kernels.hip) ahead of a launch group, when the active half's top has
// passed far_gc_at: every moved side goes to a region of nextpow2(n) entries in the other half, or
// back inline when it fits, and the halves swap. The sizes make overflow impossible under admission
// control (me_config.max_resting, M): a far level holds >= 1 resting order, so the sides' peak counts
// during one group sum to <= M and the regions one group allocates to <= 2 + 4 + ... <= 4 x peak,
// i.e. <= 4M; a collection leaves <= 2M (nextpow2(n) < 2n); so a half of 6M entries, collected above
// 2M, never runs out (ERR_FAR_OOM marks that bound broken, an internal error).
//
// A kernel context C provides: fchunks() / fnchunks(), fsym() / fgsym() (local symbol, id written
// into fills), fcount(k) / fset_count(k, n), the arena: fdirp(k) (its fdir entry), farena(),
// fctl() (BookDev::far_ctl), fstats(), fcap0() (inline entries), finline() (inline region end),
// fhalf() (entries per half), falloc() / ffree(ch) (its chunk pool; a freed chunk reads all-zero
// quantities in HBM), femit(e, mask, fill) (scratch fills, lane order), fresting(delta), ferr(bits),
// floc(seq, slot) (seq-ring write).
#pragma once
#include "me_layout.hpp"
#include "me_wave.hpp"

namespace me {

// The region of side k (wave-uniform). Read with vector loads: far_grow rewrites it during a launch.
template <class C>
__device__ __forceinline__ FarDir far_dir(const C& c, uint32_t k) {
  FarDir* p = c.fdirp(k);
  FarDir d;
  d.off = rl64(__hip_atomic_load(&p->off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), 0);
  d.cap = rl32(__hip_atomic_load(&p->cap, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), 0);
  d.pad = 0;
  return d;
}
template <class C>
__device__ __forceinline__ gptr<FarLevel> far_arr(const C& c, uint32_t k) {
  return (gptr<FarLevel>)(c.farena() + far_dir(c, k).off);
}

// Side k holds n levels and its region is full: move it to a region twice as large (at least twice the
// inline size) in the active half. Returns false (ERR_FAR_OOM, sticky) only if the bound above broke.
template <class C>
__device__ bool far_grow(C& c, uint32_t k, uint32_t n) {
  const int lane = lane_id();
  const FarDir d = far_dir(c, k);
  const unsigned long long c0 = c.fcap0();
  unsigned long long ncap = 2ull * d.cap;
  if (ncap < 2ull * c0) ncap = 2ull * c0;
  unsigned long long* ctl = c.fctl();
  unsigned long long o = ~0ull;
  if (lane == 0 && ncap <= 0x80000000ull) {
    const unsigned long long h = __hip_atomic_load(ctl + FC_HALF, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1ull;
    const unsigned long long t = atomicAdd(ctl + h, ncap);
    if (t + ncap <= c.fhalf()) o = c.finline() + h * c.fhalf() + t;
  }
  o = rl64(o, 0);
  if (o == ~0ull) {
    c.ferr(ERR_FAR_OOM);
    return false;
  }
  const gptr<FarLevel> src = (gptr<FarLevel>)(c.farena() + d.off);
  const gptr<FarLevel> dst = (gptr<FarLevel>)(c.farena() + o);
  for (uint32_t i = (uint32_t)lane; i < n; i += 64) dst[i] = src[i];
  wave_mem_order();
  if (lane == 0) {
    FarDir* p = c.fdirp(k);
    __hip_atomic_store(&p->off, o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&p->cap, (uint32_t)ncap, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    atomicAdd(c.fstats() + ST_FAR_GROW, 1ull);
  }
  wave_mem_order();
  return true;
}

// Wave-uniform read of entry i (every lane loads the same 32 B).
__device__ __forceinline__ FarLevel far_get(gptr<FarLevel> a, uint32_t i) {
  FarLevel e = a[i];
  e.price = rli64(e.price, 0);
  e.total = rli64(e.total, 0);
  e.head = rl32(e.head, 0);
  e.tail = rl32(e.tail, 0);
  e.tend = rl32(e.tend, 0);
  e.pad = 0;
  return e;
}
__device__ __forceinline__ void far_put(gptr<FarLevel> a, uint32_t i, const FarLevel& e) {
  if (lane_id() == 0) a[i] = e;
}

// Entries of a[0, n) ordered before price p on side k (0: price < p, 1: price > p): the insert
// position of p, and the index of p's level when it exists. 64-ary search: each step samples 64
// positions in one load and narrows the range 64x.
__device__ __forceinline__ uint32_t far_rank(gptr<FarLevel> a, uint32_t n, long long p, uint32_t k) {
  const int lane = lane_id();
  uint32_t lo = 0, hi = n;
  while (hi - lo > 64) {
    const uint32_t step = (hi - lo + 63) / 64;
    const uint32_t pos = lo + (uint32_t)lane * step;
    const long long v = a[pos < hi ? pos : lo].price;
    const bool before = pos < hi && (k ? v > p : v < p);
    const uint32_t c = (uint32_t)__popcll(__ballot(before));
    if (c == 0) return lo;
    const uint32_t nlo = lo + (c - 1) * step + 1;
    uint32_t nhi = lo + c * step;
    lo = nlo;
    hi = nhi < hi ? nhi : hi;
  }
  const uint32_t pos = lo + (uint32_t)lane;
  const long long v = a[pos < hi ? pos : (hi ? hi - 1 : 0)].price;
  const bool before = pos < hi && (k ? v > p : v < p);
  return lo + (uint32_t)__popcll(__ballot(before));
}

// a[i + 1] = a[i] for i in [pos, n): blocks of 64 from the top (every block reads before it writes,
// and no later block reads what an earlier one wrote).
__device__ __forceinline__ void far_shift_up(gptr<FarLevel> a, uint32_t pos, uint32_t n) {
  const int lane = lane_id();
  for (uint32_t top = n; top > pos;) {
    const uint32_t lo = top - pos > 64 ? top - 64 : pos;
    const uint32_t i = top - 1 - (uint32_t)lane;
    const bool v = (int)i >= (int)lo && i < top;
    FarLevel e{};
    if (v) e = a[i];
    if (v) a[i + 1] = e;
    top = lo;
  }
}
// a[i] = a[i + 1] for i in [pos, n - 1): blocks of 64 from the bottom.
__device__ __forceinline__ void far_shift_down(gptr<FarLevel> a, uint32_t pos, uint32_t n) {
  const int lane = lane_id();
  for (uint32_t b = pos; b + 1 < n; b += 64) {
    const uint32_t i = b + (uint32_t)lane;
    const bool v = i + 1 < n;
    FarLevel e{};
    if (v) e = a[i + 1];
    if (v) a[i] = e;
  }
}

// Append level e at the best end of side k (re-centring: levels leaving the window).
template <class C>
__device__ __forceinline__ bool far_push(C& c, uint32_t k, const FarLevel& e) {
  const uint32_t n = c.fcount(k);
  if (n >= far_dir(c, k).cap && !far_grow(c, k, n)) return false;
  far_put(far_arr(c, k), n, e);
  c.fset_count(k, n + 1);
  return true;
}

// A taker crossing beyond its window: consume from the far side it trades against (BUY: asks above,
// side 1; SELL: bids below, side 0), best level first, oldest order first, up to rem and (unless
// MARKET) while the level's price is within the limit. Fills go to the context's scratch run in
// order. Returns the quantity taken.
template <class C>
__device__ uint32_t far_take(C& c, bool buy, bool market, long long limit, uint32_t rem, unsigned long long taker) {
  const int lane = lane_id();
  const int sl = lane & (ME_C - 1);
  const uint32_t k = buy ? 1u : 0u;
  const gptr<FarLevel> a = far_arr(c, k);
  const gptr<Chunk> chunks = c.fchunks();
  const uint32_t NC = c.fnchunks();
  uint32_t n = c.fcount(k);
  const uint32_t want = rem;
  wave_mem_order();
  while (rem != 0u && n != 0u) {
    FarLevel e = far_get(a, n - 1u);
    if (!market && (buy ? e.price > limit : e.price < limit)) break;
    uint32_t ch = e.head;
    long long taken = 0;
    bool emptied = false;
    for (;;) {
      if (ch >= NC) {
        c.ferr(ERR_INCONSISTENT);
        c.fset_count(k, n);
        return want - rem;
      }
      const int q = chunks[ch].qty[sl];
      const unsigned long long ms = chunks[ch].seq[sl];
      const uint32_t nx = rl32(chunks[ch].hdr.next, 0);
      const uint32_t uq = lane < ME_C && q > 0 ? (uint32_t)q : 0u;
      const uint32_t inc = scan16_sat(uq);
      const uint32_t ex = inc - uq;
      uint32_t f = rem > ex ? rem - ex : 0u;
      f = f < uq ? f : uq;
      const bool fe = f != 0u;
      const unsigned long long fm = __ballot(fe);
      me_fill F;
      F.taker_seq = taker;
      F.maker_seq = ms;
      F.price_q4 = e.price;
      F.qty = (int)f;
      F.symbol = c.fgsym();
      c.femit(fe, fm, F);
      if (fe) chunks[ch].qty[sl] = (int)(uq - f);
      c.fresting(-__popcll(__ballot(fe && f == uq)));
      const uint32_t live = rl32(inc, 15);
      const uint32_t t = rem < live ? rem : live;
      rem -= t;
      taken += t;
      if ((__ballot(uq > f) & 0xFFFFull) != 0ull) break;  // live slots remain: the taker is done
      // every slot of the chunk is now zero in HBM: back to the pool
      const bool last = ch == e.tail;
      c.ffree(ch);
      if (last) {
        emptied = true;
        break;
      }
      ch = nx;
      if (rem == 0u) break;
    }
    e.total -= taken;
    if (emptied) {
      if (e.total != 0) c.ferr(ERR_INCONSISTENT);
      n -= 1u;  // the level is gone (it was the last entry)
      continue;
    }
    if (ch != e.head && lane == 0 && ch < NC) chunks[ch].hdr.prev = NIL;  // new FIFO head
    e.head = ch;
    far_put(a, n - 1u, e);
    break;
  }
  c.fset_count(k, n);
  return want - rem;
}

// Rest (seq, qty) at price p on far side k (0: a bid below the window, 1: an ask above it).
template <class C>
__device__ bool far_rest(C& c, uint32_t k, long long p, unsigned long long seq, uint32_t qty) {
  const FarDir d = far_dir(c, k);
  gptr<FarLevel> a = (gptr<FarLevel>)(c.farena() + d.off);
  const gptr<Chunk> chunks = c.fchunks();
  uint32_t n = c.fcount(k);
  wave_mem_order();
  const uint32_t pos = far_rank(a, n, p, k);
  FarLevel e{};
  bool exists = false;
  if (pos < n) {
    e = far_get(a, pos);
    exists = e.price == p;
  }
  if (!exists) {
    if (n >= d.cap) {  // the region is full: a larger one (same entries, so pos still holds)
      if (!far_grow(c, k, n)) return false;
      a = far_arr(c, k);
    }
    far_shift_up(a, pos, n);
    e.price = p;
    e.total = 0;
    e.head = e.tail = NIL;
    e.tend = 0;
    e.pad = 0;
    c.fset_count(k, n + 1u);
  }
  uint32_t ch, slot;
  if (e.tail != NIL && e.tend < (uint32_t)ME_C) {
    if (e.tail >= c.fnchunks()) {
      c.ferr(ERR_INCONSISTENT);
      return false;
    }
    ch = e.tail;
    slot = e.tend;
    e.tend += 1u;
  } else {
    ch = c.falloc();
    if (ch == NIL) return false;
    if (lane_id() == 0) {
      ChunkHdr h;
      h.next = NIL;
      h.prev = e.tail;
      h.price = p;
      chunks[ch].hdr = h;
      if (e.tail != NIL) chunks[e.tail].hdr.next = ch;
    }
    if (e.tail == NIL) e.head = ch;
    e.tail = ch;
    e.tend = 1u;
    slot = 0;
  }
  if (lane_id() == 0) {
    chunks[ch].qty[slot] = (int)qty;
    chunks[ch].seq[slot] = seq;
  }
  c.floc(seq, ch * ME_C + slot);
  e.total += qty;
  far_put(a, pos, e);
  c.fresting(1);
  return true;
}

// Cancel the live order in slot `slot` of chunk ch (quantity q) of the far level at price p, side k.
// qv: the chunk's live quantities (lanes 0..15, 0 elsewhere); nxt / prv: its FIFO links. The caller
// verified owner, seq and liveness. A chunk left without live orders is unlinked and freed; a level
// left empty leaves the array.
template <class C>
__device__ uint32_t far_cancel(C& c, uint32_t k, long long p, uint32_t ch, uint32_t slot, int q, int qv,
                               uint32_t nxt, uint32_t prv) {
  const int lane = lane_id();
  const gptr<FarLevel> a = far_arr(c, k);
  const gptr<Chunk> chunks = c.fchunks();
  const uint32_t n = c.fcount(k);
  wave_mem_order();
  const uint32_t pos = far_rank(a, n, p, k);
  if (pos >= n) {
    c.ferr(ERR_INCONSISTENT);
    return 0;
  }
  FarLevel e = far_get(a, pos);
  if (e.price != p) {
    c.ferr(ERR_INCONSISTENT);
    return 0;
  }
  if (lane == 0) chunks[ch].qty[slot] = 0;
  e.total -= q;
  c.fresting(-1);
  const uint32_t live_after = (uint32_t)__popcll(__ballot(qv > 0)) - 1u;
  if (live_after == 0u) {
    if (e.head == ch && e.tail == ch) {
      e.head = e.tail = NIL;
      e.tend = 0;
    } else if (e.head == ch) {
      e.head = nxt;
      if (lane == 0 && nxt < c.fnchunks()) chunks[nxt].hdr.prev = NIL;
    } else if (e.tail == ch) {
      e.tail = prv;
      e.tend = ME_C;  // a non-tail chunk is always full
      if (lane == 0 && prv < c.fnchunks()) chunks[prv].hdr.next = NIL;
    } else if (lane == 0 && prv < c.fnchunks() && nxt < c.fnchunks()) {
      chunks[prv].hdr.next = nxt;
      chunks[nxt].hdr.prev = prv;
    }
    c.ffree(ch);
  }
  if (e.total == 0) {
    if (e.head != NIL) c.ferr(ERR_INCONSISTENT);
    far_shift_down(a, pos, n);
    c.fset_count(k, n - 1u);
  } else {
    far_put(a, pos, e);
  }
  return (uint32_t)q;
}

// Old-order table lookup (after a seq-ring miss): the slot k_seq_sweep recorded for seq tgt in
// epoch `epoch`, or NIL. Linear probing, 64 entries per load.
__device__ __forceinline__ uint32_t old_lookup(gptr<const OldEnt> old, unsigned long long mask, uint32_t epoch,
                                               unsigned long long tgt) {
  const int lane = lane_id();
  const unsigned long long h = old_hash(tgt) & mask;
  for (unsigned long long i = 0; i <= mask; i += 64) {
    const OldEnt e = old[(h + i + (unsigned long long)lane) & mask];
    const bool empty = e.epoch != epoch;
    const unsigned long long me_ = __ballot(empty);
    const unsigned long long mh = __ballot(!empty && e.seq == tgt);
    if (mh && (!me_ || __builtin_ctzll(mh) < __builtin_ctzll(me_))) return rl32(e.slot, __builtin_ctzll(mh));
    if (me_) return NIL;
  }
  return NIL;
}

// New window base for a re-centre around `target`: target - L/2, kept inside the range where
// invariant I holds afterwards (every bid below base + L, every ask at or above base) and where
// base + L cannot overflow. best_bid / best_ask are the symbol's overall best prices (with_bid /
// with_ask: whether any exists).
__device__ __forceinline__ long long recentre_base(long long target, uint32_t L, bool with_bid, long long best_bid,
                                                   bool with_ask, long long best_ask) {
  const long long half = (long long)(L / 2);
  const long long lo_lim = INT64_MIN, hi_lim = INT64_MAX - (long long)L + 1;
  long long nb = target < lo_lim + half ? lo_lim : target - half;
  if (nb > hi_lim) nb = hi_lim;
  if (with_bid) {
    const long long need = best_bid < lo_lim + (long long)L ? lo_lim : best_bid - (long long)L + 1;
    if (nb < need) nb = need;
  }
  if (with_ask && nb > best_ask) nb = best_ask;
  return nb;
}

}  // namespace me

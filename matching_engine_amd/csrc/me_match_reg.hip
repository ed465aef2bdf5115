// me_match_reg.hip — k_match_reg: the matching kernel for ladders of at most 128 levels (the
// depth of benchmark configurations 1, 2, 3 and 5). Same book layout in HBM and same semantics as
// the generic k_match (me_kernels.hip; pinned by oracle/oracle_book.cpp), built for the shortest
// per-record instruction chain, since a symbol's records are an inherently serial chain and one
// wavefront per symbol leaves nothing else to hide latency behind:
//
//   * the ladder's FIFO ends (head chunk, tail chunk, tail fill) live in VGPRs — level l is lane
//     l & 63 of row l >> 6 — so reading one is a v_readlane and writing one a lane select;
//   * occupancy is a 128-bit SGPR mask, so the next best price is a bit scan; whether the head
//     chunk sits in the cache is the top bit of the head row (read with the head id itself);
//   * the head chunk of every level can sit in LDS (16 slots of qty + seq: 26 KB per wave, no
//     evictions); fills, appends and cancels of a cached head never touch HBM, and every valid
//     entry is written back once at the end of the launch;
//   * level totals are only ever added to on the hot path: fire-and-forget LDS atomics;
//   * a chunk's 16 slots are ranked with a 4-step DPP scan of 32-bit saturating adds (one DPP row;
//     saturation keeps the comparison with the remaining taker quantity exact);
//   * reject reasons, prices -> levels and the per-record result records are computed for 64
//     records at a time in vector form; the serial loop visits only records that touch the book
//     and hands back three numbers per record (quantity, fill count, first scratch fill).
//
// Scalar discipline: the wave index goes through readfirstlane, so the divergence analysis sees
// every per-symbol value and branch as wave-uniform (scalar branches, no exec-mask juggling). The
// scalar file (102 SGPRs) then holds only the hot state: launch arguments live in LDS and are read
// where used (ldsu), rarely used cursors live in the wave's LDS, and the pointers / constants that
// only feed vector memory operations and vector arithmetic are kept in VGPRs (vreg).
//
// Memory-counter discipline (gfx950 counts loads AND stores in vmcnt, in issue order): a wait for a
// load also waits for every store issued before it, i.e. a full HBM write round trip. So the serial
// loop issues no global load on its common paths: the miss path of the head-chunk cache copies a
// chunk into LDS and the walk then reads LDS only; free chunk ids live in a VGPR stack (never a
// prefetched list pointer); every symbol owns a scratch slab (no per-wave atomic reservation);
// global loads are never predicated (clamped indices + selects, no branch around a load).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "me_far.hpp"
#include "me_layout.hpp"
#include "me_wave.hpp"

// Compiled twice (Makefile): rc128 (a head-chunk cache entry per level, one workgroup per CU) and
// rc64 (64 shared entries, half the LDS: two workgroups per CU). launch_match_reg (me_kernels.hip)
// takes rc128 while the grid fits the chip — every symbol's chain has a SIMD to itself, no entry is
// ever evicted — and rc64 beyond it, where two matching waves per SIMD hide each other's latency
// (same-box A/B, DESIGN.md §4: config 2 1,056 vs 888M, config 3 777 vs 1,231M orders/s).
#ifndef ME_REG_VARIANT
#define ME_REG_VARIANT rc64
#endif
namespace me {
namespace ME_REG_VARIANT {

constexpr int RL = 128;  // levels covered by this kernel
#ifndef ME_REG_CACHE
#define ME_REG_CACHE 64
#endif
// Head-chunk cache entries per wave: level l uses entry l & (RC - 1). At 64, levels l and l + 64 share
// an entry (the one cached is written back when the other comes in), which halves the wave's LDS so
// that two matching workgroups fit a CU (two matching waves per SIMD) at grids beyond one per CU.
constexpr int RC = ME_REG_CACHE;
static_assert(RC == 64 || RC == 128, "head cache: 64 or 128 entries");
// Rescan window (records of a batch scanned per pass for a bucket that overflowed): 64 * RSU.
#ifndef ME_RESCAN_UNITS
#define ME_RESCAN_UNITS 12
#endif
constexpr int RSU = ME_RESCAN_UNITS;
constexpr uint32_t RSW = 64u * RSU;
__device__ __forceinline__ int ce(int lvl) { return lvl & (RC - 1); }
constexpr int FSTK = 64; // free chunk ids a wave keeps in its VGPR stack (= fcache row length)
// Head-row flag: set unless cache entry l holds level l's head chunk (chunk ids stay below 2^31;
// NIL, an empty level, reads as not cached).
constexpr uint32_t HC = 0x80000000u;

// One wave's LDS: the head-chunk cache (entry ce(l) = head chunk of level l when l is cached) and the
// level totals.
struct RegLds {
  int cq[RC][ME_C];
  unsigned long long cs[RC][ME_C];
  long long tot[RL];
  long long tdummy[64];  // tot_add: the slots of lanes 1..63
  uint32_t cnext[RC];  // chunks[head].hdr.next of the cached head (kept in step with HBM)
  uint32_t free_head;  // overflow free list in HBM (hdr.next links), NIL if empty
  uint32_t bump_cur, bump_end;  // chunk ids reserved from the global bump allocator
  uint32_t resting0;  // the symbol's resting orders when the wave started (ST_RESTING delta)
  uint32_t scan_cur, scan_cnt, scan_pos;  // rescan of an overfull bucket: next batch index, list fill, list read
  uint32_t mode;  // record source: 0 bucket, 1 rescan, 2 sort path (perm run [run_lo, run_lo + run_n))
  uint32_t g_cur, g_next;  // batch of the group being matched (its outputs: G.bt[g_cur]), the next one
  uint32_t run_lo, run_n;
  int dq;                 // reg_rest: LDS target of an append to an uncached tail
  unsigned long long dsq;
  uint32_t nfar[2];       // far-level counts of the symbol (me_far.hpp), rare-path state
  uint32_t epoch;         // old-order table epoch of this launch
  uint32_t pad2;
  unsigned long long horizon;  // seqs below it may live in the old-order table instead of the ring
  union {
    struct {  // the symbol's bucket, staged for the batch-order gather
      unsigned long long seq[BK_CAP];
      long long px[BK_CAP];
      int qty[BK_CAP];
      uint32_t ok[BK_CAP];
    } b;
    uint32_t lst[RSW];  // rescan: batch indices of the symbol's records in one RSW-record window
  } in;
};
#ifndef ME_REG_WAVES
#define ME_REG_WAVES 4
#endif
constexpr int REG_WAVES = ME_REG_WAVES;  // matching waves (symbols) per workgroup; as many side-job waves follow
constexpr int VMCNT0 = 0x0F70;  // s_waitcnt immediate: vmcnt(0), expcnt / lgkmcnt untouched (gfx9 encoding)

// One 32-bit field of the 128-level ladder: level l is lane (l & 63) of row (l >> 6).
struct Row2 {
  uint32_t r0, r1;
  __device__ __forceinline__ uint32_t get(int l) const { return rl32(l < 64 ? r0 : r1, l & 63); }
  __device__ __forceinline__ void put(int l, uint32_t v) {
    const int lane = lane_id();
    r0 = lane == l ? v : r0;  // l >= 64 never matches a lane of row 0
    r1 = lane == l - 64 ? v : r1;
  }
};

// 128-bit wave-uniform bit set over the levels.
struct Mask2 {
  unsigned long long w0, w1;
  static __device__ __forceinline__ unsigned long long lo(int l) { return l < 64 ? (1ull << (l & 63)) : 0ull; }
  static __device__ __forceinline__ unsigned long long hi(int l) { return l >= 64 ? (1ull << (l & 63)) : 0ull; }
  __device__ __forceinline__ bool bit(int l) const { return ((l < 64 ? w0 : w1) >> (l & 63)) & 1ull; }
  __device__ __forceinline__ void set(int l) {
    w0 |= lo(l);
    w1 |= hi(l);
  }
  __device__ __forceinline__ void clr(int l) {
    w0 &= ~lo(l);
    w1 &= ~hi(l);
  }
  // smallest set bit >= x (x may be 128), or 128 if none
  __device__ __forceinline__ int next(int x) const {
    if (x < 64) {
      const unsigned long long w = w0 & (~0ull << x);
      if (w) return __builtin_ctzll(w);
      return w1 ? 64 + __builtin_ctzll(w1) : RL;
    }
    if (x >= RL) return RL;
    const unsigned long long w = w1 & (~0ull << (x - 64));
    return w ? 64 + __builtin_ctzll(w) : RL;
  }
  // largest set bit <= x (x may be -1), or -1 if none
  __device__ __forceinline__ int prev(int x) const {
    if (x >= 64) {
      const unsigned long long w = w1 & (~0ull >> (63 - (x - 64)));
      if (w) return 127 - __builtin_clzll(w);
      return w0 ? 63 - __builtin_clzll(w0) : -1;
    }
    if (x < 0) return -1;
    const unsigned long long w = w0 & (~0ull >> (63 - x));
    return w ? 63 - __builtin_clzll(w) : -1;
  }
};

// The launch arguments, copied to LDS once per workgroup. Everything the serial loop does not
// touch on its common paths is read back from here where it is used (ldsu), so those values hold
// no SGPRs across the loop — the hot state (masks, best prices, cursors) keeps the scalar file.
struct ColdArgs {
  BookDev bk;
  BatchDev bt[ME_GMAX];  // the match job: batches [0, ng) of group J-1, in stream order
  AuxDev ax;
  uint32_t ng;
  uint32_t pad;
};

// A wave-uniform value read from LDS at the point of use. A relaxed atomic load is never hoisted out
// of a loop (a plain load would be, pinning the value in SGPRs for the whole loop) and, unlike a
// volatile one, keeps its LDS address space (ds_read, not flat); readfirstlane makes it scalar.
template <class T>
__device__ __forceinline__ T ldsu(const T& f) {
  static_assert(sizeof(T) == 8 || sizeof(T) == 4, "ldsu: 4- or 8-byte values");
  if constexpr (sizeof(T) == 8) {
    const unsigned long long v = __hip_atomic_load((const unsigned long long*)&f, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
    // readfirstlane (first ACTIVE lane): readlane 0 may read an inactive lane in a divergent branch
    const unsigned long long r =
        ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    return __builtin_bit_cast(T, r);
  } else {
    const uint32_t v = __hip_atomic_load((const uint32_t*)&f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return __builtin_bit_cast(T, (uint32_t)__builtin_amdgcn_readfirstlane((int)v));
  }
}

// A pointer launch argument read from LDS, as a global-address-space pointer (global_* ops).
template <class T>
__device__ __forceinline__ gptr<T> ldsg(T* const& f) {
  return (gptr<T>)ldsu(reinterpret_cast<const unsigned long long&>(f));
}

// Store a wave-uniform 32-bit value into the wave's LDS (lane 0; read back with ldsu).
__device__ __forceinline__ void ldsw(uint32_t& f, uint32_t v) {
  if (lane_id() == 0) __hip_atomic_store(&f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}


struct RegCtx {
  gptr<Chunk> chunks;    // VGPR
  gptr<uint32_t> loc;    // VGPR
  unsigned long long rmask;  // VGPR: seq ring mask
  gptr<me_fill> scratch; // VGPR
  RegLds* M;
  const ColdArgs* G;
  long long base;      // VGPR (price of level 0: vector uses only)
  uint32_t gs;         // VGPR (symbol id written into fills)
  uint32_t nchunks;
  uint32_t s;
  Row2 hd, tl, te;     // head chunk (| HC unless cached), tail chunk, slots written in the tail chunk
  Mask2 occ;           // occupied levels
  int bb, ba;          // best bid level (-1: none), best ask level (RL: none)
  uint32_t fstk;       // VGPR stack of free chunk ids: lane i holds entry i ...
  uint32_t nfs;        // ... entries [0, nfs) are valid
  uint32_t recs_left;  // records of this wave not yet processed (>= chunks it can still need)
  int resting;
  uint32_t wptr, wend; // next scratch fill of this wave and the end of its reservation
#ifdef ME_STAMPS
  unsigned long long st[PH_N];
  unsigned long long st_t;
#endif
  // far-level interface (me_far.hpp): all rare-path, state read back from LDS where used
  __device__ __forceinline__ gptr<Chunk> fchunks() const { return chunks; }
  __device__ __forceinline__ uint32_t fnchunks() const { return nchunks; }
  __device__ __forceinline__ uint32_t fsym() const { return s; }
  __device__ __forceinline__ uint32_t fgsym() const { return gs; }
  __device__ __forceinline__ FarDir* fdirp(uint32_t k) const {
    return (FarDir*)(ldsg(G->bk.fdir) + (size_t)s * 2u + k);
  }
  __device__ __forceinline__ FarLevel* farena() const { return (FarLevel*)ldsg(G->bk.far); }
  __device__ __forceinline__ unsigned long long* fctl() const { return (unsigned long long*)ldsg(G->bk.far_ctl); }
  __device__ __forceinline__ unsigned long long* fstats() const { return (unsigned long long*)ldsg(G->bk.stats); }
  __device__ __forceinline__ uint32_t fcap0() const { return ldsu(G->bk.fcap); }
  __device__ __forceinline__ unsigned long long finline() const { return 2ull * ldsu(G->bk.S) * fcap0(); }
  __device__ __forceinline__ unsigned long long fhalf() const { return ldsu(G->bk.far_half); }
  __device__ __forceinline__ gptr<FarLevel> farr(uint32_t k) const { return far_arr(*this, k); }
  __device__ __forceinline__ uint32_t fcount(uint32_t k) const { return ldsu(M->nfar[k]); }
  __device__ __forceinline__ void fset_count(uint32_t k, uint32_t n) {
    if (lane_id() == 0) __hip_atomic_store(&M->nfar[k], n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __device__ __forceinline__ void femit(bool fe, unsigned long long fm, const me_fill& F) {
    if (fe) scratch[wptr + (uint32_t)__builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u)] = F;  // lanes 0..15
    wptr += (uint32_t)__popcll(fm);
  }
  __device__ __forceinline__ void fresting(int d) { resting += d; }
  __device__ __forceinline__ void floc(unsigned long long seq, uint32_t g) {
    if (lane_id() == 0) loc[seq & rmask] = g;
  }
  __device__ __forceinline__ void ferr(uint32_t bits);
  __device__ __forceinline__ uint32_t falloc();
  __device__ __forceinline__ void ffree(uint32_t ch);
};

__device__ __forceinline__ void reg_err(const RegCtx& c, uint32_t bits) {
  if (lane_id() == 0) atomicOr(ldsg(c.G->bk.err), bits);
}
__device__ __forceinline__ void RegCtx::ferr(uint32_t bits) { reg_err(*this, bits); }

// Level totals only ever change by adds. Every lane issues the atomic — lane 0 into the level's
// total, lanes 1..63 into their own dummy slot — so a one-lane update needs no exec-mask dance.
__device__ __forceinline__ void tot_add(RegCtx& c, int lvl, long long d) {
  const int lane = lane_id();
  long long* p = lane == 0 ? &c.M->tot[lvl] : &c.M->tdummy[lane];
  __hip_atomic_fetch_add(p, d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// ---- chunk pool ----------------------------------------------------------------------------
// Free-list push of a chunk whose HBM quantities are all zero: onto the VGPR stack, or (stack
// full) onto the HBM overflow list — a store, never a load.
__device__ __forceinline__ void reg_free(RegCtx& c, uint32_t ch) {
  if (ME_LIKELY(c.nfs < (uint32_t)FSTK)) {
    c.fstk = lane_id() == (int)c.nfs ? ch : c.fstk;
    c.nfs += 1;
  } else {
    const uint32_t fh = ldsu(c.M->free_head);
    if (lane_id() == 0) c.chunks[ch].hdr.next = fh;
    ldsw(c.M->free_head, ch);
  }
}

// Stack ran dry: pop the HBM overflow list (one dependent load) or reserve a block of the global
// pool, which becomes the (empty) stack. Rare path.
__device__ __forceinline__ uint32_t reg_alloc_slow(RegCtx& c) {
  const uint32_t fh = ldsu(c.M->free_head);
  if (fh != NIL) {
    if (fh >= c.nchunks) {
      reg_err(c, ERR_INCONSISTENT);
      return NIL;
    }
    ldsw(c.M->free_head, rl32(c.chunks[fh].hdr.next, 0));
    return fh;
  }
  // each record needs at most one new chunk: never reserve more than the records left
  const uint32_t blk = min(16u, max(c.recs_left, 1u));
  uint32_t got = 0;
  if (lane_id() == 0) got = atomicAdd(ldsg(c.G->bk.chunk_top), blk);
  got = rl32(got, 0);
  const CPool p = cp_read(ldsg(c.G->bk.cpool));
  const uint32_t vcap = cp_vcap(p, c.nchunks);
  if (got >= vcap) {
    reg_err(c, ERR_CHUNK_OOM);
    return NIL;
  }
  const uint32_t nb = min(blk, vcap - got);
  const uint32_t l = (uint32_t)lane_id();
  const uint32_t id = l < nb ? cp_id(ldsg(c.G->bk.recl), p, got + l) : NIL;
  // the chunks belong to this symbol until a reclamation finds them free (unused ones stay on its stack)
  if (l < nb) c.chunks[id].owner = c.s;
  c.fstk = l < nb ? id : c.fstk;  // (reg_alloc pops the stack first: it is empty here)
  c.nfs = nb - 1u;
  return rl32(id, (int)(nb - 1u));
}

__device__ __forceinline__ uint32_t reg_alloc(RegCtx& c) {
  if (ME_LIKELY(c.nfs != 0u)) {
    c.nfs -= 1;
    return rl32(c.fstk, (int)c.nfs);
  }
  return reg_alloc_slow(c);
}
__device__ __forceinline__ uint32_t RegCtx::falloc() { return reg_alloc(*this); }
__device__ __forceinline__ void RegCtx::ffree(uint32_t ch) { reg_free(*this, ch); }

// ---- head-chunk cache ------------------------------------------------------------------------
// Level lvl's head is about to enter entry ce(lvl): if the level sharing the entry holds it, that
// level's head goes back to HBM and becomes uncached (its head row gets HC again).
__device__ __forceinline__ void reg_evict_partner(RegCtx& c, int lvl) {
  if constexpr (RC < RL) {
    const int p = lvl ^ RC;
    const uint32_t hv = c.hd.get(p);
    if (ME_UNLIKELY((hv & HC) == 0u)) {
      const int lane = lane_id();
      const int e = ce(lvl);
      if (lane < ME_C) {
        c.chunks[hv].qty[lane] = c.M->cq[e][lane];
        c.chunks[hv].seq[lane] = c.M->cs[e][lane];
      }
      c.hd.put(p, hv | HC);
    }
  }
}

// Miss: copy chunk ch (the head of level lvl) into cache entry lvl. The only global load of a walk;
// its registers die at the LDS writes, so no wait on it leaks into the hit path.
__device__ __forceinline__ bool reg_fill_entry(RegCtx& c, int lvl, uint32_t ch) {
  if (ME_UNLIKELY(ch >= c.nchunks)) {  // NIL or corrupt: never index with it
    reg_err(c, ERR_INCONSISTENT);
    return false;
  }
  const int lane = lane_id();
  const int sl = lane & (ME_C - 1);
  const uint32_t nx = c.chunks[ch].hdr.next;
  const int qv = c.chunks[ch].qty[sl];
  const unsigned long long sv = c.chunks[ch].seq[sl];
  // Resolve the loads on every path here (vmcnt(0)): a load left pending behind the lane-masked
  // LDS writes below would make the compiler wait for it (and all later stores) in the hit path.
  __builtin_amdgcn_s_waitcnt(VMCNT0);
  if (lane < ME_C) {
    c.M->cq[ce(lvl)][sl] = qv;
    c.M->cs[ce(lvl)][sl] = sv;
  }
  if (lane == 0) c.M->cnext[ce(lvl)] = nx;
  return true;
}

// ---- taking liquidity ----------------------------------------------------------------------
// Consume up to `rem` from the chunk held by cache entry lvl (the head of level lvl), oldest slot
// first, one fill per maker slot touched. Returns true if every slot of the chunk is consumed.
// A slot is live iff its qty > 0.
__device__ __forceinline__ bool reg_take_chunk(RegCtx& c, int lvl, uint32_t& rem, uint32_t& taken,
                                               unsigned long long taker, long long price) {
  const int lane = lane_id();
  const bool act = lane < ME_C;
  const int sl = lane & (ME_C - 1);
  COUNT(c, CT_WALK);
  const int q_ = c.M->cq[ce(lvl)][sl];
  // read with the quantities (one LDS round trip); the opaque use keeps it from sinking into the
  // fill branch, where it would be a second round trip
  const unsigned long long mseq = vreg64(c.M->cs[ce(lvl)][sl]);
  const uint32_t uq = act ? (uint32_t)q_ : 0u;
  const uint32_t inc = scan16_sat(uq);
  const uint32_t ex = inc - uq;
  uint32_t f = rem > ex ? rem - ex : 0u;
  f = f < uq ? f : uq;
  const bool fe = f != 0u;
  const unsigned long long fm = __ballot(fe);
  if (fe) {
    me_fill F;
    F.taker_seq = taker;
    F.maker_seq = mseq;
    F.price_q4 = price;
    F.qty = (int)f;
    F.symbol = c.gs;
    // fills only ever come from lanes 0..15: mbcnt_lo alone ranks them
    c.scratch[c.wptr + (uint32_t)__builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u)] = F;
    c.M->cq[ce(lvl)][sl] = (int)(uq - f);
  }
  c.wptr += (uint32_t)__popcll(fm);
  c.resting -= __popcll(__ballot(f == uq) & fm);  // makers filled completely leave the book
  const uint32_t live = rl32(inc, 15);
  const uint32_t t = rem < live ? rem : live;
  rem -= t;
  taken += t;
  return (__ballot(uq > f) & 0xFFFFull) == 0ull;  // no live slot left (slots are lanes 0..15)
}

// Taker against level lvl. The common case is straight-line: the cached head chunk keeps live
// slots once the taker is done. Returns true if the level emptied.
__device__ __forceinline__ bool reg_walk(RegCtx& c, int lvl, uint32_t& rem, unsigned long long taker) {
  const int lane = lane_id();
  const long long price = c.base + lvl;
  const uint32_t hv = c.hd.get(lvl);
  uint32_t ch = hv & ~HC;  // an occupied level: a real chunk id
  if (ME_UNLIKELY(hv & HC)) {
    COUNT(c, CT_MISS);
    reg_evict_partner(c, lvl);
    if (!reg_fill_entry(c, lvl, ch)) return false;
    c.hd.put(lvl, ch);  // now cached
  }
  uint32_t taken = 0;
  if (ME_LIKELY(!reg_take_chunk(c, lvl, rem, taken, taker, price))) {
    tot_add(c, lvl, -(long long)taken);
    return false;
  }
  // the head chunk is exhausted: free it and continue down the FIFO (each next chunk is a miss)
  const uint32_t tail = c.tl.get(lvl);
  bool cached = false;  // whether the level's new head ends up in the cache
  for (;;) {
    const uint32_t nx = rl32(c.M->cnext[ce(lvl)], 0);
    if (lane < ME_C) c.chunks[ch].qty[lane] = 0;  // a freed chunk must read all-zero in HBM
    reg_free(c, ch);
    if (ch == tail) {
      c.hd.put(lvl, NIL);
      c.tl.put(lvl, NIL);
      c.occ.clr(lvl);
      tot_add(c, lvl, -(long long)taken);
      return true;
    }
    ch = nx;
    if (rem == 0u) break;
    COUNT(c, CT_MISS);
    if (!reg_fill_entry(c, lvl, ch)) {
      c.hd.put(lvl, ch | HC);
      return false;
    }
    if (!reg_take_chunk(c, lvl, rem, taken, taker, price)) {
      cached = true;
      break;
    }
  }
  tot_add(c, lvl, -(long long)taken);
  c.hd.put(lvl, cached ? ch : (ch | HC));
  if (lane == 0 && ch < c.nchunks) c.chunks[ch].hdr.prev = NIL;  // new FIFO head
  return false;
}

// ---- resting -------------------------------------------------------------------------------
// Append (seq, qty) at the tail of level lvl. Common case first: a free slot in the tail chunk
// (written on chip when the tail is the cached head). The new-chunk path is out of line.
__device__ __forceinline__ bool reg_rest_new_chunk(RegCtx& c, int lvl, unsigned long long seq, uint32_t qty,
                                                   uint32_t tl) {
  const int lane = lane_id();
  const uint32_t ch = reg_alloc(c);
  if (ch == NIL) return false;
  if (lane == 0) {
    ChunkHdr h;
    h.next = NIL;
    h.prev = tl;
    h.price = c.base + lvl;
    c.chunks[ch].hdr = h;
    c.loc[seq & c.rmask] = ch * ME_C;
  }
  if (tl == NIL) {  // empty level: the new chunk is its head, installed in the cache
    reg_evict_partner(c, lvl);
    c.hd.put(lvl, ch);  // cached
    if (lane < ME_C) c.M->cq[ce(lvl)][lane] = lane == 0 ? (int)qty : 0;
    if (lane == 0) {
      c.M->cs[ce(lvl)][0] = seq;
      c.M->cnext[ce(lvl)] = NIL;
    }
    c.occ.set(lvl);
  } else {
    const bool tl_cached = c.hd.get(lvl) == tl;  // the tail is the cached head
    if (lane == 0) {
      if (tl < c.nchunks) c.chunks[tl].hdr.next = ch;
      if (tl_cached) c.M->cnext[ce(lvl)] = ch;
      c.chunks[ch].qty[0] = (int)qty;
      c.chunks[ch].seq[0] = seq;
    }
  }
  c.tl.put(lvl, ch);
  c.te.put(lvl, 1u);
  return true;
}

__device__ __forceinline__ bool reg_rest(RegCtx& c, int lvl, unsigned long long seq, uint32_t qty, bool buy) {
  const int lane = lane_id();
  const uint32_t tl = c.tl.get(lvl);
  const uint32_t te = c.te.get(lvl);
  if (ME_LIKELY(tl != NIL && te < (uint32_t)ME_C)) {
    if (ME_UNLIKELY(tl >= c.nchunks)) {
      reg_err(c, ERR_INCONSISTENT);
      return false;
    }
    const bool in_cache = c.hd.get(lvl) == tl;  // the tail is the cached head
    if (lane == 0) {
      // no branch on in_cache: the HBM slot is written either way (a cached tail is written back
      // from LDS at the end anyway) and the LDS copy goes to the entry or to a dummy slot
      int* lq = in_cache ? &c.M->cq[ce(lvl)][te] : &c.M->dq;
      unsigned long long* ls = in_cache ? &c.M->cs[ce(lvl)][te] : &c.M->dsq;
      *lq = (int)qty;
      *ls = seq;
      c.chunks[tl].qty[te] = (int)qty;
      c.chunks[tl].seq[te] = seq;
      c.loc[seq & c.rmask] = tl * ME_C + te;
    }
    c.te.put(lvl, te + 1u);
  } else if (!reg_rest_new_chunk(c, lvl, seq, qty, tl)) {
    return false;
  }
  tot_add(c, lvl, (long long)qty);
  if (buy)
    c.bb = lvl > c.bb ? lvl : c.bb;
  else
    c.ba = lvl < c.ba ? lvl : c.ba;
  c.resting += 1;
  return true;
}

// ---- cancelling ----------------------------------------------------------------------------
// Remove the live resting order `tgt` of this symbol; returns its qty, 0 if not live. The seq ring
// names its slot unless a later seq overwrote the entry, in which case an order older than the
// horizon is in the old-order table; every candidate slot is verified (owner, seq, qty > 0). A chunk
// left without live orders is unlinked at once (chunks in use never exceed resting orders).
// kSlow = false (k_match_reg<false>): a window order named by its ring entry is cancelled here; every
// other case (a far level, a stale ring entry of an order older than the horizon) returns HANDOFF
// before anything changed, and the continuation launch (kSlow = true) does the whole cancel.
constexpr uint32_t HANDOFF = 0xFFFFFFFFu;
// gh: the ring entry read for the whole block at its start (NIL: none); a slot it names is verified like
// any other, and one that does not hold tgt sends the cancel to the ring as if there were no hint.
template <bool kSlow>
__device__ __forceinline__ uint32_t reg_cancel(RegCtx& c, unsigned long long tgt, uint32_t gh) {
  const int lane = lane_id();
  const bool act = lane < ME_C;
  if (tgt == 0ull) return 0;
  bool hinted = gh != NIL;
  uint32_t g = gh;
  if (!hinted) {
    wave_mem_order();
    g = rl32(c.loc[tgt & c.rmask], 0);
    __builtin_amdgcn_s_waitcnt(VMCNT0);
  }
  for (int pass = 0;; ++pass) {
    if (g != NIL && g / ME_C < c.nchunks) {
      const uint32_t ch = g / ME_C, slot = g % ME_C;
      // one round trip: header, price, the chunk's quantities and the target seq
      const ChunkHdr hdr = c.chunks[ch].hdr;
      const uint32_t owner = c.chunks[ch].owner;
      const long long price = hdr.price;
      const int qg = c.chunks[ch].qty[lane & (ME_C - 1)];
      unsigned long long sq = rl64(c.chunks[ch].seq[slot], 0);
      __builtin_amdgcn_s_waitcnt(VMCNT0);  // resolved on every path (see reg_fill_entry)
      int qv = act ? qg : 0;
      const uint32_t own = rl32(owner, 0);
      const long long prc = rli64(price, 0);
      const long long lv64 = prc - rli64(c.base, 0);
      // in the window: [0, L) — not [0, RL): at L = 64 the second ladder row is no level (a far order
      // 64..127 levels above base was once cancelled as a window order, corrupting the book)
      const bool inw = own == c.s && (unsigned long long)lv64 < (unsigned long long)ldsu(c.G->bk.L);
      const int lvl = inw ? (int)lv64 : 0;
      const uint32_t hv = c.hd.get(lvl);
      const bool in_cache = inw && hv == ch;  // ch is the cached head: the on-chip copy is authoritative
      if (in_cache) {
        const int qc = c.M->cq[ce(lvl)][lane & (ME_C - 1)];
        qv = act ? qc : 0;
        sq = rl64(c.M->cs[ce(lvl)][slot], 0);
      }
      if (own == c.s && sq == tgt) {  // the order's slot: live or dead, it never moves
        const int q = rli32(qv, (int)slot);
        if (q <= 0) return 0;
        const uint32_t nxt = rl32(hdr.next, 0), prv = rl32(hdr.prev, 0);
        if (ME_UNLIKELY(!inw)) {  // a far level (me_far.hpp)
          if constexpr (kSlow)
            return far_cancel(c, prc < rli64(c.base, 0) ? 0u : 1u, prc, ch, slot, q, qv, nxt, prv);
          else
            return HANDOFF;
        }
        const uint32_t t = c.tl.get(lvl);
        const uint32_t h = hv == NIL ? NIL : (hv & ~HC);
        const uint32_t live_after = (uint32_t)__popcll(__ballot(qv > 0)) - 1u;
        if (lane == 0) {
          if (in_cache)
            c.M->cq[ce(lvl)][slot] = 0;
          else
            c.chunks[ch].qty[slot] = 0;
        }
        tot_add(c, lvl, -(long long)q);
        if (live_after == 0u) {
          if (h >= c.nchunks || t >= c.nchunks) {
            reg_err(c, ERR_INCONSISTENT);
            return (uint32_t)q;
          }
          if (in_cache) {  // the chunk leaves the cache; its HBM copy must read all-zero
            if (act) c.chunks[ch].qty[lane] = 0;
          }
          const bool mirror = hv == prv;  // the cached head is ch's predecessor
          if (h == t) {  // ch was the level's only chunk: the level empties
            c.hd.put(lvl, NIL);
            c.tl.put(lvl, NIL);
            c.occ.clr(lvl);
            if (lvl == c.bb) c.bb = c.occ.prev(lvl);
            if (lvl == c.ba) c.ba = c.occ.next(lvl);
          } else if (ch == h) {
            c.hd.put(lvl, nxt | HC);  // the new head is not cached
            if (lane == 0) c.chunks[nxt].hdr.prev = NIL;
          } else if (ch == t) {
            c.tl.put(lvl, prv);
            c.te.put(lvl, ME_C);  // a non-tail chunk is always full
            if (lane == 0) {
              c.chunks[prv].hdr.next = NIL;
              if (mirror) c.M->cnext[ce(lvl)] = NIL;
            }
          } else {
            if (lane == 0) {
              c.chunks[prv].hdr.next = nxt;
              c.chunks[nxt].hdr.prev = prv;
              if (mirror) c.M->cnext[ce(lvl)] = nxt;
            }
          }
          reg_free(c, ch);
        }
        c.resting -= 1;
        return (uint32_t)q;
      }
    }
    if (hinted) {  // the block-start entry is stale: the ring now
      hinted = false;
      wave_mem_order();
      g = rl32(c.loc[tgt & c.rmask], 0);
      __builtin_amdgcn_s_waitcnt(VMCNT0);
      --pass;
      continue;
    }
    // the ring entry is someone else's: only an order older than the horizon can still be live
    if (pass != 0 || tgt >= ldsu(c.M->horizon)) return 0;
    if constexpr (kSlow) {
      g = old_lookup(ldsg(c.G->bk.old), ldsu(c.G->bk.old_mask), ldsu(c.M->epoch), tgt);
      if (g == NIL) return 0;
    } else {
      return HANDOFF;
    }
  }
}

// ---- re-centring the window (rare) ----------------------------------------------------------
// Level j of a 128-lane row pair after a shift by d: old level j + d, or `fill` outside [0, L).
__device__ __forceinline__ uint32_t row_pick(uint32_t o0, uint32_t o1, int src, uint32_t L, uint32_t fill) {
  const int a = (src & 63) << 2;
  const uint32_t v0 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)o0);
  const uint32_t v1 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)o1);
  return (src >= 0 && src < (int)L) ? (src < 64 ? v0 : v1) : fill;
}
__device__ __forceinline__ void row_shift(Row2& r, int d, uint32_t L, uint32_t fill) {
  const int lane = lane_id();
  const uint32_t o0 = r.r0, o1 = r.r1;
  r.r0 = row_pick(o0, o1, lane + d, L, fill);
  const uint32_t n1 = row_pick(o0, o1, 64 + lane + d, L, fill);
  r.r1 = 64u + (uint32_t)lane < L ? n1 : fill;
}

// Install far level e as window level j (its head chunk is not cached).
__device__ __forceinline__ void reg_install(RegCtx& c, int j, const FarLevel& e) {
  c.hd.put(j, e.head | HC);
  c.tl.put(j, e.tail);
  c.te.put(j, e.tend);
  if (lane_id() == 0) c.M->tot[j] = e.total;
}

// Move the window so that it is centred on `target` as far as invariant I allows (me_far.hpp
// recentre_base): cached heads go back to HBM (the cache is indexed by window level), levels leaving
// the window become far levels at the best end of their side, the ladder rows and totals shift, and
// far levels now inside the window are popped into it. Chunks name their level by price, so none
// of them changes.
__device__ __forceinline__ void reg_recentre(RegCtx& c, long long target) {
  const int lane = lane_id();
  const uint32_t L = ldsu(c.G->bk.L);
  const long long base = rli64(c.base, 0);
  const uint32_t n0 = c.fcount(0), n1 = c.fcount(1);
  const bool wb = c.bb >= 0, wa = c.ba < (int)L;
  long long bbp = 0, bap = 0;
  if (wb)
    bbp = base + c.bb;
  else if (n0)
    bbp = far_get(c.farr(0), n0 - 1u).price;
  if (wa)
    bap = base + c.ba;
  else if (n1)
    bap = far_get(c.farr(1), n1 - 1u).price;
  const long long nb = recentre_base(target, L, wb || n0 != 0u, bbp, wa || n1 != 0u, bap);
  if (nb == base) return;
  const bool up = nb > base;
  const unsigned long long dist =
      up ? (unsigned long long)nb - (unsigned long long)base : (unsigned long long)base - (unsigned long long)nb;
  const int dm = dist >= L ? (int)L : (int)dist;
  const int d = up ? dm : -dm;
  // 1. cached heads back to HBM
  for (int row = 0; row < 2; ++row) {
    unsigned long long cm = __ballot(((row ? c.hd.r1 : c.hd.r0) & HC) == 0u);
    while (cm) {
      const int jj = __builtin_ctzll(cm);
      cm &= cm - 1ull;
      const uint32_t cid = rl32(row ? c.hd.r1 : c.hd.r0, jj);
      const int e = ce(row * 64 + jj);
      if (lane < ME_C) {
        c.chunks[cid].qty[lane] = c.M->cq[e][lane];
        c.chunks[cid].seq[lane] = c.M->cs[e][lane];
      }
    }
  }
  c.hd.r0 |= HC;
  c.hd.r1 |= HC;
  // 2. levels leaving the window: bids at the bottom (moving up), asks at the top (moving down)
  if (d > 0) {
    for (int l = c.occ.next(0); l < d; l = c.occ.next(l + 1)) {
      if (l > c.bb) reg_err(c, ERR_INCONSISTENT);
      FarLevel e;
      e.price = base + l;
      e.total = ldsu(c.M->tot[l]);
      e.head = c.hd.get(l) & ~HC;
      e.tail = c.tl.get(l);
      e.tend = c.te.get(l);
      e.pad = 0;
      far_push(c, 0u, e);
    }
  } else {
    for (int l = c.occ.prev((int)L - 1); l >= (int)L + d; l = c.occ.prev(l - 1)) {
      if (l < c.ba) reg_err(c, ERR_INCONSISTENT);
      FarLevel e;
      e.price = base + l;
      e.total = ldsu(c.M->tot[l]);
      e.head = c.hd.get(l) & ~HC;
      e.tail = c.tl.get(l);
      e.tend = c.te.get(l);
      e.pad = 0;
      far_push(c, 1u, e);
    }
  }
  // 3. shift the window
  row_shift(c.hd, d, L, NIL);
  row_shift(c.tl, d, L, NIL);
  row_shift(c.te, d, L, 0u);
  {
    const long long t0 = c.M->tot[lane], t1 = c.M->tot[64 + lane];
    const uint32_t l0 = row_pick((uint32_t)t0, (uint32_t)t1, lane + d, L, 0u);
    const uint32_t h0 = row_pick((uint32_t)(t0 >> 32), (uint32_t)(t1 >> 32), lane + d, L, 0u);
    const uint32_t l1 = row_pick((uint32_t)t0, (uint32_t)t1, 64 + lane + d, L, 0u);
    const uint32_t h1 = row_pick((uint32_t)(t0 >> 32), (uint32_t)(t1 >> 32), 64 + lane + d, L, 0u);
    c.M->tot[lane] = (long long)(((unsigned long long)h0 << 32) | l0);
    c.M->tot[64 + lane] = 64u + (uint32_t)lane < L ? (long long)(((unsigned long long)h1 << 32) | l1) : 0ll;
  }
  int nbb = (c.bb >= 0 && c.bb - d >= 0) ? c.bb - d : -1;
  int nba = (c.ba < (int)L && c.ba - d < (int)L) ? c.ba - d : RL;
  c.base = (long long)vreg64((unsigned long long)nb);
  // 4. far levels now inside the window
  if (d < 0) {
    const gptr<FarLevel> a = c.farr(0);
    uint32_t n = c.fcount(0);
    while (n) {
      const FarLevel e = far_get(a, n - 1u);
      if (e.price < nb) break;
      const unsigned long long off = (unsigned long long)e.price - (unsigned long long)nb;
      if (off >= L) {  // impossible by recentre_base (every bid is below nb + L)
        reg_err(c, ERR_INCONSISTENT);
        break;
      }
      const int j = (int)off;
      reg_install(c, j, e);
      nbb = j > nbb ? j : nbb;
      --n;
    }
    c.fset_count(0, n);
  } else {
    const gptr<FarLevel> a = c.farr(1);
    uint32_t n = c.fcount(1);
    while (n) {
      const FarLevel e = far_get(a, n - 1u);
      const unsigned long long off = (unsigned long long)e.price - (unsigned long long)nb;  // asks >= nb
      if (off >= L) break;
      const int j = (int)off;
      reg_install(c, j, e);
      nba = j < nba ? j : nba;
      --n;
    }
    c.fset_count(1, n);
  }
  c.bb = nbb;
  c.ba = nba;
  c.occ.w0 = __ballot(c.M->tot[lane] > 0);
  c.occ.w1 = __ballot(c.M->tot[64 + lane] > 0);
}

// Rest (seq, qty) at price p outside the window. Re-centre first when the rest would put a bid above
// the window or an ask below it (invariant I) or when the window is empty; then rest in the window
// or on the far side. Returns -1 on a capacity failure, 1 when the window moved (the block's control
// words must be rebuilt), 0 otherwise.
__device__ __forceinline__ int reg_far_rest(RegCtx& c, long long p, unsigned long long seq, uint32_t qty, bool buy) {
  const uint32_t L = ldsu(c.G->bk.L);
  long long base = rli64(c.base, 0);
  const bool above = p > base;  // p is outside [base, base + L)
  const bool mandatory = buy == above;
  int moved = 0;
  if (mandatory || (c.occ.w0 | c.occ.w1) == 0ull) {
    reg_recentre(c, p);
    moved = 1;
    base = rli64(c.base, 0);
  }
  const unsigned long long off = (unsigned long long)p - (unsigned long long)base;
  if (off < L) return reg_rest(c, (int)off, seq, qty, buy) ? moved : -1;
  if (mandatory) {
    reg_err(c, ERR_INCONSISTENT);
    return -1;
  }
  return far_rest(c, p < base ? 0u : 1u, p, seq, qty) ? moved : -1;
}

// ---- scratch ---------------------------------------------------------------------------------
// The taker about to run may emit up to `resting` fills. If they might not fit the wave's slab,
// reserve the batch bound of everything left (resting + 2 * records left) in the
// shared overflow region once; after that no further check can fail.
__device__ __forceinline__ bool reg_reserve_overflow(RegCtx& c) {
  const BatchDev& B = c.G->bt[ldsu(c.M->g_cur)];
  unsigned long long* top = ldsg(B.scratch_top);
  const unsigned long long base = ldsu(B.ovf_base), cap = ldsu(B.scratch_cap);
  const unsigned long long need = (unsigned long long)(uint32_t)c.resting + 2ull * c.recs_left;
  unsigned long long w0 = 0;
  if (lane_id() == 0) w0 = atomicAdd(top, need);
  w0 = base + rl64(w0, 0);
  if (w0 + need > cap) {
    reg_err(c, ERR_SCRATCH_OOM);
    return false;
  }
  c.wptr = (uint32_t)w0;
  c.wend = 0xFFFFFFFFu;  // never re-checked
  return true;
}

// ---- batch order of a bucket -----------------------------------------------------------------
// Bitonic sort of 64 (one register) or 128 (two registers: element 64 + lane in b) distinct 32-bit
// keys across the wave, ascending; partners come over DPP / permlane swaps (xor_lane, me_wave.hpp).
template <int J>
__device__ __forceinline__ uint32_t bitonic_step(uint32_t v, bool asc) {
  const uint32_t p = xor_lane<J>(v);
  // (opaque lane id: the per-lane masks are rebuilt per sort, not hoisted out of the batch loop,
  // where they would be live SGPR pairs across the serial loop)
  const bool lower = ((int)vreg((uint32_t)lane_id()) & J) == 0;
  return (lower == asc) ? min(v, p) : max(v, p);
}
template <int K>
__device__ __forceinline__ uint32_t bitonic_merge(uint32_t v, bool asc) {
  if constexpr (K >= 64) v = bitonic_step<32>(v, asc);
  if constexpr (K >= 32) v = bitonic_step<16>(v, asc);
  if constexpr (K >= 16) v = bitonic_step<8>(v, asc);
  if constexpr (K >= 8) v = bitonic_step<4>(v, asc);
  if constexpr (K >= 4) v = bitonic_step<2>(v, asc);
  v = bitonic_step<1>(v, asc);
  return v;
}
// stages 2..64 of one register; dir1: direction of the 64-run (element 64 + lane sorts descending)
__device__ __forceinline__ uint32_t sort64(uint32_t v, bool desc64) {
  const int lane = (int)vreg((uint32_t)lane_id());
  v = bitonic_merge<2>(v, (lane & 2) == 0);
  v = bitonic_merge<4>(v, (lane & 4) == 0);
  v = bitonic_merge<8>(v, (lane & 8) == 0);
  v = bitonic_merge<16>(v, (lane & 16) == 0);
  v = bitonic_merge<32>(v, (lane & 32) == 0);
  v = bitonic_merge<64>(v, !desc64);
  return v;
}
__device__ __forceinline__ void sort128(uint32_t& a, uint32_t& b) {
  a = sort64(a, false);
  b = sort64(b, true);
  const uint32_t lo = min(a, b), hi = max(a, b);
  a = bitonic_merge<64>(lo, true);
  b = bitonic_merge<64>(hi, true);
}

// Rescan of an overfull bucket: the next RSW-record window of the batch that holds records of
// bin s, as a list of batch indices in LDS (batch order). Returns false when the batch is done.
__device__ __forceinline__ bool rescan_window(RegLds* M, const ColdArgs& G, uint32_t g, uint32_t s) {
  const int lane = lane_id();
  const uint32_t n = ldsu(G.bt[g].n), S = ldsu(G.bk.S);
  const gptr<const uint32_t> sym = ldsg(G.bt[g].sym);
  uint32_t cur = ldsu(M->scan_cur);
  while (cur < n) {
    uint32_t sy[RSU];
#pragma unroll
    for (int u = 0; u < RSU; ++u) sy[u] = sym[min(cur + 64u * u + (uint32_t)lane, n - 1u)];
    uint32_t cnt = 0;
#pragma unroll
    for (int u = 0; u < RSU; ++u) {
      const uint32_t idx = cur + 64u * u + (uint32_t)lane;
      const bool m = idx < n && min(sy[u], S) == s;
      const unsigned long long bm = __ballot(m);
      if (m) M->in.lst[cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u))] = idx;
      cnt += (uint32_t)__popcll(bm);
    }
    cur += RSW;
    if (cnt) {
      ldsw(M->scan_cur, cur);
      ldsw(M->scan_cnt, cnt);
      ldsw(M->scan_pos, 0u);
      return true;
    }
  }
  ldsw(M->scan_cur, cur);
  return false;
}

// (pipelined path: no fill start of its own — the tape job reads a record's scratch start from its
// result's tape_offset, see aux_tape_tile)
__device__ __forceinline__ void reject_bad_at(gptr<me_order_result> res, uint32_t i) {
  me_order_result r;
  r.filled_qty = 0;
  r.remaining_qty = 0;
  r.fill_count = 0;
  r.tape_offset = 0;
  r.status = ME_ST_REJECTED;
  r.reason = ME_RJ_BAD_SYMBOL;
  r.pad[0] = r.pad[1] = 0;
  res[i] = r;
}
__device__ __forceinline__ void reject_bad(const ColdArgs& G, uint32_t g, uint32_t i, bool v) {
  if (!v) return;
  me_order_result r;
  r.filled_qty = 0;
  r.remaining_qty = 0;
  r.fill_count = 0;
  r.tape_offset = 0;
  r.status = ME_ST_REJECTED;
  r.reason = ME_RJ_BAD_SYMBOL;
  r.pad[0] = r.pad[1] = 0;
  ldsg(G.bt[g].res)[i] = r;
  ldsg(G.bt[g].fstart)[i] = 0;
}

// The bad-symbol bin of the sort path (one batch): every record rejected (order irrelevant).
__device__ __forceinline__ void reject_bad_run(const ColdArgs& G, uint32_t lo, uint32_t hi) {
  const gptr<const uint32_t> perm = ldsg(G.bt[0].perm);
  for (uint32_t i = lo + (uint32_t)lane_id(); i < hi; i += 64) reject_bad(G, 0, perm[i], true);
}

// ---- side jobs of a pipelined launch (the workgroup's waves REG_WAVES .. 2*REG_WAVES-1) -------
// Memory-latency work with few instructions, so sharing the SIMDs with the matching waves costs
// them little; what it saves is two launches per batch.

// Bucket job: records [r0, r1) of bucket job j, one returning atomic per record on its bin's counter.
template <class GA>
__device__ __forceinline__ void aux_bucket(const GA& G, uint32_t j, uint32_t r0, uint32_t r1) {
  const int lane = lane_id();
  const AuxBucket& J = G.ax.b[j];
  const gptr<const uint32_t> sym = ldsg(J.sym);
  const gptr<const uint64_t> seq = ldsg(J.seq);
  const gptr<const int64_t> px = ldsg(J.px);
  const gptr<const int32_t> qty = ldsg(J.qty);
  const gptr<const uint8_t> kind = ldsg(J.kind);
  const gptr<uint32_t> bcnt = ldsg(J.bcnt);
  const gptr<BkRec> brec = ldsg(J.b_rec);
  const uint32_t S = ldsu(G.ax.S);
  const gptr<me_order_result> bres = ldsg(J.bres);
  bool order_ok = true;
  for (uint32_t i0 = r0; i0 < r1; i0 += 64) {
    const uint32_t i = i0 + (uint32_t)lane;
    if (i < r1) {
      const uint32_t k = kind[i];
      // API precondition (the seq ring relies on it): seqs ascending through the batch (seq_follows)
      if (i > 0) order_ok &= seq_follows(seq[i - 1], seq[i], k);
      const uint32_t b = min(sym[i], S);
      if (b == S) {  // unknown symbol: rejected here, never bucketed (the batch's result set is free)
        reject_bad_at(bres, i);
        continue;
      }
      const uint64_t sq = seq[i];  // the payload loads are in flight while the atomic returns
      const int64_t p = px[i];
      const int32_t q = qty[i];
      const uint32_t r = atomicAdd(&bcnt[(size_t)b * BK_CNT_STRIDE], 1u);
      if (r < (uint32_t)BK_CAP) {
        const size_t d = (size_t)b * BK_CAP + r;
        brec[d].seq = sq;
        brec[d].px = p;
        brec[d].qty = q;
        brec[d].ok = i | ((k & 15u) << BK_KIND_SHIFT);
      }
    }
  }
  if (__ballot(!order_ok) && lane == 0) atomicOr(ldsg(G.bk.err), ERR_SEQ_ORDER);
}

// Tape job j, one TILE_TAPE-record tile per wave: tape offsets of its records and the copy of their
// fills from scratch into the batch's tape (ordered by taker seq).
template <class GA>
__device__ __forceinline__ void aux_tape_tile(const GA& G, uint32_t jb, uint32_t t, uint32_t ntiles,
                                              uint32_t tn) {
  const int lane = lane_id();
  const AuxTape& J = G.ax.t[jb];
  const gptr<const uint32_t> tile_sum = ldsg(J.tile_sum);
  const gptr<me_order_result> res = ldsg(J.res);
  const gptr<const me_fill> scratch = ldsg(J.scratch);
  const gptr<me_fill> tape = ldsg(J.tape);
  const gptr<me_order_result> hres = ldsg(J.hres);
  const bool host = hres != nullptr;  // a host batch: soft tape cap, results and scratch starts kept
  const unsigned long long cap = ldsu(J.cap);
  long long acc = 0;  // fills of the earlier tiles
  for (uint32_t u = (uint32_t)lane; u < t; u += 64) acc += tile_sum[u];
  for (int d = 32; d >= 1; d >>= 1) acc += __shfl_xor(acc, d, 64);
  const unsigned long long base = (unsigned long long)rli64(acc, 0);
  const uint32_t r0 = t * TILE_TAPE;
  const uint32_t cnt = min((uint32_t)TILE_TAPE, tn - r0);
  uint32_t c[TILE_TAPE / 64], src[TILE_TAPE / 64];
  long long loc = 0;
#pragma unroll
  for (int k = 0; k < TILE_TAPE / 64; ++k) {  // lane holds records 4*lane .. 4*lane+3 of the tile
    const uint32_t j = (uint32_t)(lane * (TILE_TAPE / 64) + k);
    // the match job left the record's scratch start in tape_offset (same line as fill_count)
    c[k] = j < cnt ? res[r0 + j].fill_count : 0u;
    src[k] = j < cnt ? res[r0 + j].tape_offset : 0u;
    loc += c[k];
  }
  const long long incl = wave_incl_scan(loc);
  const uint32_t total = (uint32_t)rli64(incl, 63);
  uint32_t o = (uint32_t)(incl - loc);
#pragma unroll
  for (int k = 0; k < TILE_TAPE / 64; ++k) {
    const uint32_t j = (uint32_t)(lane * (TILE_TAPE / 64) + k);
    if (j < cnt) res[r0 + j].tape_offset = (uint32_t)(base + o);
    o += c[k];
  }
  if (host) {  // the slot's copy of the final results; the scratch starts stay for me_collect's spill
    const gptr<uint32_t> fst = ldsg(J.fstart);
    uint32_t o3 = (uint32_t)(incl - loc);
#pragma unroll
    for (int k = 0; k < TILE_TAPE / 64; ++k) {
      const uint32_t j = (uint32_t)(lane * (TILE_TAPE / 64) + k);
      if (j < cnt) {
        me_order_result r = res[r0 + j];  // written by the match job of an earlier launch
        r.tape_offset = (uint32_t)(base + o3);
        hres[r0 + j] = r;
        fst[r0 + j] = src[k];
      }
      o3 += c[k];
    }
  } else if (base + total > cap) {
    if (lane == 0) atomicOr(ldsg(G.bk.err), ERR_SCRATCH_OOM);
    return;
  }
  // The tile's fills are one contiguous tape run [base, base + total): lane i copies fill f0 + i, found
  // by a binary search over the lanes' exclusive offsets (one record per lane), so every store
  // instruction writes 64 consecutive 32-B records — whole lines in HBM, full-size PCIe writes when
  // the tape is a host slot's pinned buffer.
  static_assert(TILE_TAPE == 64, "one record per lane");
  {
    const uint32_t ex = (uint32_t)(incl - loc);
    for (uint32_t f0 = 0; f0 < total; f0 += 64) {
      const uint32_t f = f0 + (uint32_t)lane;
      int lo = 0;  // last lane whose exclusive offset is <= f: the record that owns fill f
#pragma unroll
      for (int step = 32; step >= 1; step >>= 1) {
        const uint32_t e = (uint32_t)__shfl((int)ex, min(lo + step, 63), 64);
        if (lo + step < 64 && e <= f) lo += step;
      }
      const uint32_t s0 = (uint32_t)__shfl((int)src[0], lo, 64);
      const uint32_t e0 = (uint32_t)__shfl((int)ex, lo, 64);
      if (f < total && base + f < cap) tape[base + f] = scratch[s0 + (f - e0)];
    }
  }
  if (t == ntiles - 1 && lane == 0) {
    *ldsg(J.tape_count) = base + total;
    atomicAdd(ldsg(G.ax.fills_acc), base + total);
    if (host) *ldsg(J.err_out) = __hip_atomic_load(ldsg(G.bk.err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Side-job wave k of side workgroup b (of nwg): its share of every bucket / clear job of group J and
// every tape job of J-2. A batch's bucket job runs on the side waves of the
// workgroups b = j (mod 8) only — one XCD under round-robin placement (speed only): every bucket of the
// batch is then written from one L2, whole lines instead of partial lines from eight XCDs.
__device__ __forceinline__ void aux_jobs(const ColdArgs& G, uint32_t b, uint32_t k, uint32_t nwg) {
  const int lane = lane_id();
  const uint32_t a = b * REG_WAVES + k, A = nwg * REG_WAVES;
  const uint32_t nb = ldsu(G.ax.nb);
  const bool xg = nwg >= 8u;
  const uint32_t x = b % 8u, ax_ = (b / 8u) * REG_WAVES + k, Ax = ((nwg - x + 7u) / 8u) * REG_WAVES;
  for (uint32_t j = 0; j < nb; ++j) {
    const AuxBucket& J = G.ax.b[j];
    const uint32_t zt = ldsu(J.zero_tiles);
    const gptr<uint32_t> z = ldsg(J.zero_tile_sum);
    for (uint32_t i = a * 64u + (uint32_t)lane; i < zt; i += A * 64u) z[i] = 0u;
    if (a == 0 && lane == 0) *ldsg(J.zero_top) = 0ull;
    if (xg && j % 8u != x) continue;
    const uint32_t wa = xg ? ax_ : a, WA = xg ? Ax : A;
    const uint32_t n = ldsu(J.n);
    const uint32_t per = (((n + WA - 1u) / WA) + 63u) & ~63u;
    const uint32_t r0 = min(n, wa * per);
    aux_bucket(G, j, r0, min(n, r0 + per));
  }
  const uint32_t nt = ldsu(G.ax.nt);
  for (uint32_t j = 0; j < nt; ++j) {
    const uint32_t tn = ldsu(G.ax.t[j].tn);
    const uint32_t ntiles = (tn + TILE_TAPE - 1) / TILE_TAPE;
    for (uint32_t t = a; t < ntiles; t += A) aux_tape_tile(G, j, t, ntiles, tn);
  }
}

// ---- launches with no match job: the side jobs alone ------------------------------------------
// The pipeline's first launch of a run (bucket only) and its last (tape only) have no matching waves to
// hide behind: in k_match_reg they ran on its 4 side waves per CU (one 145-KB workgroup per CU), 74 and
// 87 us for a 20-batch group at config 2. k_side carries only the side jobs' arguments in LDS.
//  * bucket: one workgroup per SB_REC records of a batch counts its records per symbol in LDS, then
//    reserves each symbol's run with ONE returning global atomic (device-scope atomics execute at the
//    memory side, one request each: one per record capped the fill launch at ~20 G records/s), then
//    writes the records at run + rank. A bucket's order is free (the match wave sorts by batch index).
//    Needs (S + 1) counters in LDS; above SB_SMAX symbols the waves bucket 64-record blocks with one
//    atomic per record as the pipelined launch does.
//  * tape: tiles dealt round-robin to the tape waves over a list flattened across the group's batches.
struct SideArgs {
  struct {
    uint32_t* err;
  } bk;
  AuxDev ax;
};
#ifndef ME_SIDE_THREADS
#define ME_SIDE_THREADS 512
#endif
#ifndef ME_SB_REC
#define ME_SB_REC 2048  // records per bucket workgroup: same box, config 2's driver shape 1,818-1,836M at 4,096,
                        // 1,911-1,918M at 2,048, 1,804-1,820M at 1,024; 640 steps 2,561 / 2,604 / 2,572M; config
                        // 3 1,301 / 1,317M (profiles/r4/sb) — the group's walk + resolve 549 -> 514 us
#endif
constexpr int SIDE_THREADS = ME_SIDE_THREADS;
constexpr int SIDE_WAVES = SIDE_THREADS / 64;
#ifndef ME_TAPE_XCD
#define ME_TAPE_XCD 1  // tape tiles: each half of a batch's tape on one XCD (1) or dealt over all (0); profiles/r5/tx
#endif
constexpr uint32_t SB_REC = ME_SB_REC;             // records per bucket workgroup
constexpr uint32_t SB_PER = SB_REC / SIDE_THREADS;  // records per thread
constexpr uint32_t SB_SMAX = 16383;                // symbols bucketed through an LDS histogram (64 KB)

// Units [off, off + cnt) of a list flattened over batches, dealt round-robin to waves: wave a's first.
__device__ __forceinline__ uint32_t flat_first(uint32_t off, uint32_t a, uint32_t A) {
  return off + (a + A - off % A) % A;
}

// The early fill's launch (me_engine.cpp early_fill): bucket jobs only, at most FILL_NB of them — a
// ~0.8-KB argument block instead of SideArgs' ~5.7 KB (the host's launch call is the early fill's cost:
// ~13 us per launch with SideArgs).
constexpr uint32_t FILL_NB = 8;
struct FillArgs {
  struct {
    uint32_t* err;
  } bk;
  struct {
    uint32_t S, nb;
    AuxBucket b[FILL_NB];
  } ax;
};

// Bucket records [r0, r1) of bucket job j with a workgroup histogram (cnt: S + 1 LDS counters).
template <class GA>
__device__ __forceinline__ void side_bucket_wg(const GA& G, uint32_t j, uint32_t r0, uint32_t r1, uint32_t* cnt) {
  const uint32_t tid = threadIdx.x;
  const AuxBucket& J = G.ax.b[j];
  const uint32_t S = ldsu(G.ax.S);
  const gptr<const uint32_t> sym = ldsg(J.sym);
  const gptr<const uint64_t> seq = ldsg(J.seq);
  const gptr<const int64_t> px = ldsg(J.px);
  const gptr<const int32_t> qty = ldsg(J.qty);
  const gptr<const uint8_t> kind = ldsg(J.kind);
  const gptr<uint32_t> bcnt = ldsg(J.bcnt);
  const gptr<BkRec> brec = ldsg(J.b_rec);
  const gptr<me_order_result> bres = ldsg(J.bres);
  for (uint32_t b = tid; b <= S; b += SIDE_THREADS) cnt[b] = 0u;
  {  // the tile sums of this record range, and the batch's scratch top, start at zero
    const gptr<uint32_t> z = ldsg(J.zero_tile_sum);
    const uint32_t t1 = min((r1 + TILE_TAPE - 1) / TILE_TAPE, ldsu(J.zero_tiles));
    for (uint32_t t = r0 / TILE_TAPE + tid; t < t1; t += SIDE_THREADS) z[t] = 0u;
    if (r0 == 0 && tid == 0) *ldsg(J.zero_top) = 0ull;
  }
  __syncthreads();
  uint32_t bin[SB_PER], rank[SB_PER];
  uint64_t sq[SB_PER];
  int64_t p[SB_PER];
  int32_t q[SB_PER];
  uint32_t k8[SB_PER];
  bool order_ok = true;
#pragma unroll
  for (uint32_t k = 0; k < SB_PER; ++k) {
    const uint32_t i = r0 + k * SIDE_THREADS + tid;
    bin[k] = S;
    if (i < r1) {
      bin[k] = min(sym[i], S);
      sq[k] = seq[i];
      p[k] = px[i];
      q[k] = qty[i];
      k8[k] = kind[i];
      // API precondition (the seq ring relies on it): seqs ascending through the batch (seq_follows)
      if (i > 0) order_ok &= seq_follows(seq[i - 1], sq[k], k8[k]);
    }
  }
#pragma unroll
  for (uint32_t k = 0; k < SB_PER; ++k) {
    const uint32_t i = r0 + k * SIDE_THREADS + tid;
    if (i < r1 && bin[k] == S) reject_bad_at(bres, i);  // unknown symbol: rejected here, never bucketed
    if (bin[k] < S) rank[k] = atomicAdd(&cnt[bin[k]], 1u);
  }
  if (__ballot(!order_ok) && lane_id() == 0) atomicOr(ldsg(G.bk.err), ERR_SEQ_ORDER);
  __syncthreads();
  for (uint32_t b = tid; b < S; b += SIDE_THREADS) {
    const uint32_t c = cnt[b];
    if (c) cnt[b] = atomicAdd(&bcnt[(size_t)b * BK_CNT_STRIDE], c);
  }
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < SB_PER; ++k) {
    if (bin[k] >= S) continue;
    const uint32_t r = cnt[bin[k]] + rank[k];
    if (r < (uint32_t)BK_CAP) {
      const uint32_t i = r0 + k * SIDE_THREADS + tid;
      const size_t d = (size_t)bin[k] * BK_CAP + r;
      brec[d].seq = sq[k];
      brec[d].px = p[k];
      brec[d].qty = q[k];
      brec[d].ok = i | ((k8[k] & 15u) << BK_KIND_SHIFT);
    }
  }
}

// Grid: 8 x the most units a batch has; batch j on the blocks b = j (mod 8), its units in turn (k_side's
// xseq form, one batch per XCD).
__global__ __launch_bounds__(SIDE_THREADS) void k_side_fill(FillArgs args) {
  __shared__ FillArgs G;
  extern __shared__ uint32_t side_cnt[];
  static_assert(sizeof(FillArgs) % 8 == 0, "FillArgs copy");
  for (uint32_t i = threadIdx.x; i < sizeof(FillArgs) / 8; i += SIDE_THREADS)
    reinterpret_cast<unsigned long long*>(&G)[i] = reinterpret_cast<const unsigned long long*>(&args)[i];
  __syncthreads();
  const uint32_t nb = ldsu(G.ax.nb), x = blockIdx.x % 8u, k = blockIdx.x / 8u;
  for (uint32_t j = x; j < nb; j += 8) {
    const uint32_t n = ldsu(G.ax.b[j].n), r0 = k * SB_REC;
    if (r0 >= n) continue;  // (uniform over the workgroup)
    side_bucket_wg(G, j, r0, min(n, r0 + SB_REC), side_cnt);
    __syncthreads();  // the LDS counters are zeroed again by the next batch
  }
}

// Grid: [0, nbu) bucket workgroups (histogram path; 0 on the per-record path), then tape workgroups.
__global__ __launch_bounds__(SIDE_THREADS) void k_side(SideArgs args, uint32_t nbu) {
  __shared__ SideArgs G;
  extern __shared__ uint32_t side_cnt[];
  static_assert(sizeof(SideArgs) % 8 == 0, "SideArgs copy");
  for (uint32_t i = threadIdx.x; i < sizeof(SideArgs) / 8; i += SIDE_THREADS)
    reinterpret_cast<unsigned long long*>(&G)[i] = reinterpret_cast<const unsigned long long*>(&args)[i];
  __syncthreads();
  const int lane = lane_id();
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nb = ldsu(G.ax.nb);
  if (blockIdx.x < nbu) {  // histogram bucket unit: batch j, records [u * SB_REC, ...)
    // Blocks b and b + 8 share an XCD (round-robin placement; speed only): every unit of batch j runs
    // on blocks b = j (mod 8), so the runs its workgroups write side by side into one bucket array
    // meet in one L2 and leave it as whole lines, not as partial lines from several XCDs.
    const uint32_t x = blockIdx.x % 8u, k = blockIdx.x / 8u;
    if (ldsu(G.ax.xseq)) {
      // beside a walk (off the critical path): unit k of each of the XCD's batches in turn, so one
      // batch's buckets (1.5 MB at config 2) are being filled per L2 at a time, not four batches' 6 MB
      // whose partial lines the 4-MB L2 evicts before the later units complete them (profiles/r4/xs)
      for (uint32_t j = x; j < nb; j += 8) {
        const uint32_t n = ldsu(G.ax.b[j].n), r0 = k * SB_REC;
        if (r0 >= n) continue;  // (uniform over the workgroup)
        side_bucket_wg(G, j, r0, min(n, r0 + SB_REC), side_cnt);
        __syncthreads();  // the LDS counters are zeroed again by the next batch
      }
      return;
    }
    uint32_t off = 0;
    for (uint32_t j = x; j < nb; j += 8) {
      const uint32_t n = ldsu(G.ax.b[j].n), nu = (n + SB_REC - 1) / SB_REC;
      if (k < off + nu) {
        const uint32_t r0 = (k - off) * SB_REC;
        side_bucket_wg(G, j, r0, min(n, r0 + SB_REC), side_cnt);
        return;
      }
      off += nu;
    }
    return;
  }
  const uint32_t A = (gridDim.x - nbu) * SIDE_WAVES, a = (blockIdx.x - nbu) * SIDE_WAVES + wv;
  uint32_t off = 0;
  if (nbu == 0) {  // per-record bucket path (too many symbols for the LDS histogram)
    for (uint32_t j = 0; j < nb; ++j) {
      const AuxBucket& J = G.ax.b[j];
      const uint32_t zt = ldsu(J.zero_tiles);
      const gptr<uint32_t> z = ldsg(J.zero_tile_sum);
      for (uint32_t i = a * 64u + (uint32_t)lane; i < zt; i += A * 64u) z[i] = 0u;
      if (a == 0 && lane == 0) *ldsg(J.zero_top) = 0ull;
      const uint32_t n = ldsu(J.n), nblk = (n + 63u) / 64u;
      for (uint32_t u = flat_first(off, a, A); u < off + nblk; u += A) {
        const uint32_t r0 = (u - off) * 64u;
        aux_bucket(G, j, r0, min(n, r0 + 64u));
      }
      off += nblk;
    }
  }
  const uint32_t nt = ldsu(G.ax.nt);
#if ME_TAPE_XCD
  // Each half of a batch's tape on one XCD (blocks b = x mod 8 under round-robin placement; speed only): a
  // 128-B line of a symbol's scratch slab holds fills of takers ~16 tiles apart, so the tiles that read it
  // meet in one L2 instead of fetching the line once per XCD. Halves, not batches, keep the XCDs balanced.
  if (gridDim.x - nbu >= 8u) {
    const uint32_t x = blockIdx.x % 8u;
    const uint32_t b0 = nbu + (x + 8u - nbu % 8u) % 8u;  // the first tape block on XCD x
    const uint32_t AX = ((gridDim.x - b0 + 7u) / 8u) * SIDE_WAVES, ax = ((blockIdx.x - b0) / 8u) * SIDE_WAVES + wv;
    for (uint32_t v = x; v < 2u * nt; v += 8u) {
      const uint32_t j = v >> 1, h = v & 1u;
      const uint32_t tn = ldsu(G.ax.t[j].tn);
      const uint32_t ntiles = (tn + TILE_TAPE - 1) / TILE_TAPE, half = (ntiles + 1u) / 2u;
      const uint32_t t0 = h * half, t1 = min(ntiles, t0 + half);
      for (uint32_t t = t0 + ax; t < t1; t += AX) aux_tape_tile(G, j, t, ntiles, tn);
    }
    return;
  }
#endif
  off = 0;
  for (uint32_t j = 0; j < nt; ++j) {
    const uint32_t tn = ldsu(G.ax.t[j].tn);
    const uint32_t ntiles = (tn + TILE_TAPE - 1) / TILE_TAPE;
    for (uint32_t u = flat_first(off, a, A); u < off + ntiles; u += A) aux_tape_tile(G, j, u - off, ntiles, tn);
    off += ntiles;
  }
}

// ---- the kernel ----------------------------------------------------------------------------
// Per-record control word built in vector form: (window limit level + 1) | BUY | MARKET | CANCEL |
// FAR (the limit reaches past the window on the side the taker crosses: MARKET, a BUY above the
// window, a SELL below it) | OUT (a LIMIT priced outside the window: its rest takes the far path).
// HAND (common launch only): the record needs a far level — OUT, or a MARKET while the side it crosses
// has far levels (far counts only change in the continuation launch, so they are fixed per launch).
constexpr uint32_t CW_BUY = 1u << 8, CW_MKT = 1u << 9, CW_CXL = 1u << 10, CW_FAR = 1u << 11, CW_OUT = 1u << 12,
                   CW_HAND = 1u << 13;

// far: bit 0 = the symbol has far bids (side 0), bit 1 = far asks (side 1)
__device__ __forceinline__ uint32_t make_cw(long long opx, uint32_t kd, long long base, uint32_t L, uint32_t far_nz) {
  const uint32_t side = kd & 3u;
  const bool market = (kd >> 2) & 1u, cancel = (kd >> 3) & 1u;
  const bool buy = side == ME_SIDE_BUY;
  const unsigned long long off = (unsigned long long)opx - (unsigned long long)base;
  const bool inw = off < (unsigned long long)L;
  const bool above = !inw && opx > base;
  // the last window level the taker may trade at, -1 .. L (none below / above the window)
  const int lim = market ? (buy ? (int)L - 1 : 0)
                : inw    ? (int)off
                : buy    ? (above ? (int)L - 1 : -1)
                         : (above ? (int)L : 0);
  // a CANCEL's price field is its target seq: none of the window / far tests apply to it
  const bool far = !cancel && (market || (buy ? above : (!inw && !above)));
  const bool out = !market && !cancel && !inw;
  const bool hand = out || (market && ((far_nz >> (buy ? 1 : 0)) & 1u));
  return (uint32_t)(lim + 1) | (buy ? CW_BUY : 0u) | (market ? CW_MKT : 0u) | (cancel ? CW_CXL : 0u) |
         (far ? CW_FAR : 0u) | (out ? CW_OUT : 0u) | (hand ? CW_HAND : 0u);
}

// One wavefront per symbol. kSlow = false: the common launch — every symbol of the group, no far-level
// code at all (it cost the serial loop 19-27 % through register allocation even when never run,
// DESIGN.md §8): a record that needs a far level (a LIMIT priced outside the window, a MARKET while the
// opposite side has far levels, a cancel of a far or old order) hands its symbol off before it changes
// anything. kSlow = true: the continuation launch right after it — the handed-off symbols only, from
// their hand-off record to the end of the group, with the far-level code inline.
template <bool kSlow>
__global__ __launch_bounds__(128 * REG_WAVES) void k_match_reg(ColdArgs args) {
  __shared__ RegLds lds[REG_WAVES];
  __shared__ ColdArgs G;
  static_assert(sizeof(ColdArgs) % 8 == 0, "ColdArgs copy");
  const BookDev& bk = args.bk;
  uint32_t nhand = 0;
  if constexpr (kSlow) {  // nothing handed off (the usual case): leave before the argument copy
    nhand = min(*(volatile uint32_t*)bk.hcount, bk.S);
    if (blockIdx.x * REG_WAVES >= nhand) return;
    if (blockIdx.x == 0 && threadIdx.x == 0 && bk.stats) {
      const unsigned long long h = atomicAdd(bk.stats + ST_HANDOFFS, (unsigned long long)nhand) + nhand;
      // published at once (k_seq_sweep would publish it only ahead of the launch after next): the
      // engine's grouped-aggregate policy sees this group's hand-offs before it launches the next group
      if (bk.pub)
        bk.pub[1] = ((bk.stats[ST_LAUNCH] + 1ull) << 32) | (h < 0xFFFFFFFFull ? h : 0xFFFFFFFFull);
    }
  }
  {
    for (uint32_t i = threadIdx.x; i < sizeof(ColdArgs) / 8; i += 128 * REG_WAVES)
      reinterpret_cast<unsigned long long*>(&G)[i] = reinterpret_cast<const unsigned long long*>(&args)[i];
    __syncthreads();
  }
  const int lane = lane_id();
  // wave index: readfirstlane tells the divergence analysis it is wave-uniform (threadIdx.x >> 6 is
  // not recognised as such), so every per-symbol value and branch below is scalar
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wv >= (uint32_t)REG_WAVES) {  // side-job wave (only in the workgroups of the first dispatch round)
    const uint32_t k = wv - REG_WAVES, nwg = max(min(args.ax.nwg, gridDim.x), 1u);
    if (!kSlow && blockIdx.x < nwg) aux_jobs(G, blockIdx.x, k, nwg);
    return;
  }
#ifndef ME_NO_SETPRIO
  // the serial record loop outranks the side jobs sharing its SIMD at the issue arbiter (the side
  // jobs are latency work with slack until the next launch)
  __builtin_amdgcn_s_setprio(3);
#endif
  const uint32_t ng = args.ng;
  if (ng == 0u) return;  // no match job in this launch
  // kSlow: hand-off entries wv, wv + REG_WAVES * gridDim.x, ... of this workgroup's share
  for (uint32_t hi_ = blockIdx.x * REG_WAVES + wv; !kSlow || hi_ < nhand; hi_ += REG_WAVES * gridDim.x) {
  Handoff ho{};
  uint32_t s;
  if constexpr (kSlow) {
    ho = bk.hand[hi_];
    s = rl32(ho.s, 0);
    ho.g = rl32(ho.g, 0);
    ho.pos = rl32(ho.pos, 0);
    ho.nsg = rl32(ho.nsg, 0);
    ho.wptr = rl32(ho.wptr, 0);
    ho.wend = rl32(ho.wend, 0);
  } else {
    s = blockIdx.x * REG_WAVES + wv;
    if (s > bk.S) return;  // no symbol
  }
#ifdef ME_STAMPS
  unsigned long long st_t0 = stamp_now();
#endif
  const bool bucketed = args.bt[0].bcnt != nullptr;
  const uint32_t L = bk.L;
  const uint32_t sl = s < bk.S ? s : bk.S - 1u;  // the bad-symbol wave's ladder loads are discarded
  // ---- one round trip: the symbol's record count in every batch of the group, ladder rows, tail
  // fills, symbol scalars, parked free chunks (no predicated loads: row 1 of a 64-level ladder
  // re-reads row 0 and is then discarded)
  uint32_t lo = 0, nsv = 0, ns;
  if (bucketed) {  // lane g < ng: the symbol's count in batch g
    const uint32_t gl = min((uint32_t)lane, ng - 1u);
    const uint32_t* cp = G.bt[gl].bcnt;
    nsv = (uint32_t)lane < ng ? cp[(size_t)s * BK_CNT_STRIDE] : 0u;
    if constexpr (kSlow) {  // batches before the hand-off are done; its own counter is already reset
      nsv = (uint32_t)lane < ho.g ? 0u : ((uint32_t)lane == ho.g ? ho.nsg : nsv);
    }
    ns = 0;
  } else if (args.bt[0].bin_start) {  // single-pass sort: the run table
    lo = args.bt[0].bin_start[s];
    ns = args.bt[0].bin_start[s + 1] - lo;
  } else {
    lo = wave_lower_bound(args.bt[0].skeys, args.bt[0].n, s);
    ns = wave_lower_bound(args.bt[0].skeys, args.bt[0].n, s + 1) - lo;
  }
  const Level* p_lv = bk.levels + (size_t)sl * L;
  const uint8_t* p_tend = bk.tend + (size_t)sl * L;
  const bool in1 = 64u + (uint32_t)lane < L;
  const uint32_t l1 = in1 ? 64u + (uint32_t)lane : (uint32_t)lane;
  const Level a = p_lv[lane];
  const Level b = p_lv[l1];
  const uint32_t te0 = p_tend[lane];
  const uint32_t te1 = p_tend[l1];
  const SymState st = bk.sym[sl];
  const uint32_t fst = bk.fcache[(size_t)sl * FSTK + lane];
  const uint32_t gsv = bk.gsym[sl];
  if (bucketed) {
    // the symbol's records over every batch of the group: lanes 0 .. ng-1 (up to ME_GMAX = 64) hold
    // the per-batch counts. (An 8-lane sum here once dropped batches 8+ of a group: a continuation
    // whose hand-off came in batch 8 or later saw 0 records and left them unmatched —
    // test_long_drift_soak.)
    long long t = (long long)nsv;
    for (int d = 1; d < 64; d <<= 1) t += __shfl_xor(t, d, 64);
    ns = (uint32_t)rli64(t, 0);
  }
  if (ns == 0u) {
    if constexpr (kSlow) continue;
    else return;
  }
  if (!kSlow && s == bk.S) {  // the sort path's bad-symbol bin (bucketed batches carry none)
    reject_bad_run(G, lo, lo + ns);
    return;
  }
  RegCtx c;
  c.chunks = vptr(bk.chunks);
  c.loc = vptr(bk.loc);
  c.rmask = vreg64(bk.ring_mask);
  c.G = &G;
  c.M = &lds[wv];
  c.nchunks = bk.nchunks;
  c.s = s;
  c.gs = vreg(gsv);
#ifdef ME_STAMPS
  for (int p = 0; p < PH_N; ++p) c.st[p] = 0;
  c.st_t = st_t0;
  STAMP_ADD(c, PH_SW_WINDOW);  // run bounds
#endif
  c.hd.r0 = a.head | HC;  // nothing cached yet (NIL stays NIL)
  c.hd.r1 = in1 ? (b.head | HC) : NIL;
  c.tl.r0 = a.tail;
  c.tl.r1 = in1 ? b.tail : NIL;
  c.te.r0 = te0;
  c.te.r1 = in1 ? te1 : 0u;
  const long long tb = in1 ? b.total : 0ll;
  c.M->tot[lane] = a.total;
  c.M->tot[64 + lane] = tb;
  c.occ.w0 = __ballot(a.total > 0);
  c.occ.w1 = __ballot(tb > 0);
  c.base = (long long)vreg64((unsigned long long)st.base);
  c.bb = rli32(st.best_bid, 0);
  c.ba = rli32(st.best_ask, 0);
  if (c.ba > RL) c.ba = RL;
  {
    const SeqState sqs = bk.sq[bk.sq_idx];
    if (lane == 0) {
      c.M->free_head = st.free_head;
      c.M->resting0 = st.resting;
      c.M->bump_cur = 0;
      c.M->bump_end = 0;
      c.M->nfar[0] = st.nfar[0];
      c.M->nfar[1] = st.nfar[1];
      c.M->horizon = sqs.horizon;
      c.M->epoch = sqs.epoch;
    }
  }
  c.nfs = min(rl32(st.nfree, 0), (uint32_t)FSTK);
  c.fstk = fst;
  c.resting = (int)rl32(st.resting, 0);
  c.wptr = 0;
  c.wend = 0;
  c.recs_left = ns;
  // ---- the batches of the group, in stream order; the book stays on chip between them
  ldsw(c.M->g_next, kSlow ? ho.g : 0u);
  ldsw(c.M->run_lo, lo);  // the sort path's run (one batch)
  ldsw(c.M->run_n, ns);
  for (;;) {  // the batch cursor lives in LDS: no SGPR of it is live across the serial loop
    const uint32_t g = ldsu(c.M->g_next);
    if (g >= ldsu(G.ng)) break;
    ldsw(c.M->g_next, g + 1u);
    ldsw(c.M->g_cur, g);
    uint32_t nsg = ldsu(c.M->run_n);
    uint32_t k0 = ~0u, k1 = ~0u;
    uint32_t mode = 2u;  // 0: bucket, 1: rescan, 2: sort path (perm)
    if (ldsu(G.bt[0].bcnt) != nullptr) {
      nsg = rl32(nsv, (int)g);
      if (nsg == 0u) continue;
      const BatchDev& B = G.bt[g];
      const size_t bb = (size_t)s * BK_CAP;
      const gptr<const BkRec> prec = ldsg(B.b_rec);
      const unsigned long long bq0 = prec[bb + lane].seq, bq1 = prec[bb + 64 + lane].seq;
      const long long bp0 = prec[bb + lane].px, bp1 = prec[bb + 64 + lane].px;
      const int bn0 = prec[bb + lane].qty, bn1 = prec[bb + 64 + lane].qty;
      const uint32_t bo0 = prec[bb + lane].ok, bo1 = prec[bb + 64 + lane].ok;
      if (lane == 0) ldsg(B.bcnt)[(size_t)s * BK_CNT_STRIDE] = 0u;  // ready for a later group's bucket job
      // ---- batch order. A bucket (<= BK_CAP records, arbitrary order) is staged in LDS and its keys
      // (batch index << 7 | bucket slot) sorted across the wave; an overfull bucket is replaced by a
      // rescan of the batch (RSW-record windows, batch order by construction).
      mode = nsg <= (uint32_t)BK_CAP ? 0u : 1u;
      if (mode == 0u) {
        c.M->in.b.seq[lane] = bq0;
        c.M->in.b.seq[64 + lane] = bq1;
        c.M->in.b.px[lane] = bp0;
        c.M->in.b.px[64 + lane] = bp1;
        c.M->in.b.qty[lane] = bn0;
        c.M->in.b.qty[64 + lane] = bn1;
        c.M->in.b.ok[lane] = bo0;
        c.M->in.b.ok[64 + lane] = bo1;
        k0 = (uint32_t)lane < nsg ? ((bo0 & BK_IDX_MASK) << 7) | (uint32_t)lane : ~0u;
        k1 = 64u + (uint32_t)lane < nsg ? ((bo1 & BK_IDX_MASK) << 7) | (64u + (uint32_t)lane) : ~0u;
        if (nsg > 64u)
          sort128(k0, k1);
        else
          k0 = sort64(k0, false);
      }
    }
    c.scratch = vptr(ldsu(G.bt[g].scratch));
    c.wptr = s * ldsu(G.bt[g].slab);
    c.wend = c.wptr + ldsu(G.bt[g].slab);
    uint32_t skip = 0;  // (continuation) records of the hand-off batch the common launch finished
    if constexpr (kSlow) {
      if (g == ho.g) {
        skip = ho.pos;
        c.wptr = ho.wptr;
        c.wend = ho.wend;
      }
    }
    c.recs_left = nsg - skip;
    if (lane == 0) {  // read back where used: nothing of this holds an SGPR across the serial loop
      c.M->mode = mode;
      c.M->scan_cur = 0;
      c.M->scan_cnt = 0;
      c.M->scan_pos = 0;
    }
    STAMP_ADD(c, PH_PROLOGUE);
    // left: records of the symbol not yet visited (its count; the rescan keeps its own cursors)
    for (uint32_t left = nsg;;) {
      // ---- up to 64 records in vector form, batch order
      uint32_t oi, cnt;
      unsigned long long oseq_;
      long long opx_;
      int oq_;
      uint32_t kd_;
      const uint32_t md = ldsu(c.M->mode);
      if (md == 0u) {
        if (left == 0u) break;
        cnt = min(64u, left);
        const uint32_t pos = k0 & (BK_CAP - 1);  // past the count: key ~0, slot 127 (discarded)
        oi = k0 >> 7;
        k0 = k1;  // the second block, if any
        oseq_ = c.M->in.b.seq[pos];
        opx_ = c.M->in.b.px[pos];
        oq_ = c.M->in.b.qty[pos];
        kd_ = c.M->in.b.ok[pos] >> BK_KIND_SHIFT;
      } else {
        if (md == 1u) {
          if (ldsu(c.M->scan_pos) >= ldsu(c.M->scan_cnt) && !rescan_window(c.M, G, ldsu(c.M->g_cur), s)) break;
          const uint32_t p0 = ldsu(c.M->scan_pos), lc = ldsu(c.M->scan_cnt);
          cnt = min(64u, lc - p0);
          oi = c.M->in.lst[p0 + min((uint32_t)lane, cnt - 1u)];
          ldsw(c.M->scan_pos, p0 + cnt);
        } else {
          if (left == 0u) break;
          cnt = min(64u, left);
          const uint32_t at = ldsu(c.M->run_lo) + (ldsu(c.M->run_n) - left);
          oi = ldsg(G.bt[0].perm)[at + min((uint32_t)lane, cnt - 1u)];  // clamp: never branch around a load
        }
        const BatchDev& B = G.bt[ldsu(c.M->g_cur)];
        oseq_ = ldsg(B.seq)[oi];
        opx_ = ldsg(B.px)[oi];
        oq_ = ldsg(B.qty)[oi];
        kd_ = ldsg(B.kind)[oi];
      }
      const uint32_t j = (uint32_t)lane;  // record j of the block
      const uint32_t hi = cnt;
      const uint32_t vis = nsg - left;    // records of the batch before this block
      // validation in vector form; only the packed control word and the reject code stay live
      uint32_t cw, rj;
      {
        const bool v = j < hi && (!kSlow || vis + j >= skip);
        const unsigned long long oseq = v ? oseq_ : 0ull;
        const int oq = v ? oq_ : 0;
        const uint32_t kd = v ? kd_ : 0u;
        const uint32_t side = kd & 3u;
        const bool cancel = (kd >> 3) & 1u;
        rj = ME_RJ_NONE;
        if (!cancel) {
          if (oq <= 0)
            rj = ME_RJ_BAD_QTY;
          else if (side != ME_SIDE_BUY && side != ME_SIDE_SELL)
            rj = ME_RJ_BAD_SIDE;
          else if (oseq == 0ull)
            rj = ME_RJ_BAD_SEQ;  // no OID is 0 (the counter starts at 1, storage.cpp:254-267)
        }
        const uint32_t fnz = kSlow ? 0u : ((ldsu(c.M->nfar[0]) != 0u) | ((ldsu(c.M->nfar[1]) != 0u) << 1));
        cw = make_cw(v ? opx_ : 0ll, kd, c.base, L, fnz);
        if (!v) rj = 0xFFu;  // lanes past the run (or before the continuation point): no record
      }
      unsigned long long work = __ballot(rj == ME_RJ_NONE);
      // cancels: every target's ring entry in one gather at the block start, so that a cancel's chunk read
      // is its only round trip on the chain (the ring load in reg_cancel was the other; reg_cancel verifies
      // the slot a hint names). No wait here: a block-start vmcnt(0) also waits for the stores of the block
      // before (measured slower: 1,003 -> 990M on config 5, profiles/r5/cx)
      const unsigned long long cxm = __ballot(rj == ME_RJ_NONE && (cw & CW_CXL));
      uint32_t gpre = NIL;
      if (cxm && ((cxm >> lane) & 1ull)) gpre = c.loc[(unsigned long long)opx_ & c.rmask];
      uint32_t stop = cnt;  // records [0, stop) of the block get results
      bool handoff = false;
      if constexpr (!kSlow) {  // from the first record that needs a far level on: the continuation's
        const unsigned long long hm = __ballot(rj == ME_RJ_NONE && (cw & CW_HAND));
        if (ME_UNLIKELY(hm != 0ull)) {
          const int h = __builtin_ctzll(hm);
          work &= (1ull << h) - 1ull;
          stop = (uint32_t)h;
          handoff = true;
        }
      }
      uint32_t out_q = 0, out_n = 0, out_w = 0;
  #ifdef ME_STAMPS
      __builtin_amdgcn_s_waitcnt(0);
  #endif
      STAMP_ADD(c, PH_FETCH);
      // ---- the serial chain: records that touch the book, in seq order
      while (work) {
        const int k = __builtin_ctzll(work);
        work &= work - 1ull;
        const uint32_t ctl = rl32(cw, k);
        c.recs_left = left - (uint32_t)k;
        uint32_t outq;
        COUNT(c, CT_FAST);
        STAMP_ADD(c, PH_SWEEP);
        if (ME_UNLIKELY(ctl & CW_CXL)) {
          const unsigned long long tgt = (unsigned long long)rli64(opx_, k);
          // (a target an earlier record of this block rested as: its block-start ring entry is stale)
          const bool inblk = __ballot(lane < k && oseq_ == tgt) != 0ull;
          outq = reg_cancel<kSlow>(c, tgt, inblk ? NIL : rl32(gpre, k));
          if (!kSlow && ME_UNLIKELY(outq == HANDOFF)) {
            stop = (uint32_t)k;
            handoff = true;
            break;
          }
          STAMP_ADD(c, PH_CANCEL);
        } else {
          const bool buy = (ctl & CW_BUY) != 0u;
          if (ME_UNLIKELY(c.wptr + (uint32_t)c.resting > c.wend) && !reg_reserve_overflow(c)) {
            stop = (uint32_t)k;
            handoff = false;
            break;
          }
          const unsigned long long seq = rl64(oseq_, k);
          const uint32_t q = (uint32_t)rli32(oq_, k);
          const int lm = (int)(ctl & 0xFFu) - 1;
          const uint32_t w_in = c.wptr;
          uint32_t rem = q;
          // one walk loop for both sides (one copy of the walk): the opposite best moves away from
          // the taker's limit as levels empty
          int lvl = buy ? c.ba : c.bb;
          for (;;) {
            const int gap = buy ? lm - lvl : lvl - lm;  // >= 0: the level crosses the limit (int select, scalar)
            if (rem == 0u || gap < 0) break;
            if (ME_LIKELY(!reg_walk(c, lvl, rem, seq))) break;
            lvl = buy ? c.occ.next(lvl + 1) : c.occ.prev(lvl - 1);
          }
          if (buy)
            c.ba = lvl;
          else
            c.bb = lvl;
          int rr = 0;
          if constexpr (kSlow) {
            // the window side is exhausted and the limit reaches further: far levels
            if (rem != 0u && (ctl & CW_FAR) && c.fcount(buy ? 1u : 0u) != 0u)
              rem -= far_take(c, buy, (ctl & CW_MKT) != 0u, (long long)rl64((unsigned long long)opx_, k), rem, seq);
            // a LIMIT priced outside the window rests through the far path (may re-centre the window)
            if ((ctl & CW_OUT) && rem != 0u)
              rr = reg_far_rest(c, (long long)rl64((unsigned long long)opx_, k), seq, rem, buy) < 0 ? -1 : 1;
          }
          outq = q - rem;
          STAMP_ADD(c, PH_WALK);
          const bool me_ = lane == k;
          out_n = me_ ? c.wptr - w_in : out_n;
          out_w = me_ ? w_in : out_w;
          if (kSlow && rr != 0) {
            if (rr < 0) {
              stop = (uint32_t)k;
              handoff = false;
              break;
            }
            const bool v = j < hi && vis + j >= skip;
            cw = make_cw(v ? opx_ : 0ll, v ? kd_ : 0u, c.base, L, 0u);  // the window may have moved
          } else if (!(ctl & (CW_MKT | CW_OUT)) && rem != 0u && ME_UNLIKELY(!reg_rest(c, lm, seq, rem, buy))) {
            stop = (uint32_t)k;  // chunk pool exhausted: the batch fails (sticky error word)
            handoff = false;
            break;
          }
          STAMP_ADD(c, PH_REST);
        }
        out_q = lane == k ? outq : out_q;
      }
      // ---- results of the block in vector form
      me_order_result* res = ldsg(G.bt[ldsu(c.M->g_cur)].res);
      uint32_t* fstart = ldsg(G.bt[ldsu(c.M->g_cur)].fstart);
      const bool sortp = ldsu(G.bt[0].bcnt) == nullptr;
      uint32_t* tile_sum = ldsg(G.bt[ldsu(c.M->g_cur)].tile_sum);
      if (rj != 0xFFu && (uint32_t)lane < stop) {
        const bool market = (kd_ >> 2) & 1u, cancel = (kd_ >> 3) & 1u;
        me_order_result r;
        r.tape_offset = out_w;  // scratch start until the tape job writes the tape offset
        r.pad[0] = r.pad[1] = 0;
        r.fill_count = out_n;
        r.reason = (uint8_t)rj;
        if (rj != ME_RJ_NONE) {
          r.filled_qty = 0;
          r.remaining_qty = rj == ME_RJ_BAD_QTY ? 0 : oq_;
          r.status = ME_ST_REJECTED;
        } else if (cancel) {
          r.filled_qty = 0;
          r.remaining_qty = (int)out_q;
          r.status = out_q ? ME_ST_CANCELED : ME_ST_REJECTED;
          r.reason = out_q ? ME_RJ_NONE : ME_RJ_UNKNOWN_ORDER;
        } else {
          const int rem = oq_ - (int)out_q;
          r.filled_qty = (int)out_q;
          r.remaining_qty = rem;
          r.status = rem == 0 ? ME_ST_FILLED
                   : market   ? ME_ST_CANCELED
                   : out_q    ? ME_ST_PARTIALLY_FILLED
                              : ME_ST_NEW;
        }
        res[oi] = r;
        if (sortp) fstart[oi] = out_w;  // k_tape_compact (sort path) reads the fill starts array
        if (out_n) atomicAdd(&tile_sum[oi / TILE_TAPE], out_n);
      }
      STAMP_ADD(c, PH_RESULT);
      if (!kSlow && handoff) {  // the rest of the symbol's records go to the continuation launch
        uint32_t idx = 0;
        if (lane == 0) idx = atomicAdd(ldsg(G.bk.hcount), 1u);
        idx = rl32(idx, 0);
        if (lane == 0) {
          Handoff h;
          h.s = s;
          h.g = ldsu(c.M->g_cur);
          h.pos = vis + stop;
          h.nsg = nsg;
          h.wptr = c.wptr;
          h.wend = c.wend;
          h.pad[0] = h.pad[1] = 0;
          ldsg(G.bk.hand)[idx] = h;
        }
      }
      left -= cnt;
      if (stop < cnt) {  // hand-off, or a capacity failure (the sticky error word fails the launch)
        ldsw(c.M->g_next, ME_GMAX);
        break;
      }
    }
  }
  // ---- write the symbol back
  {  // unused reserved chunks
    uint32_t cur = ldsu(c.M->bump_cur);
    const uint32_t end = ldsu(c.M->bump_end);
    while (cur < end) reg_free(c, cur++);
  }
  for (int row = 0; row < 2; ++row) {  // every valid cached head back to HBM (entry l holds the head of l)
    unsigned long long d = __ballot(((row ? c.hd.r1 : c.hd.r0) & HC) == 0u);  // cached heads
    while (d) {
      const int jj = __builtin_ctzll(d);
      d &= d - 1ull;
      const uint32_t cid = rl32(row ? c.hd.r1 : c.hd.r0, jj);
      const int e = ce(row * 64 + jj);
      if (lane < ME_C) {
        c.chunks[cid].qty[lane] = c.M->cq[e][lane];
        c.chunks[cid].seq[lane] = c.M->cs[e][lane];
      }
    }
  }
  Level* g_lv = ldsg(G.bk.levels) + (size_t)s * L;
  uint8_t* g_tend = ldsg(G.bk.tend) + (size_t)s * L;
  Level o;
  o.total = c.M->tot[lane];
  o.head = c.hd.r0 == NIL ? NIL : (c.hd.r0 & ~HC);
  o.tail = c.tl.r0;
  g_lv[lane] = o;
  g_tend[lane] = (uint8_t)c.te.r0;
  if (in1) {
    o.total = c.M->tot[64 + lane];
    o.head = c.hd.r1 == NIL ? NIL : (c.hd.r1 & ~HC);
    o.tail = c.tl.r1;
    g_lv[64 + lane] = o;
    g_tend[64 + lane] = (uint8_t)c.te.r1;
  }
  ldsg(G.bk.fcache)[(size_t)s * FSTK + lane] = c.fstk;
  const uint32_t Lwords = ldsu(G.bk.Lwords);
  unsigned long long* g_occ = ldsg(G.bk.occ) + (size_t)s * Lwords;  // for the host-side book dump
  const uint32_t fh = ldsu(c.M->free_head);
  const uint32_t nf0 = c.fcount(0), nf1 = c.fcount(1);
  if (lane == 0) {
    g_occ[0] = c.occ.w0;
    if (Lwords > 1) g_occ[1] = c.occ.w1;
    SymState so;
    so.base = c.base;
    so.best_bid = c.bb;
    so.best_ask = c.ba >= (int)L ? (int)L : c.ba;
    so.free_head = fh;
    so.resting = (uint32_t)c.resting;
    so.nfree = c.nfs;
    so.nfar[0] = nf0;
    so.nfar[1] = nf1;
    for (int k = 0; k < 5; ++k) so.pad[k] = 0;
    ldsg(G.bk.sym)[s] = so;
    const long long d = (long long)(uint32_t)c.resting - (long long)c.M->resting0;
    if (d) atomicAdd(ldsg(G.bk.stats) + ST_RESTING, (unsigned long long)d);
  }
#ifdef ME_STAMPS
  __builtin_amdgcn_s_waitcnt(0);
  STAMP_ADD(c, PH_EPILOGUE);
  unsigned long long* dbg = ldsg(G.bk.dbg);
  if (lane == 0 && dbg)
    for (int p = 0; p < PH_N; ++p) dbg[(size_t)s * 24 + p] = c.st[p];
#endif
  if constexpr (!kSlow) break;
  }
}

// One launch: the match job of bt[0, ng) (ng == 0: none) on S / REG_WAVES workgroups (S + 1 for the
// sort path's bad-symbol bin) and the side jobs of ax on the first dispatch round's extra waves; then,
// when it matched anything, the continuation launch over the symbols it handed off (one wave per
// symbol, like the common launch; workgroups with nothing to do leave at once). ev0 / ev1 bracket both.
// The early fill (bucket jobs of at most FILL_NB batches, symbols within the LDS histogram); false: not
// this launch's shape (the caller uses launch_match_reg's side launch).
hipError_t launch_fill_early(hipStream_t st, const BookDev& bk, const AuxDev& ax, bool& done) {
  done = false;
  if (ax.nb == 0 || ax.nb > FILL_NB || ax.S > SB_SMAX || ax.nt) return hipSuccess;
  FillArgs FA{};
  FA.bk.err = bk.err;
  FA.ax.S = ax.S;
  FA.ax.nb = ax.nb;
  uint32_t per = 0;
  for (uint32_t j = 0; j < ax.nb; ++j) {
    FA.ax.b[j] = ax.b[j];
    per = max(per, (ax.b[j].n + SB_REC - 1) / SB_REC);
  }
  hipLaunchKernelGGL(k_side_fill, dim3(8u * max(per, 1u)), dim3(SIDE_THREADS), (size_t)(ax.S + 1) * sizeof(uint32_t),
                     st, FA);
  done = true;
  return hipGetLastError();
}

hipError_t launch_match_reg(hipStream_t st, const BookDev& bk, const BatchDev* bt, uint32_t ng, const AuxDev& ax,
                            hipEvent_t ev0, hipEvent_t ev1) {
  if (bk.L > (uint32_t)RL || bk.L < 64u || !bk.fcache || !bk.gsym || !bk.hand || !bk.hcount)
    return hipErrorInvalidValue;
  if (ng > (uint32_t)ME_GMAX || ax.nb > (uint32_t)ME_GMAX || ax.nt > (uint32_t)ME_GMAX) return hipErrorInvalidValue;
  ColdArgs A{};
  A.bk = bk;
  A.ax = ax;
  A.ng = ng;
  for (uint32_t g = 0; g < ng; ++g) {
    // the group's batches are all bucketed, or it is one sort-path batch
    if (bt[g].n == 0u || (g > 0 && (!bt[g].bcnt || !bt[0].bcnt))) return hipErrorInvalidValue;
    A.bt[g] = bt[g];
  }
  // bucketed batches carry no bad-symbol bin (the bucket job rejects those records)
  const uint32_t waves = ng && A.bt[0].bcnt ? bk.S : bk.S + 1;
  const uint32_t match_wgs = ng ? (waves + REG_WAVES - 1) / REG_WAVES : 0u;
  uint32_t nbr = 0, ntr = 0;
  for (uint32_t j = 0; j < ax.nb; ++j) nbr += ax.b[j].n;
  for (uint32_t j = 0; j < ax.nt; ++j) ntr += ax.t[j].tn;
  if (!ng) {  // side jobs only (the pipeline's fill and drain): k_side, all waves on them
    SideArgs SA{};
    SA.bk.err = bk.err;
    SA.ax = ax;
    const bool hist = ax.S <= SB_SMAX;
    uint32_t nbu = 0;
    if (hist) {  // 8 x the most units any XCD's batches have (batch j on blocks = j mod 8)
      uint32_t per[8] = {};
      for (uint32_t j = 0; j < ax.nb; ++j) {
        const uint32_t nu = (ax.b[j].n + SB_REC - 1) / SB_REC;
        per[j % 8] = ax.xseq ? max(per[j % 8], nu) : per[j % 8] + nu;  // xseq: the batches in turn
      }
      for (uint32_t x = 0; x < 8; ++x) nbu = max(nbu, 8u * per[x]);
    }
    // the waves after the bucket workgroups: tape tiles (and per-record bucket blocks without hist)
    const uint32_t units = max(hist ? 0u : (nbr + 63u) / 64u, (ntr + TILE_TAPE - 1) / TILE_TAPE);
    const uint32_t twg = min((units + SIDE_WAVES - 1) / SIDE_WAVES, max(ax.nwg, 1u) * 4u);
    const uint32_t sgrid = max(nbu + twg, 1u);
    const size_t lds = hist ? (size_t)(ax.S + 1) * sizeof(uint32_t) : 0;
    hipExtLaunchKernelGGL(k_side, dim3(sgrid), dim3(SIDE_THREADS), lds, st, ev0, ev1, 0, SA, nbu);
    return hipGetLastError();
  }
  const uint32_t aux_wgs = min((max(nbr, ntr) + 256u * REG_WAVES - 1) / (256u * REG_WAVES), max(ax.nwg, 1u));
  const uint32_t grid = max(max(match_wgs, aux_wgs), 1u);
  hipExtLaunchKernelGGL(k_match_reg<false>, dim3(grid), dim3(128 * REG_WAVES), 0, st, ev0, ng ? nullptr : ev1, 0, A);
  if (ng) {
    A.ax = AuxDev{};
    // one wave per possible hand-off: workgroups past the hand-off count leave before the argument copy
    hipExtLaunchKernelGGL(k_match_reg<true>, dim3(match_wgs), dim3(128 * REG_WAVES), 0, st, nullptr, ev1, 0, A);
  }
  return hipGetLastError();
}

// The continuation launch alone (grouped launches through the aggregate path, me_agg.hip: the walk
// handed its symbols off into bk.hand / hcount[0] exactly as the common launch does).
hipError_t launch_match_reg_cont(hipStream_t st, const BookDev& bk, const BatchDev* bt, uint32_t ng, hipEvent_t ev1) {
  if (!ng || ng > (uint32_t)ME_GMAX || bk.L > (uint32_t)RL) return hipErrorInvalidValue;
  ColdArgs A{};
  A.bk = bk;
  A.ng = ng;
  for (uint32_t g = 0; g < ng; ++g) A.bt[g] = bt[g];
  const uint32_t match_wgs = (bk.S + REG_WAVES - 1) / REG_WAVES;
  hipExtLaunchKernelGGL(k_match_reg<true>, dim3(match_wgs), dim3(128 * REG_WAVES), 0, st, nullptr, ev1, 0, A);
  return hipGetLastError();
}

}  // namespace ME_REG_VARIANT
}  // namespace me

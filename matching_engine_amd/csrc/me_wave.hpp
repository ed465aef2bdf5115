// me_wave.hpp — wavefront (64-lane) helpers shared by the gfx950 kernels: lane reads, DPP
// scans, the wave-wide lower bound over the grouped symbol keys, and the diagnostic stamps.
#pragma once
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
// Inclusive scan of a 16-lane row (each DPP row scans on its own), saturating at 2^32 - 1. The row
// shifts use bound_ctrl (a lane with no source reads 0), so no "old" value is materialised.
template <int kCtrl>
__device__ __forceinline__ uint32_t shr_row(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kCtrl, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t scan16_sat(uint32_t x) {
  x = __builtin_elementwise_add_sat(x, shr_row<0x111>(x));  // row_shr:1
  x = __builtin_elementwise_add_sat(x, shr_row<0x112>(x));  // row_shr:2
  x = __builtin_elementwise_add_sat(x, shr_row<0x114>(x));  // row_shr:4
  x = __builtin_elementwise_add_sat(x, shr_row<0x118>(x));  // row_shr:8
  return x;
}

// v of lane (lane ^ J), with no LDS round trip (a ds_bpermute is a ~50-cycle dependent LDS access):
// DPP inside a 16-lane row — quad_perm for 1 and 2, row_ror:8 for 8, two row rotations and a select for
// 4 — and gfx950's permlane swaps across rows for 16 and 32 (the swap of a register with itself hands
// each half the other's values in one of its two results).
template <int J>
__device__ __forceinline__ uint32_t xor_lane(uint32_t v) {
  if constexpr (J == 1) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  } else if constexpr (J == 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  } else if constexpr (J == 4) {
    const uint32_t up = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x12C, 0xF, 0xF, false);  // row_ror:12 (i + 4)
    const uint32_t dn = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false);  // row_ror:4 (i - 4)
    return (lane_id() & 4) ? dn : up;
  } else if constexpr (J == 8) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
  } else if constexpr (J == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);  // rows {1,3} <-> rows {0,2}
    return (lane_id() & 16) ? (uint32_t)r[0] : (uint32_t)r[1];
  } else {
    static_assert(J == 32, "xor_lane: J in {1, 2, 4, 8, 16, 32}");
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);  // lanes 32-63 <-> lanes 0-31
    return (lane_id() & 32) ? (uint32_t)r[0] : (uint32_t)r[1];
  }
}

// Global-address-space (1) pointers: an opaque round trip (vreg64, ldsu) would otherwise leave a
// generic pointer, and vector memory ops on it would be flat_* (counted in both vmcnt and lgkmcnt)
// instead of global_*.
#if defined(__HIP_DEVICE_COMPILE__)
template <class T>
using gptr = T __attribute__((address_space(1)))*;
#else  // host pass of the single-source compile: the kernel body is never run there
template <class T>
using gptr = T*;
#endif

// Block placement: rare paths out of line, so the common path runs without taken branches.
#define ME_LIKELY(x) __builtin_expect(!!(x), 1)
#define ME_UNLIKELY(x) __builtin_expect(!!(x), 0)

// Keep a wave-uniform value in VGPRs: the empty asm makes it opaque (hence "divergent") to the
// compiler, so it never takes an SGPR. For pointers and constants that only feed vector memory
// operations and vector arithmetic.
__device__ __forceinline__ uint32_t vreg(uint32_t x) {
  asm volatile("" : "+v"(x));
  return x;
}
__device__ __forceinline__ unsigned long long vreg64(unsigned long long x) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  asm volatile("" : "+v"(lo), "+v"(hi));
  return ((unsigned long long)hi << 32) | lo;
}

template <class T>
__device__ __forceinline__ gptr<T> vptr(T* p) {
  return (gptr<T>)vreg64((unsigned long long)p);
}

// Orders the wave's own global stores before its later loads of the same lines (another lane
// may read what this lane wrote). Same-CU ordering: no cache maintenance, a compiler barrier.
__device__ __forceinline__ void wave_mem_order() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

// Diagnostic build only (-DME_STAMPS): per-wave cycle shares of the matching phases, read with
// me_debug_stamps(). The product build compiles every stamp away.
enum { PH_PROLOGUE, PH_FETCH, PH_SWEEP, PH_WALK, PH_REST, PH_CANCEL, PH_RESULT, PH_EPILOGUE,
       PH_SW_WINDOW, PH_SW_UPDATE, PH_SW_JUMP, PH_SW_BEST, CT_MISS, CT_WALK, CT_EVICT, CT_FAST,
       WK_GET, WK_SCAN, WK_EMIT, WK_TAIL, PH_N };
#ifdef ME_STAMPS
__device__ __forceinline__ unsigned long long stamp_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define STAMP_MARK(c) (c).st_t = stamp_now()
#define COUNT(c, ct) ((c).st[ct] += 1)
#define STAMP_ADD(c, ph)                    \
  do {                                      \
    unsigned long long _n = stamp_now();    \
    (c).st[ph] += _n - (c).st_t;            \
    (c).st_t = _n;                          \
  } while (0)
#else
#define STAMP_MARK(c) ((void)0)
#define STAMP_ADD(c, ph) ((void)0)
#define COUNT(c, ct) ((void)0)
#endif

// First index p in [0, n) with keys[p] >= key (keys ascending), by a 64-ary search:
// every step the wave samples 64 positions, ballots, and narrows the range 64x.
__device__ __forceinline__ uint32_t wave_lower_bound(const uint32_t* keys, uint32_t n, uint32_t key) {
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

// Records whose symbol id is out of range (grouped into bin S): REJECTED / BAD_SYMBOL.
__device__ __forceinline__ void reject_bad_symbols(const BatchDev& bt, uint32_t lo, uint32_t hi) {
  for (uint32_t j = lo + (uint32_t)lane_id(); j < hi; j += 64) {
    const uint32_t i = bt.perm[j];
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
}

}  // namespace me

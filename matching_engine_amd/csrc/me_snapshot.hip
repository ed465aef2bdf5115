// me_snapshot.hip — device book snapshots (GetOrderBook, src/server/matching_engine_service.cpp:123-129;
// OrderBookResponse = repeated Order, proto/matching_engine.proto:16-23,57-60).
//
// k_book_snapshot: one 1024-thread workgroup per (symbol, side) of the request. It walks the side's
// price levels best first — the window from the best level outward, then the far levels (best last
// in their array) — and, for the first `depth` non-empty ones, writes each level's aggregate
// (price, total, order count) and every resting order of its FIFO (seq, price, qty, side) in
// priority order. Levels are taken in passes of up to SNAP_P: the pass's levels are found by a
// block-wide compaction of the window's totals, every thread then walks ONE level's chunk chain to
// count its live slots, a block scan turns the counts into output offsets, and a second walk writes
// the orders. Chains are short (a chunk holds 16 slots), so a pass costs a few chunk-load latencies
// however deep the book is: a 10,000-level side is five passes of one launch.
//
// Bytes per resting order: one 256-B chunk read per 16 orders (twice: count + write) + 24 B out;
// per level 16 B (window) or 32 B (far) read + 24 B out. HBM-bound in principle, latency-bound in
// practice (dependent chunk loads).
#include <hip/hip_runtime.h>

#include "me_layout.hpp"

namespace me {

constexpr int SNAP_T = 1024;  // threads per workgroup
constexpr int SNAP_P = 2048;  // levels per pass (LDS: 24 B each + counts)


__device__ __forceinline__ uint32_t snap_block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t& total) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint32_t incl = v;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(incl, d, 64);
    if (lane >= d) incl += o;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint32_t before = 0, tot = 0;
  for (int k = 0; k < SNAP_T / 64; ++k) {
    const uint32_t x = wsum[k];
    if (k < w) before += x;
    tot += x;
  }
  __syncthreads();
  total = tot;
  return before + incl - v;
}

__global__ __launch_bounds__(SNAP_T) void k_book_snapshot(BookDev bk, SnapReq rq) {
  __shared__ long long p_price[SNAP_P];
  __shared__ long long p_total[SNAP_P];
  __shared__ uint32_t p_head[SNAP_P];
  __shared__ uint32_t p_tail[SNAP_P];
  __shared__ uint32_t p_off[SNAP_P];
  __shared__ uint32_t wsum[SNAP_T / 64];
  __shared__ int s_cur;          // window cursor (next level to look at)
  __shared__ uint32_t s_far;     // far levels taken so far
  __shared__ uint32_t s_np;      // levels in this pass
  const int tid = threadIdx.x;
  const uint32_t q = blockIdx.x >> 1, side = blockIdx.x & 1u;
  const uint32_t s = rq.sym[q];
  const int L = (int)bk.L;
  const SymState st = bk.sym[s];
  const Level* lv = bk.levels + (size_t)s * L;
  const FarDir fd = bk.fdir[(size_t)s * 2u + side];
  const FarLevel* far = bk.far + fd.off;
  const uint32_t nfar = min(st.nfar[side], fd.cap);
  const size_t reg = (size_t)q * 2 + side;
  me_level* lv_out = rq.lv + reg * rq.depth;
  me_book_entry* ord_out = rq.ord ? rq.ord + reg * rq.ocap : nullptr;
  if (tid == 0) {
    s_cur = side == 0 ? min(st.best_bid, L - 1) : max(st.best_ask, 0);
    s_far = 0;
  }
  __syncthreads();
  uint32_t found = 0;
  unsigned long long norders = 0;
  while (found < rq.depth) {
    const uint32_t want = min((uint32_t)SNAP_P, rq.depth - found);
    if (tid == 0) s_np = 0;
    __syncthreads();
    // ---- this pass's levels: window levels in scan order, then far levels
    for (;;) {
      const int cur = s_cur;
      const uint32_t np = s_np;
      const bool win_left = side == 0 ? cur >= 0 : cur < L;
      if (np >= want || !win_left) break;
      const int l = side == 0 ? cur - tid : cur + tid;
      const bool inwin = side == 0 ? l >= 0 : l < L;
      const long long tot = inwin ? lv[l].total : 0;
      const uint32_t nz = tot > 0;
      uint32_t all = 0;
      const uint32_t pos = snap_block_excl_scan(nz, wsum, all);
      if (nz && np + pos < want) {
        const Level x = lv[l];
        p_price[np + pos] = st.base + l;
        p_total[np + pos] = x.total;
        p_head[np + pos] = x.head;
        p_tail[np + pos] = x.tail;
      }
      // the cursor moves past the last level taken (or the whole block when it all fits)
      __syncthreads();
      if (tid == 0) {
        const uint32_t take = min(all, want - np);
        s_np = np + take;
      }
      if (nz && np + pos + 1 == want) s_cur = side == 0 ? l - 1 : l + 1;  // the pass filled at l
      __syncthreads();
      if (tid == 0 && s_np < want) s_cur = side == 0 ? cur - SNAP_T : cur + SNAP_T;
      __syncthreads();
    }
    {
      const uint32_t np = s_np;
      const uint32_t fr = s_far;
      const uint32_t nf = min(want - np, nfar - fr);
      for (uint32_t j = tid; j < nf; j += SNAP_T) {
        const FarLevel f = far[nfar - 1 - (fr + j)];
        p_price[np + j] = f.price;
        p_total[np + j] = f.total;
        p_head[np + j] = f.head;
        p_tail[np + j] = f.tail;
      }
      __syncthreads();
      if (tid == 0) {
        s_np = np + nf;
        s_far = fr + nf;
      }
      __syncthreads();
    }
    const uint32_t np = s_np;
    if (np == 0) break;
    // ---- count every level's live orders (one thread per level), scan, write
    uint32_t cnt[SNAP_P / SNAP_T];
    uint32_t mine = 0;
#pragma unroll
    for (int k = 0; k < SNAP_P / SNAP_T; ++k) {
      const uint32_t i = (uint32_t)tid * (SNAP_P / SNAP_T) + k;
      uint32_t c = 0;
      if (i < np) {
        uint32_t ch = p_head[i], guard = 0;
        while (ch != NIL) {
          if (ch >= bk.nchunks || ++guard > bk.nchunks) {
            atomicOr(rq.err, 1u);
            break;
          }
          const int4* qv = reinterpret_cast<const int4*>(bk.chunks[ch].qty);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int4 v = qv[u];
            c += (v.x > 0) + (v.y > 0) + (v.z > 0) + (v.w > 0);
          }
          if (ch == p_tail[i]) break;
          ch = bk.chunks[ch].hdr.next;
        }
      }
      cnt[k] = c;
      mine += c;
    }
    uint32_t pass_total = 0;
    uint32_t off = snap_block_excl_scan(mine, wsum, pass_total);
#pragma unroll
    for (int k = 0; k < SNAP_P / SNAP_T; ++k) {
      const uint32_t i = (uint32_t)tid * (SNAP_P / SNAP_T) + k;
      if (i < np) {
        p_off[i] = off;
        me_level o;
        o.price_q4 = p_price[i];
        o.total_qty = p_total[i];
        o.order_count = cnt[k];
        o.pad = 0;
        lv_out[found + i] = o;
      }
      off += cnt[k];
    }
    if (ord_out) {
#pragma unroll
      for (int k = 0; k < SNAP_P / SNAP_T; ++k) {
        const uint32_t i = (uint32_t)tid * (SNAP_P / SNAP_T) + k;
        if (i >= np || !cnt[k]) continue;
        unsigned long long o = norders + p_off[i];
        uint32_t ch = p_head[i], guard = 0;
        while (ch != NIL && ch < bk.nchunks && ++guard <= bk.nchunks) {
          const Chunk& c = bk.chunks[ch];
          for (int u = 0; u < ME_C; ++u) {
            const int qq = c.qty[u];
            if (qq > 0) {
              if (o < rq.ocap) {
                me_book_entry e;
                e.seq = c.seq[u];
                e.price_q4 = p_price[i];
                e.qty = qq;
                e.side = side == 0 ? ME_SIDE_BUY : ME_SIDE_SELL;
                e.pad[0] = e.pad[1] = e.pad[2] = 0;
                ord_out[o] = e;
              }
              ++o;
            }
          }
          if (ch == p_tail[i]) break;
          ch = c.hdr.next;
        }
      }
    }
    norders += pass_total;
    found += np;
    __syncthreads();
    if (np < want) break;  // both sources exhausted
  }
  if (tid == 0) {
    rq.nlv[reg] = found;
    rq.nord[reg] = norders;
  }
}

hipError_t launch_book_snapshot(hipStream_t st, const BookDev& bk, const SnapReq& rq) {
  if (!rq.nsym || !rq.depth) return hipSuccess;
  hipLaunchKernelGGL(k_book_snapshot, dim3(rq.nsym * 2), dim3(SNAP_T), 0, st, bk, rq);
  return hipGetLastError();
}

}  // namespace me

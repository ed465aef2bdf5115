// me_engine.cpp — host side of the batched matching core: owns the HBM-resident books of one
// shard, stages batches, enqueues the gfx950 pipeline (me_kernels.hip) and implements the
// C-ABI of include/me_engine.h. No CPU matching path exists here: without a HIP device
// me_create fails and every call reports it.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "me_engine.h"
#include "me_layout.hpp"

static_assert(me::ME_C == ME_CHUNK_SLOTS, "chunk width mismatch");
static_assert(sizeof(me_fill) == 32, "me_fill must be 32 B");
static_assert(sizeof(me_order_result) == 20, "me_order_result must be 20 B");

namespace me {
hipError_t launch_sort_pass(hipStream_t st, const uint32_t* keys_in, const uint32_t* idx_in, uint32_t n,
                            uint32_t clamp_key, int shift, int dbits, uint32_t* hist, uint32_t* tot,
                            uint32_t* keys_out, uint32_t* idx_out, uint32_t* zero_buf,
                            uint32_t zero_words, unsigned long long* scratch_top, uint32_t* bin_start,
                            const uint64_t* seq, const uint8_t* kind, uint32_t* err);
hipError_t launch_seq_sweep(hipStream_t st, const BookDev& bk, const uint64_t* const* seq, const uint8_t* const* kind,
                            const uint32_t* n, uint32_t ng, uint32_t in_idx, uint32_t grid, uint32_t launch);
hipError_t launch_match(hipStream_t st, const BookDev& bk, const BatchDev& bt, hipEvent_t ev0, hipEvent_t ev1,
                        const HotLaunch& hot);
hipError_t launch_match_reg(hipStream_t st, const BookDev& bk, const BatchDev* bt, uint32_t ng, const AuxDev& ax, hipEvent_t ev0,
                            hipEvent_t ev1, const HotLaunch* hot);
namespace rc64 {
hipError_t launch_fill_early(hipStream_t st, const BookDev& bk, const AuxDev& ax, bool& done);
}
uint32_t sort_tile(uint32_t n);
hipError_t launch_tape(hipStream_t st, const BatchDev& bt, me_fill* tape, unsigned long long tape_cap,
                       unsigned long long* tape_count, unsigned long long* fills_acc, uint32_t* err,
                       me_order_result* hres, uint32_t* err_out);
hipError_t launch_tape_spill(hipStream_t st, const me_order_result* res, const uint32_t* fstart, uint32_t n,
                             const me_fill* scratch, unsigned long long cap, me_fill* spill);
hipError_t launch_init_levels(hipStream_t st, Level* levels, size_t count);
hipError_t launch_book_snapshot(hipStream_t st, const BookDev& bk, const SnapReq& rq);
hipError_t launch_init_chunks(hipStream_t st, Chunk* chunks, size_t count);
}  // namespace me

using namespace me;

namespace {
std::mutex g_err_mu;
std::string g_create_err;

struct TimedLaunch {
  hipEvent_t m0, m1;  // start / end of one match-kernel launch (recorded by the launch itself)
  uint64_t orders;
  uint64_t idx;       // batches matched (since timing was enabled) before this launch
};

// A few host threads for the staging copy of large host batches (me_submit_host): one memcpy into
// pinned memory runs at ~10 GB/s, which alone would cap the host path near 400M orders/s (25 B each).
class CopyPool {
 public:
  struct Piece {
    void* dst;
    const void* src;
    size_t bytes;
  };
  explicit CopyPool(int n) {
    for (int i = 0; i < n; ++i) th_.emplace_back([this] { worker(); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  // Copies every piece (the caller works too); no worker touches them after it returns.
  void run(const std::vector<Piece>& p) {
    std::unique_lock<std::mutex> lk(mu_);
    jobs_ = p.data();
    njobs_ = p.size();
    next_.store(0);
    done_ = 0;
    ++gen_;
    cv_.notify_all();
    lk.unlock();
    work(jobs_, njobs_);
    lk.lock();
    done_cv_.wait(lk, [&] { return done_ == njobs_ && active_ == 0; });
    jobs_ = nullptr;
    njobs_ = 0;
  }

 private:
  void work(const Piece* jobs, size_t nj) {
    size_t mine = 0;
    for (;;) {
      const size_t i = next_.fetch_add(1);
      if (i >= nj) break;
      memcpy(jobs[i].dst, jobs[i].src, jobs[i].bytes);
      ++mine;
    }
    std::lock_guard<std::mutex> lk(mu_);
    done_ += mine;
    if (done_ == njobs_) done_cv_.notify_all();
  }
  void worker() {
    std::unique_lock<std::mutex> lk(mu_);
    uint64_t seen = 0;
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || (gen_ != seen && jobs_); });
      if (stop_) return;
      seen = gen_;
      const Piece* jobs = jobs_;
      const size_t nj = njobs_;
      ++active_;
      lk.unlock();
      work(jobs, nj);
      lk.lock();
      --active_;
      done_cv_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const Piece* jobs_ = nullptr;
  size_t njobs_ = 0;
  std::atomic<size_t> next_{0};
  size_t done_ = 0;
  int active_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// Output block of a host slot in pinned memory: SlotMeta, the results (max_batch records), the tape
// (cap records, 64-B aligned). The tape job writes all of it straight over PCIe (device-mapped).
struct SlotMeta {
  unsigned long long count;  // the batch's tape length (may exceed the slot's cap)
  uint32_t err;              // the device error word when the tape job finished
  uint32_t pad;
};
static_assert(sizeof(SlotMeta) == 16, "SlotMeta");

// One slot of the host-batch pipeline (me_submit_host / me_collect).
struct HostSlot {
  char* h_in = nullptr;   // pinned staging: the batch packed as seq[n] px[n] qty[n] sym[n] kind[n]
  char* d_in = nullptr;   // its HBM copy
  char* h_out = nullptr;  // pinned outputs (SlotMeta | tape | results): the tape job writes the meta and
                          // the tape straight into it over PCIe; the results arrive by DMA
  char* h_out_dev = nullptr;  // h_out as the device addresses it
  hipEvent_t ev_in = nullptr;    // H2D done (H2D stream)
  hipEvent_t ev_done = nullptr;  // outputs in pinned memory (recorded after the launch with the tape job)
  uint64_t ticket = 0;
  uint32_t n = 0;
  int state = 0;  // 0 free (collected), 1 enqueued, 2 outputs copy enqueued
  int oset = 0;   // output set (results / scratch starts / scratch) the batch used, and its generation
  uint64_t oset_gen = 0;
  std::vector<me_fill> big;  // the whole tape when it outgrew the slot (spilled at me_collect)
};
}  // namespace

struct me_engine {
  me_config cfg{};
  int dev = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  HotLaunch hot;  // deep windows with hot symbols: k_match_hot's stream and fork / join events
  BookDev bk{};
  std::vector<int64_t> base_host;
  // grouping sort plan
  int passes = 1;
  int dbits[2] = {0, 0};
  // Everything the grouping sort of a batch writes: sorted keys, permutation, histogram, run
  // table, and the per-batch counters it zeroes.
  struct SortBufs {
    uint32_t* keys[2] = {nullptr, nullptr};
    uint32_t* idx[2] = {nullptr, nullptr};
    uint32_t* hist = nullptr;
    uint32_t* tot = nullptr;        // [2 passes][2048] bin totals
    uint32_t* bin_start = nullptr;  // [2049] run table of the single-pass sort
  } sb;
  // Per-batch outputs. The pipelined register-ladder path rotates three groups of `group` sets
  // (group J is bucketed while J-1 is matched and J-2's tapes are compacted); the
  // other paths use set 0.
  struct OutSet {
    me_order_result* res = nullptr;
    uint32_t* fstart = nullptr;
    uint32_t* tile_sum = nullptr;
    me_fill* scratch = nullptr;
    unsigned long long* top = nullptr;
  } os[3 * ME_GMAX];
  int nsets = 1;
  int last_set = 0;  // output set of the most recent batch
  // Bucketed grouping (register-ladder kernel): per-bin counts and BK_CAP-record buckets.
  struct BucketBufs {
    uint32_t* cnt = nullptr;
    BkRec* rec = nullptr;
  } bu[2 * ME_GMAX];
  bool bucketed = false;
  // Pipelined path: batches submitted but not finished. Submits fill a group of up to `group`
  // batches; a full group is bucketed in one launch, matched in the next, its tapes compacted in the
  // one after; me_sync (and everything that reads outputs or the book) flushes.
  struct Pend {
    bool valid = false;
    const uint64_t* seq = nullptr;
    const int64_t* px = nullptr;
    const int32_t* qty = nullptr;
    const uint32_t* sym = nullptr;
    const uint8_t* kind = nullptr;
    uint32_t n = 0;
    int oset = 0, bset = 0;
    int slot = -1;  // host slot (me_submit_host), -1: a device batch
    uint32_t nadm = 0;  // records admission control counted for it
  };
  struct Group {
    Pend b[ME_GMAX];
    uint32_t n = 0;
    uint32_t filled = 0;  // g_fill: batches [0, filled) already bucketed by an early fill launch
  } g_fill, g_match, g_tape;
  // Early fill: while nothing is in flight (the first group after a flush), every `early_fill` submitted
  // batches are bucketed at once, so the fill overlaps the submits of the rest of the group (0: off;
  // ME_EARLY_FILL). Config 2's driver shape, same box: 8 -> +1.6 % over off (-0.6 to +2.4 % for earlier
  // forms), 4 and 16 no better (profiles/r6/early_fill).
  uint32_t early_fill = 8;
  uint32_t group = 1;     // batches per launch (me_config.batches_per_launch)
  uint64_t ngroup = 0;    // groups launched
  int last_tape = 0;      // tape buffer (position in its group) of the most recent batch
  uint32_t ncu = 0;  // compute units: workgroups of one dispatch round host the side jobs
  me_fill* d_tape = nullptr;                   // [group][tape_cap]: one tape per position in a group
  unsigned long long* d_tape_count = nullptr;  // [ME_GMAX]
  unsigned long long* d_fills_acc = nullptr;  // fills since timing was (re)enabled
  unsigned long long scratch_cap = 0;  // fill scratch: per-symbol slabs + overflow region
  unsigned long long tape_cap = 0;     // tape bound of one batch (max_resting + 2 * max_batch)
  uint32_t slab = 0;                   // scratch fills per symbol slab (register-ladder kernel)
  uint32_t ntiles_sort = 0;            // sort tiles of a max_batch batch (histogram row stride)
  // host-batch pipeline
  std::vector<HostSlot> hs;
  std::vector<int> free_slots;  // LIFO: a synchronous caller keeps reusing the same few warm slots (two in
                                // flight plus the one me_collect holds back)
  int held_slot = -1;           // the last collected slot: its outputs stay readable until the next
                                // me_collect (or a submit that finds every other slot busy)
  std::unordered_map<uint64_t, int> by_ticket;  // uncollected tickets -> slot
  uint64_t hcap = 0;         // tape records per slot
  uint64_t next_ticket = 0;
  hipStream_t s_h2d = nullptr;
  std::vector<uint64_t> oset_gen;  // batches assigned to each output set so far
  me_fill* d_spill = nullptr;
  size_t spill_cap = 0;
  bool last_host = false;  // the most recent batch was a host batch (the device-output fetches refuse)
  std::unique_ptr<CopyPool> copy_pool;  // started on the first large host batch
  struct SnapBufs {  // device buffers of the book snapshot kernel, grown on demand
    uint32_t* sym = nullptr;
    me_level* lv = nullptr;
    uint32_t* nlv = nullptr;
    me_book_entry* ord = nullptr;
    unsigned long long* nord = nullptr;
    uint32_t* err = nullptr;
    size_t sym_cap = 0, lv_cap = 0, n_cap = 0, ord_cap = 0, nord_cap = 0, err_cap = 0;
  } snap;
  uint32_t last_n = 0;
  uint32_t sq_idx = 0;  // seq-ring state the next k_seq_sweep reads (it writes the other one)
  struct LastGroup {    // the launch group holding the most recent batch: where its outputs live
    uint32_t n = 0;
    int oset[ME_GMAX];
    int tape[ME_GMAX];
    uint32_t bn[ME_GMAX];
  } lastg;
  bool failed = false;
  std::string err;
  // admission control (me_config.max_resting): a batch is accepted only while the resting orders
  // the device can hold after it stay within max_resting, so the scratch / tape / old-order bounds
  // sized from it can never overflow. Bound = resting orders known after k match launches + every
  // record accepted since (each rests at most once). k_seq_sweep publishes {k, resting} into pinned
  // memory ahead of every match launch; a synchronous exact count replaces it when it is too stale.
  static constexpr uint32_t ADM_RING = 256;
  unsigned long long* pub_host = nullptr;  // hipHostMalloc'd, device-mapped (bk.pub): [0] {launch, resting},
                                           // [1] {launch, hand-offs}, [2] me_sync's error-word copy
  // grouped launches through the aggregate path (hot.agg_reg) chosen by shape, not by ME_REG_AGG: turned
  // off for good when symbols hand off to the continuation in more than 1/16 of their launches (cancels,
  // far prices — config 5's stream), which then pays both paths
  bool reg_agg_auto = false;
  uint64_t ho_k = 0, ho_h = 0;  // the last {launch, hand-offs} sample
  // groups with cancels through the walk that covers them (k_agg_gwalk_cx, hot.ag.gw_cx): ME_GW_CANCEL=1 from
  // the start, =0 never; unset, from the first sample whose hand-off rate would have turned the grouped path
  // off (only if hand-offs stay that high with it does the grouped path go)
  bool gw_cx_auto = false;
  uint64_t cx_from = 0;  // (auto) samples of launches before the switch do not count against the new walk
  uint32_t launch_no = 0;                  // match launches enqueued
  uint64_t adm_total = 0;                  // records accepted
  uint64_t adm_matched = 0;                // records of the batches those launches matched
  uint64_t adm_at[ADM_RING] = {};          // adm_matched after launch k (k % ADM_RING)
  uint64_t ovr_resting = 0, ovr_adm = 0;   // the last exact count and the records accepted then
  uint64_t adm_syncs = 0;                  // exact counts taken (diagnostic)
  // timing
  int timing = 0;           // 0: off; k >= 1: time every k-th match launch
  uint64_t nlaunch = 0;     // match launches since timing was enabled
  uint64_t nbat = 0;        // batches those launches matched
  std::vector<TimedLaunch> timed;  // launches since timing was enabled
  std::vector<hipEvent_t> ev_pool;  // events reused across enable cycles (no create per launch)
  size_t ev_used = 0;
  std::vector<void*> user_allocs;

  int fail(int code, const std::string& msg) {
    err = msg;
    if (code == ME_E_CAPACITY || code == ME_E_HIP) failed = true;
    return code;
  }
  int hip_fail(hipError_t e, const char* what) {
    return fail(ME_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
  }
};

#define HIP_TRY(expr, what)                         \
  do {                                              \
    hipError_t _e = (expr);                         \
    if (_e != hipSuccess) return e->hip_fail(_e, what); \
  } while (0)

static int set_create_err(const std::string& s) {
  std::lock_guard<std::mutex> lk(g_err_mu);
  g_create_err = s;
  return 0;
}

static void free_all(me_engine* e) {
  void* ptrs[] = {e->bk.levels,   e->bk.occ,      e->bk.sym,      e->bk.chunks,     e->bk.tend,
                  e->bk.loc,      e->bk.chunk_top, e->bk.err,       (void*)e->bk.gsym,
                  e->d_tape,      e->d_tape_count, e->d_fills_acc, e->bk.dbg,      e->bk.fcache,
                  e->bk.far,      e->bk.old,       e->bk.sq,       e->bk.hcount,     e->bk.hand,
                  e->bk.stats,    e->bk.fdir,      e->bk.far_ctl,  e->bk.cpool,      e->bk.recl};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  {
    auto& sl = e->sb;
    void* sp[] = {sl.keys[0], sl.keys[1], sl.idx[0], sl.idx[1], sl.hist, sl.tot, sl.bin_start};
    for (void* p : sp)
      if (p) (void)hipFree(p);
    for (auto& b : e->bu) {
      void* bp[] = {b.cnt, b.rec};
      for (void* p : bp)
        if (p) (void)hipFree(p);
    }
    for (auto& o : e->os) {
      void* op[] = {o.res, o.fstart, o.tile_sum, o.scratch, o.top};
      for (void* p : op)
        if (p) (void)hipFree(p);
    }
  }
  {
    const AggDev& a = e->hot.ag;
    void* ap[] = {a.slot, a.ev, a.evs, a.evq, a.eva, a.evf, a.evn, a.evx, a.seg, a.segs, a.mk, a.fr, a.rec, a.ctr,
                  a.gev, a.gex, a.gbase};
    for (void* p : ap)
      if (p) (void)hipFree(p);
  }
  for (void* p : e->user_allocs) (void)hipFree(p);
  e->user_allocs.clear();
  for (auto& h : e->hs) {
    if (h.h_in) (void)hipHostFree(h.h_in);
    if (h.h_out) (void)hipHostFree(h.h_out);
    if (h.d_in) (void)hipFree(h.d_in);
    if (h.ev_in) (void)hipEventDestroy(h.ev_in);
    if (h.ev_done) (void)hipEventDestroy(h.ev_done);
  }
  e->hs.clear();
  if (e->d_spill) (void)hipFree(e->d_spill);
  {
    void* sp[] = {e->snap.sym, e->snap.lv, e->snap.nlv, e->snap.ord, e->snap.nord, e->snap.err};
    for (void* p : sp)
      if (p) (void)hipFree(p);
  }
  if (e->pub_host) (void)hipHostFree(e->pub_host);
  if (e->s_h2d) (void)hipStreamDestroy(e->s_h2d);
  for (auto ev : e->ev_pool) (void)hipEventDestroy(ev);
  e->ev_pool.clear();
  e->timed.clear();
  if (e->hot.fork) (void)hipEventDestroy(e->hot.fork);
  if (e->hot.join) (void)hipEventDestroy(e->hot.join);
  if (e->hot.st) (void)hipStreamDestroy(e->hot.st);
  if (e->hot.sfork) (void)hipEventDestroy(e->hot.sfork);
  if (e->hot.sjoin) (void)hipEventDestroy(e->hot.sjoin);
  if (e->hot.sst) (void)hipStreamDestroy(e->hot.sst);
  if (e->own_stream) (void)hipStreamDestroy(e->own_stream);
}

extern "C" int me_normalize_to_q4(int64_t price, int32_t scale, int64_t* out) {
  // include/domain/price.hpp:15-29: target scale 4, *10^diff with overflow checks, /10^-diff
  // truncating toward zero.
  static const int64_t P10[19] = {1LL,
                                  10LL,
                                  100LL,
                                  1000LL,
                                  10000LL,
                                  100000LL,
                                  1000000LL,
                                  10000000LL,
                                  100000000LL,
                                  1000000000LL,
                                  10000000000LL,
                                  100000000000LL,
                                  1000000000000LL,
                                  10000000000000LL,
                                  100000000000000LL,
                                  1000000000000000LL,
                                  10000000000000000LL,
                                  100000000000000000LL,
                                  1000000000000000000LL};
  if (scale < 0 || scale > 18) return 1;
  if (scale == 4) {
    *out = price;
    return 0;
  }
  const int diff = 4 - scale;
  if (diff > 0) {
    const int64_t mul = P10[diff];
    if (price > 0 && price > INT64_MAX / mul) return 2;
    if (price < 0 && price < INT64_MIN / mul) return 3;
    *out = price * mul;
    return 0;
  }
  *out = price / P10[-diff];
  return 0;
}

template <class T>
static hipError_t dalloc(T** p, size_t count) {
  return hipMalloc((void**)p, std::max<size_t>(count, 1) * sizeof(T));
}

static bool zero_bucket_counts(me_engine* e, hipStream_t st) {
  if (!e->bucketed) return true;
  for (uint32_t k = 0; k < 2 * e->group; ++k)
    if (hipMemsetAsync(e->bu[k].cnt, 0, (e->bk.S + 1) * (size_t)BK_CNT_STRIDE * 4, st) != hipSuccess) return false;
  return true;
}

extern "C" me_engine* me_create(const me_config* cfg) {
  if (!cfg || cfg->num_symbols == 0 || cfg->levels < 64 || (cfg->levels & (cfg->levels - 1)) ||
      cfg->levels > (1u << 20) || cfg->max_batch == 0 || !cfg->base_price ||
      (cfg->seq_ring && (cfg->seq_ring < 64 || (cfg->seq_ring & (cfg->seq_ring - 1)) || cfg->seq_ring > (1ull << 34)))) {
    set_create_err("me_create: invalid config (num_symbols>0, levels power of two in [64,2^20], "
                   "max_batch>0, base_price, seq_ring 0 or a power of two in [64, 2^34])");
    return nullptr;
  }
  const uint64_t S = cfg->num_symbols;
  // key range 0..S (S = reject bin) -> radix plan
  int bits = 1;
  while ((1ull << bits) < S + 1) ++bits;
  int passes, d0, d1;
  if (bits <= MAX_DIGIT_BITS) {
    passes = 1;
    d0 = bits;
    d1 = 0;
  } else if (bits <= 2 * MAX_DIGIT_BITS) {
    passes = 2;
    d0 = (bits + 1) / 2;
    d1 = bits - d0;
  } else {
    set_create_err("me_create: num_symbols too large for the 2-pass grouping sort (max 4M)");
    return nullptr;
  }
  int ndev = 0;
  hipError_t he = hipGetDeviceCount(&ndev);
  if (he != hipSuccess || ndev <= 0) {
    set_create_err(std::string("me_create: no HIP device (") + hipGetErrorString(he) + ")");
    return nullptr;
  }
  if (cfg->device < 0 || cfg->device >= ndev) {
    set_create_err("me_create: device ordinal out of range");
    return nullptr;
  }
  me_engine* e = new me_engine();
  e->cfg = *cfg;
  e->dev = cfg->device;
  e->passes = passes;
  e->dbits[0] = d0;
  e->dbits[1] = d1;
  const uint64_t L = cfg->levels;
  uint64_t nchunks = cfg->max_chunks;
  // chunks in use <= resting orders (every linked chunk holds a live order), whatever the book shape and
  // whichever symbols hold them: k_seq_sweep's reclamation returns every symbol's free chunks to the pool
  // before a launch group that could otherwise run out (me_kernels.hip chunk_reclaim). On top of
  // max_resting, one group draws for its LIMIT records (admission control) plus, per wave, the unused
  // rest of one reservation block (< 16 chunks) — at most two waves per symbol and group.
  if (nchunks == 0) nchunks = cfg->max_resting + 32 * S + 64;
  const uint64_t n = cfg->max_batch;
  const unsigned long long scap = cfg->max_resting + 2 * n;
  auto bail = [&](const std::string& m) -> me_engine* {
    set_create_err(m);
    free_all(e);
    delete e;
    return nullptr;
  };
  if (nchunks * ME_C >= 0xFFFFFFFFull) return bail("me_create: chunk pool exceeds 32-bit slot ids");
  // Register-ladder kernel (L <= 128): every symbol owns a scratch slab sized for ~4x its mean
  // share of a batch; a wave that might outgrow it reserves its batch bound in the overflow region.
  uint64_t slab = 0;
  if (L <= 128) {
    slab = 4 * ((n + S - 1) / S) + 16;
    slab = (slab + 15) & ~15ull;
    if (slab < 64) slab = 64;
    if (slab > 4096) slab = 4096;
  }
  const unsigned long long ovf_base = (S + 1) * slab;
  if (scap + ovf_base >= 0xFFFFFFFFull) return bail("me_create: scratch bound exceeds 32-bit fill ids");
  if (n >= 0x7FFFFFFFull) return bail("me_create: max_batch too large");
  he = hipSetDevice(e->dev);
  if (he != hipSuccess) return bail(std::string("hipSetDevice: ") + hipGetErrorString(he));
  {
    int ncu = 0;
    he = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, e->dev);
    if (he != hipSuccess) return bail(std::string("hipDeviceGetAttribute: ") + hipGetErrorString(he));
    e->ncu = (uint32_t)(ncu > 0 ? ncu : 1);
  }
  he = hipStreamCreateWithFlags(&e->own_stream, hipStreamNonBlocking);
  if (he != hipSuccess) return bail(std::string("hipStreamCreate: ") + hipGetErrorString(he));
  e->stream = e->own_stream;
  BookDev& bk = e->bk;
  bk.S = (uint32_t)S;
  bk.L = (uint32_t)L;
  bk.Lwords = (uint32_t)(L / 64);
  bk.nchunks = (uint32_t)nchunks;
  const uint64_t ring = cfg->seq_ring ? cfg->seq_ring : (1ull << 28);
  bk.ring_mask = ring - 1;
  // far levels: an inline region of fcap entries per (symbol, side), and two halves of 6 x max_resting
  // entries that sides outgrowing it move into, collected above 2 x max_resting (me_far.hpp's bound)
  bk.fcap = cfg->far_levels ? cfg->far_levels : 256u;
  bk.far_gc_at = 2 * (cfg->max_resting + 64);
  bk.far_half = 6 * (cfg->max_resting + 64) + 4ull * bk.fcap;
  if (const char* v = getenv("ME_FAR_GC_AT"))  // (tests: collect earlier — any lower trigger keeps the bound)
    bk.far_gc_at = std::min<uint64_t>(bk.far_gc_at, strtoull(v, nullptr, 10));
  // deep windows (L > 128, the sort path): a symbol with at least hot_min records in a batch runs the
  // aggregate path (me_agg.hip, L <= AGG_MAX_L) — or, with ME_HOT_AGG=0, the write-through top-of-book
  // path k_match_hot (HBM ladders, L > LDS_MAX_LEVELS); ME_HOT_MIN overrides the threshold (0 = off)
  {
    const char* v = getenv("ME_HOT_MIN");
    const char* va = getenv("ME_HOT_AGG");
    e->hot.agg = L > 128 && L <= AGG_MAX_L && !(va && atoi(va) == 0);
    // L <= 128: every symbol of a launch group through the aggregate path (k_agg_gwalk) instead of
    // k_match_reg's serial loop — ME_REG_AGG=1 (measured per workload)
    // (unset: on when a batch holds >= 8 records per symbol and a group >= 256 — config 2's shape, 64 and
    // 2,048; config 3's ~10.5 and ~336 runs 1,296M vs 1,124M on k_match_reg at the driver's shape, 1,590M
    // vs 1,209M over 64 batches, same box, profiles/r4/c3agg; a group's per-symbol set-up — the ladder
    // load, the resolve's workgroup — needs the records to amortise it — in batches of >= 8,192 records,
    // and off for good once hand-offs show up, see reg_agg_auto)
    const char* vr = getenv("ME_REG_AGG");
    const uint64_t grp = cfg->batches_per_launch ? cfg->batches_per_launch : ME_DEFAULT_GROUP;
    // (k_agg_gres keeps each event's seq as a 32-bit offset from the group's first seq: seq_ring <= 2^32)
    e->hot.agg_reg = L <= 128 && ring <= (1ull << 32) && (vr ? atoi(vr) != 0
                                     : (uint64_t)cfg->max_batch >= 8ull * S && cfg->max_batch >= 8192u &&
                                           (uint64_t)cfg->max_batch * grp >= 256ull * S &&
                                           (uint64_t)cfg->max_batch * grp <= (8ull << 20));  // (pools of a
                                                                                             // group's records)
    e->reg_agg_auto = e->hot.agg_reg && !vr;
    const char* vc = getenv("ME_GW_CANCEL");
    e->hot.ag.gw_cx = e->hot.agg_reg && vc && atoi(vc) != 0 ? 1u : 0u;
    e->gw_cx_auto = e->hot.agg_reg && !vc;
    if (const char* ve = getenv("ME_EARLY_FILL")) e->early_fill = (uint32_t)atoi(ve);  // (0: off)
    // the grouped aggregate path's side jobs on a stream of their own (ME_SIDE_STREAM=0: in line)
    const char* vs = getenv("ME_SIDE_STREAM");
    if (e->hot.agg_reg && !(vs && atoi(vs) == 0)) {
      if ((he = hipStreamCreateWithFlags(&e->hot.sst, hipStreamNonBlocking)) != hipSuccess ||
          (he = hipEventCreateWithFlags(&e->hot.sfork, hipEventDisableTiming)) != hipSuccess ||
          (he = hipEventCreateWithFlags(&e->hot.sjoin, hipEventDisableTiming)) != hipSuccess)
        return bail(std::string("side stream: ") + hipGetErrorString(he));
    }
    bk.hot_min = (e->hot.agg || L > LDS_MAX_LEVELS) ? (v ? (uint32_t)atoi(v) : 512u) : 0u;
    if (bk.hot_min) {
      if ((he = hipStreamCreateWithFlags(&e->hot.st, hipStreamNonBlocking)) != hipSuccess ||
          (he = hipEventCreateWithFlags(&e->hot.fork, hipEventDisableTiming)) != hipSuccess ||
          (he = hipEventCreateWithFlags(&e->hot.join, hipEventDisableTiming)) != hipSuccess)
        return bail(std::string("hot stream: ") + hipGetErrorString(he));
    }
  }
  // old-order table: live orders <= resting, at load <= 1/2
  uint64_t oldn = 1024;
  while (oldn < 2 * (cfg->max_resting + 64)) oldn <<= 1;
  bk.old_mask = oldn - 1;
  const uint32_t ntiles_sort = MAX_SORT_TILES;
  const uint32_t ntiles_tape = (uint32_t)((n + TILE_TAPE - 1) / TILE_TAPE);
#define ALLOC(p, cnt)                                                              \
  do {                                                                             \
    hipError_t _e = dalloc(&(p), (cnt));                                           \
    if (_e != hipSuccess) return bail(std::string("hipMalloc " #p ": ") + hipGetErrorString(_e)); \
  } while (0)
  ALLOC(bk.levels, S * L);
  ALLOC(bk.occ, S * (L / 64));
  ALLOC(bk.tend, S * L);
  ALLOC(bk.sym, S);
  ALLOC(bk.chunks, nchunks);
  ALLOC(bk.loc, ring);
  ALLOC(bk.far, S * 2 * (uint64_t)bk.fcap + 2 * bk.far_half);
  ALLOC(bk.fdir, S * 2);
  ALLOC(bk.far_ctl, FC_N);
  ALLOC(bk.old, oldn);
  ALLOC(bk.sq, 2);
  ALLOC(bk.hcount, 2);  // [0] hand-offs of a launch, [1] k_match_hot's continuations
  ALLOC(bk.hand, 2 * S);  // continuations from S on
  ALLOC(bk.stats, ME_STATS);
  if ((bk.hot_min && e->hot.agg) || e->hot.agg_reg) {
    // the aggregate path's pools (me_agg.hip): the log holds every hot symbol's events (<= 3 records +
    // its occupied levels each; a symbol that finds no room goes to the generic loop), consumed makers
    // <= fills <= max_resting + 2n, chunk ids <= 2 x consumed makers + rests. Grouped launches (L <= 128):
    // every symbol, the records of a whole group.
    AggDev& a = e->hot.ag;
    const uint64_t gmax = e->hot.agg_reg ? (cfg->batches_per_launch ? cfg->batches_per_launch : ME_DEFAULT_GROUP) : 1;
    const uint64_t nrec = n * gmax;
    const uint64_t evc = e->hot.agg_reg ? 3 * nrec + S * (L + 128) + 4096 : 3 * n + 16 * (L + 64) + 4096;
    // (per slot: resting + 2 records + 64 makers, twice that + records + 64 chunk ids; the slots of a
    // launch are at most S)
    const uint64_t mkc = cfg->max_resting + 2 * nrec + 64 * (S + 1);
    const uint64_t frc = 2 * mkc + nrec + 64 * (S + 1);
    if (evc >= 0x7FFFFFFFull || frc >= 0xFFFFFFFFull) return bail("me_create: aggregate-path pools exceed 32-bit ids");
    a.ev_cap = (uint32_t)evc;
    // k_agg_walk's two forms: the ladder walk (32-bit LDS totals indexed by level) up to ladder_max
    // levels, the top-of-book lists beyond (and for any book whose sum the 32-bit ladder cannot hold).
    // ME_AGG_LADDER overrides (up to AGG_MAX_L; 0: lists only). Ladders deeper than lw_occ find the next
    // occupied level through an occupancy bitmap in LDS (one read covers 4,096 levels) instead of scanning
    // the totals 64 levels at a time: config 4's 32,768-level books, whose takes empty a level about every
    // record with gaps of hundreds of levels to the next, ran 11.0M orders/s on the lists, 8.6M on the
    // scanning ladder and 15.6M on the bitmap ladder (same box, profiles/r5/occ). ME_LW_OCC overrides (0: off).
    const char* vl = getenv("ME_AGG_LADDER");
    a.ladder_max = vl ? (uint32_t)atoi(vl) : AGG_MAX_L;
    const char* vo = getenv("ME_LW_OCC");
    a.lw_occ = vo ? (uint32_t)atoi(vo) : 256u;
    a.mk_cap = (uint32_t)mkc;
    a.fr_cap = (uint32_t)frc;
    ALLOC(a.slot, S);
    ALLOC(a.ev, evc);
    ALLOC(a.evs, evc);
    ALLOC(a.evq, evc);
    ALLOC(a.eva, evc);
    ALLOC(a.evf, evc);
    ALLOC(a.evn, evc);
    ALLOC(a.evx, evc);
    ALLOC(a.seg, evc);
    ALLOC(a.segs, evc);
    ALLOC(a.mk, mkc);
    ALLOC(a.fr, frc);
    ALLOC(a.rec, n);
    ALLOC(a.ctr, AC_N);
    if (e->hot.agg_reg) {
      ALLOC(a.gev, S * (ME_GMAX + 1));
      ALLOC(a.gex, S * (ME_GMAX + 1));
      ALLOC(a.gbase, S * (ME_GMAX + 1));
    }
    if ((he = hipMemset(a.ctr, 0, AC_N * sizeof(uint32_t))) != hipSuccess)
      return bail(std::string("hipMemset agg ctr: ") + hipGetErrorString(he));
    bk.agg_ctr = a.ctr;
  }
  if ((he = hipHostMalloc((void**)&e->pub_host, 4 * sizeof(unsigned long long), hipHostMallocDefault)) != hipSuccess ||
      (he = hipHostGetDevicePointer((void**)&bk.pub, e->pub_host, 0)) != hipSuccess)
    return bail(std::string("me_create: pinned admission word: ") + hipGetErrorString(he));
  e->pub_host[0] = e->pub_host[1] = 0ull;  // {0 launches, 0 resting / hand-offs}
  e->pub_host[2] = e->pub_host[3] = 0ull;  // [2]: me_sync's copy of the error word
  ALLOC(bk.chunk_top, 1);
  ALLOC(bk.cpool, CP_N);
  ALLOC(bk.recl, nchunks);
  ALLOC(bk.err, 1);
  uint32_t* gsym = nullptr;
  ALLOC(gsym, S);
  bk.gsym = gsym;
  {
    auto& sl = e->sb;
    for (int k = 0; k < 2; ++k) {
      ALLOC(sl.keys[k], n);
      ALLOC(sl.idx[k], n);
    }
    ALLOC(sl.hist, (size_t)(1u << MAX_DIGIT_BITS) * ntiles_sort);
    ALLOC(sl.tot, 2u << MAX_DIGIT_BITS);
    ALLOC(sl.bin_start, (1u << MAX_DIGIT_BITS) + 1);
  }
  // Register-ladder kernel: bucketed grouping when the sort key (index << 7 | slot) fits 32 bits.
  e->bucketed = L <= 128 && n < BK_MAX_BATCH;
  e->group = e->bucketed ? (cfg->batches_per_launch ? cfg->batches_per_launch : ME_DEFAULT_GROUP) : 1u;
  if (e->group > (uint32_t)ME_GMAX) return bail("me_create: batches_per_launch exceeds " + std::to_string(ME_GMAX));
  if (e->bucketed) {
    const size_t nb = (S + 1) * (size_t)BK_CAP;
    for (uint32_t k = 0; k < 2 * e->group; ++k) {
      auto& b = e->bu[k];
      ALLOC(b.cnt, (S + 1) * BK_CNT_STRIDE);
      ALLOC(b.rec, nb);
    }
  }
  // the sort path rotates three sets too, so a host batch's scratch outlives the next two batches
  e->nsets = e->bucketed ? 3 * (int)e->group : 3;
  for (int k = 0; k < e->nsets; ++k) {
    auto& o = e->os[k];
    ALLOC(o.res, n);
    ALLOC(o.fstart, n);
    ALLOC(o.tile_sum, ntiles_tape);
    ALLOC(o.scratch, ovf_base + scap);
    ALLOC(o.top, 1);
  }
  ALLOC(bk.fcache, S * 64);
  ALLOC(e->d_tape, scap * e->group);
  ALLOC(e->d_tape_count, ME_GMAX);
  ALLOC(e->d_fills_acc, 1);
#ifdef ME_STAMPS
  ALLOC(bk.dbg, S * 24);
  (void)hipMemset(bk.dbg, 0, S * 24 * 8);
#endif
#undef ALLOC
  e->scratch_cap = ovf_base + scap;
  e->tape_cap = scap;
  e->slab = (uint32_t)slab;
  // initial book state
  hipStream_t st = e->stream;
  std::vector<SymState> ss(S);
  std::vector<uint32_t> gs(S);
  e->base_host.assign(cfg->base_price, cfg->base_price + S);
  const int64_t base_max = INT64_MAX - (int64_t)L + 1;  // base + L never overflows
  for (uint64_t i = 0; i < S; ++i) {
    memset(&ss[i], 0, sizeof(SymState));
    ss[i].base = cfg->base_price[i] > base_max ? base_max : cfg->base_price[i];
    ss[i].best_bid = -1;
    ss[i].best_ask = (int)L;
    ss[i].free_head = NIL;
    gs[i] = cfg->symbol_ids ? cfg->symbol_ids[i] : (uint32_t)i;
  }
  std::vector<FarDir> fd(2 * S);
  for (uint64_t i = 0; i < 2 * S; ++i) {
    fd[i].off = i * bk.fcap;
    fd[i].cap = bk.fcap;
    fd[i].pad = 0;
  }
  SeqState sq0[2];
  memset(sq0, 0, sizeof sq0);
  sq0[0].epoch = sq0[1].epoch = 1;  // old-order entries of epoch 0 (the zeroed table) read as empty
  bool ok = launch_init_levels(st, bk.levels, S * L) == hipSuccess &&
            zero_bucket_counts(e, st) &&
            hipMemsetAsync(bk.occ, 0, S * (L / 64) * 8, st) == hipSuccess &&
            hipMemsetAsync(bk.tend, 0, S * L, st) == hipSuccess &&
            launch_init_chunks(st, bk.chunks, nchunks) == hipSuccess &&
            hipMemsetAsync(bk.loc, 0xFF, ring * sizeof(uint32_t), st) == hipSuccess &&
            hipMemsetAsync(bk.old, 0, oldn * sizeof(OldEnt), st) == hipSuccess &&
            hipMemsetAsync(bk.hcount, 0, 8, st) == hipSuccess &&
            hipMemsetAsync(bk.stats, 0, ME_STATS * 8, st) == hipSuccess &&
            hipMemsetAsync(bk.far_ctl, 0, FC_N * 8, st) == hipSuccess &&
            hipMemcpyAsync(bk.fdir, fd.data(), fd.size() * sizeof(FarDir), hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemcpyAsync(bk.sq, sq0, sizeof sq0, hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemsetAsync(bk.fcache, 0xFF, S * 64 * sizeof(uint32_t), st) == hipSuccess &&
            hipMemsetAsync(bk.chunk_top, 0, 4, st) == hipSuccess && hipMemsetAsync(bk.err, 0, 4, st) == hipSuccess &&
            hipMemsetAsync(bk.cpool, 0, CP_N * sizeof(uint32_t), st) == hipSuccess &&
            hipMemcpyAsync(bk.sym, ss.data(), S * sizeof(SymState), hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemcpyAsync(gsym, gs.data(), S * 4, hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemsetAsync(e->d_tape_count, 0, 8 * ME_GMAX, st) == hipSuccess &&
            hipMemsetAsync(e->d_fills_acc, 0, 8, st) == hipSuccess &&
            hipStreamSynchronize(st) == hipSuccess;
  if (!ok) return bail(std::string("me_create: book init failed: ") + hipGetErrorString(hipGetLastError()));
  // host-batch pipeline: slots are allocated on first use
  {
    // 4G + 1: a synchronous-lag caller keeps submitting the group after next while the launch that
    // finishes an old group's tapes runs (3G + 1 serialised them: 372M vs 455M orders/s at G = 32)
    uint64_t H = cfg->host_slots ? cfg->host_slots : 4ull * e->group + 1;
    if (H > 4096) return bail("me_create: host_slots exceeds 4096");
    e->hs.resize(H);
    for (uint64_t k = H; k-- > 0;) e->free_slots.push_back((int)k);
    e->hcap = cfg->host_tape_cap ? cfg->host_tape_cap : 2 * n + 4096;
    e->oset_gen.assign(e->nsets, 0);
    if ((he = hipStreamCreateWithFlags(&e->s_h2d, hipStreamNonBlocking)) != hipSuccess)
      return bail(std::string("me_create: host pipeline stream: ") + hipGetErrorString(he));
  }
  // the configuration as resolved (me_get_config)
  e->cfg.max_chunks = nchunks;
  e->cfg.seq_ring = ring;
  e->cfg.far_levels = bk.fcap;
  e->cfg.batches_per_launch = e->group;
  e->cfg.host_slots = (uint32_t)e->hs.size();
  e->cfg.host_tape_cap = e->hcap;
  e->cfg.base_price = nullptr;
  e->cfg.symbol_ids = nullptr;
  return e;
}

extern "C" void me_destroy(me_engine* e) {
  if (!e) return;
  (void)hipSetDevice(e->dev);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  if (e->s_h2d) (void)hipStreamSynchronize(e->s_h2d);
  free_all(e);
  delete e;
}

extern "C" uint64_t me_fill_bound(const me_engine* e, size_t n) {
  return e ? (uint64_t)e->cfg.max_resting + 2ull * n : 0;
}

// Timing bookkeeping for one match launch (every e->timing-th launch records its own start / end).
static int timing_slot(me_engine* e, uint32_t orders, uint32_t batches, TimedLaunch& tl, bool& timed) {
  timed = e->timing > 0 && e->nlaunch % (uint64_t)e->timing == 0;
  tl = TimedLaunch{};
  e->nlaunch++;
  tl.idx = e->nbat;  // batches matched before this launch
  e->nbat += batches;
  if (timed) {
    while (e->ev_pool.size() < e->ev_used + 2) {
      hipEvent_t ev;
      HIP_TRY(hipEventCreate(&ev), "hipEventCreate");
      e->ev_pool.push_back(ev);
    }
    tl.m0 = e->ev_pool[e->ev_used++];
    tl.m1 = e->ev_pool[e->ev_used++];
    tl.orders = orders;
  }
  return ME_OK;
}

static BatchDev batch_dev(me_engine* e, const uint64_t* seq, const int64_t* px, const int32_t* qty,
                          const uint32_t* sym, const uint8_t* kind, uint32_t n, int oset) {
  const auto& o = e->os[oset];
  BatchDev bt{};
  bt.seq = seq;
  bt.px = px;
  bt.qty = qty;
  bt.sym = sym;
  bt.kind = kind;
  bt.n = n;
  bt.res = o.res;
  bt.fstart = o.fstart;
  bt.tile_sum = o.tile_sum;
  bt.scratch = o.scratch;
  bt.scratch_cap = e->scratch_cap;
  bt.scratch_top = o.top;
  bt.slab = e->slab;
  bt.ovf_base = (unsigned long long)(e->bk.S + 1) * e->slab;
  return bt;
}

// The seq-ring horizon check ahead of the match launch of a group (k_seq_sweep): flips the state
// index the match launches read.
static int seq_sweep(me_engine* e, const me_engine::Group& g) {
  const uint64_t* seq[ME_GMAX];
  const uint8_t* kind[ME_GMAX];
  uint32_t n[ME_GMAX];
  for (uint32_t k = 0; k < g.n; ++k) {
    seq[k] = g.b[k].seq;
    kind[k] = g.b[k].kind;
    n[k] = g.b[k].n;
  }
  // a small grid: the launch is on the stream before every match launch and usually decides "no
  // sweep" (a 1,024-workgroup grid cost ~0.7 us per batch at config 2); a due sweep loops over the pool
  hipError_t he = launch_seq_sweep(e->stream, e->bk, seq, kind, n, g.n, e->sq_idx, 64, e->launch_no);
  if (he != hipSuccess) return e->hip_fail(he, "seq sweep launch");
  e->sq_idx ^= 1u;
  e->bk.sq_idx = e->sq_idx;
  return ME_OK;
}

// ---- host slots ---------------------------------------------------------------------------
static size_t slot_in_bytes(uint64_t n) { return (size_t)n * (8 + 8 + 4 + 4 + 1); }
static size_t slot_res_off(const me_engine*) { return sizeof(SlotMeta); }
static size_t slot_tape_off(const me_engine* e) {
  return (sizeof(SlotMeta) + (size_t)e->cfg.max_batch * sizeof(me_order_result) + 63) & ~(size_t)63;
}
static size_t slot_out_bytes(const me_engine* e) { return slot_tape_off(e) + (size_t)e->hcap * sizeof(me_fill); }
// The packed SoA of an n-record batch at base p.
static void slot_soa(char* p, uint64_t n, uint64_t*& seq, int64_t*& px, int32_t*& qty, uint32_t*& sym,
                     uint8_t*& kind) {
  seq = (uint64_t*)p;
  px = (int64_t*)(p + 8 * n);
  qty = (int32_t*)(p + 16 * n);
  sym = (uint32_t*)(p + 20 * n);
  kind = (uint8_t*)(p + 24 * n);
}
// Where the tape job of a host batch writes: meta and tape into the slot's pinned block (device
// view), the finalised results into HBM.
static void slot_outputs(me_engine* e, HostSlot& h, me_fill*& tape, unsigned long long*& count,
                         me_order_result*& res, uint32_t*& err) {
  SlotMeta* m = (SlotMeta*)h.h_out_dev;  // the slot's pinned block as the device addresses it
  count = &m->count;
  err = &m->err;
  tape = (me_fill*)(h.h_out_dev + slot_tape_off(e));
  res = (me_order_result*)(h.h_out_dev + slot_res_off(e));
}
static int slot_alloc(me_engine* e, HostSlot& h) {
  if (h.h_in) return ME_OK;
  const size_t in = slot_in_bytes(e->cfg.max_batch) + 64, out = slot_out_bytes(e);
  HIP_TRY(hipHostMalloc((void**)&h.h_in, in, hipHostMallocDefault), "hipHostMalloc slot inputs");
  HIP_TRY(hipHostMalloc((void**)&h.h_out, out, hipHostMallocDefault), "hipHostMalloc slot outputs");
  HIP_TRY(hipMalloc((void**)&h.d_in, in), "hipMalloc slot inputs");
  HIP_TRY(hipHostGetDevicePointer((void**)&h.h_out_dev, h.h_out, 0), "hipHostGetDevicePointer");
  HIP_TRY(hipEventCreateWithFlags(&h.ev_in, hipEventDisableTiming), "hipEventCreate");
  HIP_TRY(hipEventCreateWithFlags(&h.ev_done, hipEventDisableTiming), "hipEventCreate");
  return ME_OK;
}
// After the launch whose tape jobs finished host slots[0..ns) (their meta and tapes are in pinned
// memory once it completes): the D2H stream waits for it and copies each slot's results into pinned
// memory. Nothing later on the engine stream writes those blocks before the slot is collected.
static int enqueue_host_d2h(me_engine* e, const int* slots, int ns) {
  // The tape job wrote each slot's count, error word, results and tape straight into its pinned
  // block (device-mapped): the launch's completion is the slots' completion. Measured against the
  // alternatives (tools/e2e_probe.py, config 2, G = 32, 129-193 slots): an HBM block moved by one
  // hipMemcpyAsync per slot (the runtime runs device-to-pinned copies as blit kernels, ~30 us of
  // host time per call) or by one copy kernel per launch gave the same 470-500M orders/s.
  for (int k = 0; k < ns; ++k) {
    HostSlot& h = e->hs[slots[k]];
    HIP_TRY(hipEventRecord(h.ev_done, e->stream), "hipEventRecord");
    h.state = 2;
  }
  return ME_OK;
}

// The bucket job of one pending batch (its bucket set, the output set whose counters it clears).
static void bucket_job(const me_engine* e, const me_engine::Pend& p, AuxBucket& J) {
  const auto& b = e->bu[p.bset];
  const auto& o = e->os[p.oset];
  J.sym = p.sym;
  J.seq = p.seq;
  J.px = p.px;
  J.qty = p.qty;
  J.kind = p.kind;
  J.n = p.n;
  J.bcnt = b.cnt;
  J.b_rec = b.rec;
  J.bres = o.res;
  J.bfstart = o.fstart;
  J.zero_tile_sum = o.tile_sum;
  J.zero_tiles = (p.n + TILE_TAPE - 1) / TILE_TAPE;
  J.zero_top = o.top;
}

// One launch of the pipelined register-ladder path: match group g_match (if any), bucket group nb
// (if any) and clear the counters its batches will use, compact g_tape's tapes (if any) — then the
// pipeline shifts by one group.
static int pipe_launch(me_engine* e, const me_engine::Group* nb) {
  BatchDev bt[ME_GMAX] = {};
  AuxDev ax{};
  const auto& gm = e->g_match;
  const auto& gt = e->g_tape;
  uint32_t orders = 0;
  uint64_t admitted = 0;
  for (uint32_t g = 0; g < gm.n; ++g) {
    const auto& pm = gm.b[g];
    admitted += pm.nadm;
    bt[g] = batch_dev(e, pm.seq, pm.px, pm.qty, pm.sym, pm.kind, pm.n, pm.oset);
    const auto& b = e->bu[pm.bset];
    bt[g].bcnt = b.cnt;
    bt[g].b_rec = b.rec;
    bt[g].bcap = BK_CAP;
    orders += pm.n;
  }
  ax.S = e->bk.S;
  ax.nwg = e->ncu;
  if (nb) {
    ax.nb = nb->n - nb->filled;
    for (uint32_t j = 0; j < ax.nb; ++j) bucket_job(e, nb->b[nb->filled + j], ax.b[j]);
  }
  ax.nt = gt.n;
  ax.fills_acc = e->d_fills_acc;
  bool host_tapes = false;
  for (uint32_t j = 0; j < gt.n; ++j) {
    const auto& o = e->os[gt.b[j].oset];
    AuxTape& J = ax.t[j];
    J.tn = gt.b[j].n;
    J.tile_sum = o.tile_sum;
    J.res = o.res;
    J.fstart = o.fstart;
    J.scratch = o.scratch;
    if (gt.b[j].slot >= 0) {
      host_tapes = true;
      slot_outputs(e, e->hs[gt.b[j].slot], J.tape, J.tape_count, J.hres, J.err_out);
      J.cap = e->hcap;
    } else {
      J.tape = e->d_tape + (size_t)j * e->tape_cap;
      J.tape_count = e->d_tape_count + j;
      J.cap = e->tape_cap;
    }
  }
  TimedLaunch tl{};
  bool timed = false;
  if (gm.n) {
    int rc = seq_sweep(e, gm);
    if (rc) return rc;
    rc = timing_slot(e, orders, gm.n, tl, timed);
    if (rc) return rc;
  }
  if ((e->reg_agg_auto || e->gw_cx_auto) && e->hot.agg_reg) {  // the hand-off rate since the last sample
    const unsigned long long p = *(volatile unsigned long long*)(e->pub_host + 1);  // (k_seq_sweep publishes it)
    const uint64_t k = p >> 32, h = p & 0xFFFFFFFFull;
    if (k > e->ho_k) {
      if (e->ho_k >= e->cx_from && (h - e->ho_h) * 16 > (k - e->ho_k) * (uint64_t)e->bk.S) {
        if (e->gw_cx_auto && !e->hot.ag.gw_cx) {  // cancels (config 5): the walk that covers them first
          e->hot.ag.gw_cx = 1u;
          e->cx_from = (uint64_t)e->launch_no + 1u;
        } else if (e->reg_agg_auto) {
          e->hot.agg_reg = false;
        }
      }
      e->ho_k = k;
      e->ho_h = h;
    }
  }
  if (gm.n || ax.nb || ax.nt) {  // (a group bucketed by early fills and no tapes due: nothing to launch)
    hipError_t he = launch_match_reg(e->stream, e->bk, bt, gm.n, ax, tl.m0, tl.m1, &e->hot);
    if (he != hipSuccess) return e->hip_fail(he, "pipelined match launch");
  }
  if (timed) e->timed.push_back(tl);
  if (gm.n) {
    e->adm_matched += admitted;
    e->adm_at[++e->launch_no % me_engine::ADM_RING] = e->adm_matched;
  }
  if (host_tapes) {
    int slots[ME_GMAX], ns = 0;
    for (uint32_t j = 0; j < gt.n; ++j)
      if (gt.b[j].slot >= 0) slots[ns++] = gt.b[j].slot;
    int rc = enqueue_host_d2h(e, slots, ns);
    if (rc) return rc;
  }
  e->g_tape = e->g_match;
  if (nb) {
    e->g_match = *nb;
    e->ngroup++;
  } else {
    e->g_match = me_engine::Group{};
  }
  return ME_OK;
}

// Bucket g_fill's batches [filled, n) now, on the engine stream, while nothing else is in flight: every
// launch that used their bucket and output sets is before it on the stream (a fork onto the side stream
// is joined back before the launch returns), and pipe_launch buckets only the batches after them. At the
// driver's shape (one group of 20 batches after a flush) the fill otherwise starts only at me_sync,
// after the host has submitted the whole group.
static int early_fill(me_engine* e) {
  auto& gf = e->g_fill;
  AuxDev ax{};
  ax.S = e->bk.S;
  ax.nwg = e->ncu;
  ax.nb = gf.n - gf.filled;
  for (uint32_t j = 0; j < ax.nb; ++j) bucket_job(e, gf.b[gf.filled + j], ax.b[j]);
  ax.fills_acc = e->d_fills_acc;
  bool done = false;
  hipError_t he = rc64::launch_fill_early(e->stream, e->bk, ax, done);
  if (he == hipSuccess && !done) he = launch_match_reg(e->stream, e->bk, nullptr, 0, ax, nullptr, nullptr, &e->hot);
  if (he != hipSuccess) return e->hip_fail(he, "early fill launch");
  gf.filled = gf.n;
  return ME_OK;
}

// Finish every submitted batch (the last one's outputs are then final).
static int flush_pipeline(me_engine* e) {
  if (e->g_fill.n) {  // a partial group goes out as it is
    // with early fills on and nothing in flight, the rest of the group through the light fill launch too:
    // the fill-only pipe_launch then has nothing to launch
    if (e->early_fill && e->g_fill.n > e->g_fill.filled && !e->g_match.n && !e->g_tape.n) {
      int rc = early_fill(e);
      if (rc) return rc;
    }
    int rc = pipe_launch(e, &e->g_fill);
    e->g_fill = me_engine::Group{};
    if (rc) return rc;
  }
  while (e->g_match.n || e->g_tape.n) {
    int rc = pipe_launch(e, nullptr);
    if (rc) return rc;
  }
  return ME_OK;
}

// Enqueue a device-resident batch.
static int enqueue_batch(me_engine* e, const uint64_t* seq, const int64_t* px, const int32_t* qty,
                         const uint32_t* sym, const uint8_t* kind, uint32_t n, uint32_t nadm, int slot = -1) {
  e->last_host = slot >= 0;
  if (e->bucketed) {
    auto& gf = e->g_fill;
    const uint32_t pos = gf.n;
    me_engine::Pend& nb = gf.b[pos];
    nb.valid = true;
    nb.seq = seq;
    nb.px = px;
    nb.qty = qty;
    nb.sym = sym;
    nb.kind = kind;
    nb.n = n;
    nb.oset = (int)((e->ngroup % 3) * e->group + pos);
    nb.bset = (int)((e->ngroup % 2) * e->group + pos);
    nb.slot = slot;
    nb.nadm = nadm;
    const uint64_t gen = ++e->oset_gen[nb.oset];
    if (slot >= 0) {
      e->hs[slot].oset = nb.oset;
      e->hs[slot].oset_gen = gen;
    }
    gf.n = pos + 1;
    e->last_set = nb.oset;
    e->last_tape = (int)pos;
    e->last_n = n;
    e->lastg.n = pos + 1;
    e->lastg.oset[pos] = nb.oset;
    e->lastg.tape[pos] = (int)pos;
    e->lastg.bn[pos] = n;
    if (gf.n == e->group) {
      int rc = pipe_launch(e, &gf);
      gf = me_engine::Group{};
      if (rc) return rc;
    } else if (e->early_fill && gf.n - gf.filled >= e->early_fill && !e->g_match.n && !e->g_tape.n) {
      int rc = early_fill(e);
      if (rc) return rc;
    }
    return ME_OK;
  }
  hipStream_t st = e->stream;
  auto& sl = e->sb;
  const int oset = (int)(e->ngroup++ % (uint64_t)e->nsets);
  const auto& o = e->os[oset];
  TimedLaunch tl{};
  bool timed = false;
  int rc = timing_slot(e, n, 1u, tl, timed);
  if (rc) return rc;
  const uint32_t S = e->bk.S;
  const uint32_t ntiles_tape = (n + TILE_TAPE - 1) / TILE_TAPE;
  // grouping: the stable counting sort by symbol
  const uint32_t* kin = sym;
  const uint32_t* iin = nullptr;
  uint32_t* run_table = e->passes == 1 ? sl.bin_start : nullptr;
  int shift = 0;
  {
    me_engine::Group g1;
    g1.n = 1;
    g1.b[0].seq = seq;
    g1.b[0].kind = kind;
    g1.b[0].n = n;
    int rc2 = seq_sweep(e, g1);
    if (rc2) return rc2;
  }
  for (int p = 0; p < e->passes; ++p) {
    hipError_t he = launch_sort_pass(st, kin, iin, n, S, shift, e->dbits[p], sl.hist,
                                     sl.tot + ((size_t)p << MAX_DIGIT_BITS), sl.keys[p], sl.idx[p],
                                     p == 0 ? o.tile_sum : nullptr, p == 0 ? ntiles_tape : 0, o.top,
                                     p == e->passes - 1 ? run_table : nullptr, p == 0 ? seq : nullptr, kind, e->bk.err);
    if (he != hipSuccess) return e->hip_fail(he, "grouping sort launch");
    kin = sl.keys[p];
    iin = sl.idx[p];
    shift += e->dbits[p];
  }
  BatchDev bt = batch_dev(e, seq, px, qty, sym, kind, n, oset);
  bt.skeys = kin;
  bt.perm = iin;
  bt.bin_start = run_table;  // bins are symbols: the run table
  // timing: the launch itself records start/end (hipExtLaunchKernelGGL), no marker packets
  const uint64_t gen = ++e->oset_gen[oset];
  hipError_t he = launch_match(st, e->bk, bt, tl.m0, tl.m1, e->hot);
  if (he != hipSuccess) return e->hip_fail(he, "match launch");
  e->adm_matched += nadm;
  e->adm_at[++e->launch_no % me_engine::ADM_RING] = e->adm_matched;
  if (slot >= 0) {
    HostSlot& h = e->hs[slot];
    h.oset = oset;
    h.oset_gen = gen;
    me_fill* tape;
    unsigned long long* cnt;
    me_order_result* hres;
    uint32_t* eo;
    slot_outputs(e, h, tape, cnt, hres, eo);
    he = launch_tape(st, bt, tape, e->hcap, cnt, e->d_fills_acc, e->bk.err, hres, eo);
  } else {
    he = launch_tape(st, bt, e->d_tape, e->tape_cap, e->d_tape_count, e->d_fills_acc, e->bk.err, nullptr, nullptr);
  }
  if (he != hipSuccess) return e->hip_fail(he, "tape launch");
  if (timed) e->timed.push_back(tl);
  if (slot >= 0) {
    rc = enqueue_host_d2h(e, &slot, 1);
    if (rc) return rc;
  }
  e->last_set = oset;
  e->last_tape = 0;
  e->last_n = n;
  e->lastg.n = 1;
  e->lastg.oset[0] = oset;
  e->lastg.tape[0] = 0;
  e->lastg.bn[0] = n;
  return ME_OK;
}

static int check_err_bits(me_engine* e, uint32_t w) {
  if (w) {
    std::string m = "device pool overflow/inconsistency (bits=" + std::to_string(w) + "):";
    if (w & ERR_CHUNK_OOM) m += " chunk pool exhausted (raise max_chunks);";
    if (w & ERR_SCRATCH_OOM) m += " fill scratch/tape bound exceeded (raise max_resting);";
    if (w & ERR_INCONSISTENT) m += " book inconsistency;";
    if (w & ERR_FAR_OOM) m += " far arena exhausted (internal bound broken);";
    if (w & ERR_OLD_OOM) m += " old-order table full (raise max_resting);";
    if (w & ERR_SEQ_ORDER) m += " seqs not ascending (API precondition: a NEW record's seq above every earlier seq, a CANCEL's at least the previous one);";
    if (w & ERR_SEQ_SPAN) m += " one launch group spans the whole seq ring (raise seq_ring);";
    const int code = (w & (ERR_SEQ_ORDER | ERR_SEQ_SPAN)) && !(w & ~(ERR_SEQ_ORDER | ERR_SEQ_SPAN)) ? ME_E_INVALID
                                                                                                    : ME_E_CAPACITY;
    e->fail(code, m);
    e->failed = true;  // sticky: the books may no longer be what the stream says
    return code;
  }
  return ME_OK;
}

static int check_err_word(me_engine* e) {
  uint32_t w = 0;
  HIP_TRY(hipMemcpy(&w, e->bk.err, 4, hipMemcpyDeviceToHost), "read error word");
  return check_err_bits(e, w);
}

// Records of kind LIMIT-new (neither the MARKET nor the CANCEL bit), eight kind bytes per step.
static uint64_t count_limits(const uint8_t* kind, size_t n) {
  uint64_t other = 0;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, kind + i, 8);
    const uint64_t x = (w >> 2) & 0x0303030303030303ull;  // the MARKET and CANCEL bits of each byte
    other += (uint64_t)__builtin_popcountll((x | (x >> 1)) & 0x0101010101010101ull);
  }
  for (; i < n; ++i) other += (kind[i] & 0x0Cu) != 0u;
  return (uint64_t)n - other;
}

// Upper bound on the resting orders once every accepted record has been matched.
static uint64_t admission_bound(const me_engine* e) {
  uint64_t b = e->ovr_resting + (e->adm_total - e->ovr_adm);
  const unsigned long long v = __atomic_load_n(e->pub_host, __ATOMIC_ACQUIRE);
  const uint32_t k = (uint32_t)(v >> 32);
  const uint64_t r = v & 0xFFFFFFFFull;
  if (r != 0xFFFFFFFFull && e->launch_no - k < me_engine::ADM_RING)
    b = std::min<uint64_t>(b, r + (e->adm_total - e->adm_at[k % me_engine::ADM_RING]));
  return b;
}

// Admission of an n-record batch (me_config.max_resting). Usually one pinned read. When the bound is
// too high the caller waits while two or more match launches are still ahead of the published count
// (the device stays busy meanwhile), then takes an exact count (flush + sync). A batch that still
// does not fit is refused with ME_E_CAPACITY before anything of it is enqueued: the books are
// untouched and the engine stays usable (the error is not sticky).
static int admit(me_engine* e, uint64_t n, bool commit = true) {  // n: records of the batch that may rest
  const uint64_t cap = e->cfg.max_resting;
  if (admission_bound(e) + n > cap) {
    for (;;) {
      const unsigned long long v = __atomic_load_n(e->pub_host, __ATOMIC_ACQUIRE);
      if (admission_bound(e) + n <= cap) break;
      if (e->launch_no - (uint32_t)(v >> 32) < 2u || hipStreamQuery(e->stream) != hipErrorNotReady) {
        // exact count of what the launches so far matched; batches still waiting for their match
        // launch stay in the bound, so a group being filled is not cut short unless it must be
        auto exact = [&]() -> int {
          HIP_TRY(hipStreamSynchronize(e->stream), "hipStreamSynchronize");
          int rc2 = check_err_word(e);
          if (rc2) return rc2;
          uint64_t r = 0;
          HIP_TRY(hipMemcpy(&r, e->bk.stats + ST_RESTING, 8, hipMemcpyDeviceToHost), "D2H resting count");
          e->ovr_resting = r;
          e->ovr_adm = e->adm_matched;
          e->adm_syncs++;
          return ME_OK;
        };
        int rc = exact();
        if (rc) return rc;
        if (admission_bound(e) + n <= cap) break;
        rc = flush_pipeline(e);  // the pending batches matched too
        if (rc) return rc;
        rc = exact();
        if (rc) return rc;
        const uint64_t r = e->ovr_resting;
        if (r + n > cap) {
          e->err = "batch refused: " + std::to_string(r) + " resting orders + " + std::to_string(n) +
                   " records could exceed max_resting (" + std::to_string(cap) + "); the books are unchanged";
          return ME_E_CAPACITY;
        }
        break;
      }
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
  if (commit) e->adm_total += n;
  return ME_OK;
}

extern "C" int me_admission_check(me_engine* e, uint64_t n_rest, int* ok) {
  if (!e || !ok) return ME_E_INVALID;
  *ok = 0;
  if (e->failed) return ME_E_STATE;
  HIP_TRY(hipSetDevice(e->dev), "hipSetDevice");
  const int rc = admit(e, n_rest, false);
  if (rc == ME_E_CAPACITY) return ME_OK;  // would be refused: *ok stays 0
  if (rc) return rc;
  *ok = 1;
  return ME_OK;
}

extern "C" int me_admission_read(me_engine* e, uint64_t* resting, uint64_t* bound, uint64_t* exact_counts) {
  if (!e) return ME_E_INVALID;
  HIP_TRY(hipSetDevice(e->dev), "hipSetDevice");
  if (resting) {
    uint64_t r = 0;
    HIP_TRY(hipStreamSynchronize(e->stream), "hipStreamSynchronize");
    HIP_TRY(hipMemcpy(&r, e->bk.stats + ST_RESTING, 8, hipMemcpyDeviceToHost), "D2H resting count");
    *resting = r;
  }
  if (bound) *bound = admission_bound(e);
  if (exact_counts) *exact_counts = e->adm_syncs;
  return ME_OK;
}

extern "C" int me_submit_batch_device(me_engine* e, const me_order_soa* b, size_t n) {
  return me_submit_device_limits(e, b, n, n);  // the kinds are on the device: every record counts as a LIMIT
}

extern "C" int me_submit_device_limits(me_engine* e, const me_order_soa* b, size_t n, uint64_t n_limits) {
  if (!e) return ME_E_INVALID;
  if (e->failed) return ME_E_STATE;
  if (!b || !b->seq || !b->price_q4 || !b->qty || !b->symbol || !b->kind) return e->fail(ME_E_INVALID, "null batch");
  if (n == 0) {
    e->last_n = 0;
    return ME_OK;
  }
  if (n > e->cfg.max_batch) return e->fail(ME_E_INVALID, "batch larger than max_batch");
  HIP_TRY(hipSetDevice(e->dev), "hipSetDevice");
  const uint64_t nl = std::min<uint64_t>(n_limits, n);
  const int rc = admit(e, nl);
  if (rc) return rc;
  return enqueue_batch(e, b->seq, b->price_q4, b->qty, b->symbol, b->kind, (uint32_t)n, (uint32_t)nl);
}

extern "C" int me_sync(me_engine* e) {
  if (!e) return ME_E_INVALID;
  HIP_TRY(hipSetDevice(e->dev), "hipSetDevice");
  if (!e->failed) {
    int rc = flush_pipeline(e);
    if (rc) return rc;
  }
  // the error word rides behind the last launch into pinned memory: one stream synchronisation, not a
  // second synchronous round trip after it
  uint32_t* w = reinterpret_cast<uint32_t*>(e->pub_host + 2);
  HIP_TRY(hipMemcpyAsync(w, e->bk.err, 4, hipMemcpyDeviceToHost, e->stream), "D2H error word");
  HIP_TRY(hipStreamSynchronize(e->stream), "hipStreamSynchronize");
  if (e->failed) return ME_E_STATE;
  return check_err_bits(e, *(volatile uint32_t*)w);
}

extern "C" int me_fetch_outputs(me_engine* e, me_fill* out_fills, size_t fills_cap, size_t* n_fills,
                                me_order_result* out_results, size_t n_results) {
  if (!e) return ME_E_INVALID;
  if (e->last_host) return e->fail(ME_E_INVALID, "the most recent batch was a host batch: its outputs come from me_collect");
  int rc = me_sync(e);
  if (rc) return rc;
  unsigned long long cnt = 0;
  if (e->last_n)
    HIP_TRY(hipMemcpy(&cnt, e->d_tape_count + e->last_tape, 8, hipMemcpyDeviceToHost), "read tape count");
  if (n_fills) *n_fills = (size_t)cnt;
  if (out_results && n_results) {
    if (n_results > e->last_n) return e->fail(ME_E_INVALID, "n_results exceeds last batch size");
    HIP_TRY(hipMemcpy(out_results, e->os[e->last_set].res, n_results * sizeof(me_order_result), hipMemcpyDeviceToHost),
            "D2H results");
  }
  if (out_fills && cnt) {
    if (cnt > fills_cap) return e->fail(ME_E_INVALID, "fills_cap smaller than the tape");
    HIP_TRY(hipMemcpy(out_fills, e->d_tape + (size_t)e->last_tape * e->tape_cap, cnt * sizeof(me_fill),
                      hipMemcpyDeviceToHost), "D2H tape");
  }
  return ME_OK;
}

extern "C" uint32_t me_last_group_size(const me_engine* e) { return e ? e->lastg.n : 0u; }

extern "C" int me_fetch_group_outputs(me_engine* e, uint32_t k, me_fill* out_fills, size_t fills_cap, size_t* n_fills,
                                      me_order_result* out_results, size_t n_results) {
  if (!e) return ME_E_INVALID;
  if (e->last_host) return e->fail(ME_E_INVALID, "the most recent batch was a host batch: its outputs come from me_collect");
  int rc = me_sync(e);
  if (rc) return rc;
  if (k >= e->lastg.n) return e->fail(ME_E_INVALID, "batch index outside the last launch group");
  unsigned long long cnt = 0;
  HIP_TRY(hipMemcpy(&cnt, e->d_tape_count + e->lastg.tape[k], 8, hipMemcpyDeviceToHost), "read tape count");
  if (n_fills) *n_fills = (size_t)cnt;
  if (out_results && n_results) {
    if (n_results > e->lastg.bn[k]) return e->fail(ME_E_INVALID, "n_results exceeds the batch size");
    HIP_TRY(hipMemcpy(out_results, e->os[e->lastg.oset[k]].res, n_results * sizeof(me_order_result),
                      hipMemcpyDeviceToHost),
            "D2H results");
  }
  if (out_fills && cnt) {
    if (cnt > fills_cap) return e->fail(ME_E_INVALID, "fills_cap smaller than the tape");
    HIP_TRY(hipMemcpy(out_fills, e->d_tape + (size_t)e->lastg.tape[k] * e->tape_cap, cnt * sizeof(me_fill),
                      hipMemcpyDeviceToHost),
            "D2H tape");
  }
  return ME_OK;
}

// ---- host-batch pipeline (include/me_engine.h) ----------------------------------------------
// A free slot for the next submit; the held slot (last collected) goes back only when no other is free.
static bool has_free_slot(me_engine* e) {
  if (e->free_slots.empty() && e->held_slot >= 0) {
    e->free_slots.push_back(e->held_slot);
    e->held_slot = -1;
  }
  return !e->free_slots.empty();
}

static int slots_busy(me_engine* e) {
  uint64_t oldest = UINT64_MAX;
  for (auto& kv : e->by_ticket) oldest = std::min(oldest, kv.first);
  return e->fail(ME_E_STATE, "all host slots busy: collect ticket " + std::to_string(oldest) + " first");
}

extern "C" int me_host_inputs(me_engine* e, size_t n, me_order_soa_w* out) {
  if (!e || !out) return ME_E_INVALID;
  if (n == 0 || n > e->cfg.max_batch) return e->fail(ME_E_INVALID, "me_host_inputs: n must be in [1, max_batch]");
  if (!has_free_slot(e)) return slots_busy(e);
  HostSlot& h = e->hs[e->free_slots.back()];
  HIP_TRY(hipSetDevice(e->dev), "hipSetDevice");
  int rc = slot_alloc(e, h);
  if (rc) return rc;
  // the slot's previous H2D may still be reading the staging buffer (its batch was collected, so it
  // finished long ago, but the event is cheap to wait on)
  HIP_TRY(hipEventSynchronize(h.ev_in), "hipEventSynchronize");
  slot_soa(h.h_in, n, out->seq, out->price_q4, out->qty, out->symbol, out->kind);
  return ME_OK;
}

extern "C" int me_host_reserve(me_engine* e, uint32_t nslots) {
  if (!e) return ME_E_INVALID;
  HIP_TRY(hipSetDevice(e->dev), "hipSetDevice");
  const size_t k = nslots ? std::min<size_t>(nslots, e->hs.size()) : e->hs.size();
  for (size_t i = 0; i < k; ++i) {
    int rc = slot_alloc(e, e->hs[i]);
    if (rc) return rc;
  }
  return ME_OK;
}

extern "C" int me_submit_host(me_engine* e, const me_order_soa* b, size_t n, uint64_t* ticket) {
  if (!e) return ME_E_INVALID;
  if (e->failed) return ME_E_STATE;
  if (!b || !b->seq || !b->price_q4 || !b->qty || !b->symbol || !b->kind) return e->fail(ME_E_INVALID, "null batch");
  if (n == 0 || n > e->cfg.max_batch) return e->fail(ME_E_INVALID, "host batch size must be in [1, max_batch]");
  if (!has_free_slot(e)) return slots_busy(e);
  const int slot = e->free_slots.back();
  HostSlot& h = e->hs[slot];
  HIP_TRY(hipSetDevice(e->dev), "hipSetDevice");
  const uint64_t n_rest = count_limits(b->kind, n);  // only LIMIT records can rest (kinds are on the host)
  int rc = admit(e, n_rest);
  if (rc) return rc;
  rc = slot_alloc(e, h);
  if (rc) return rc;
  uint64_t* seq;
  int64_t* px;
  int32_t* qty;
  uint32_t* sym;
  uint8_t* kind;
  slot_soa(h.h_in, n, seq, px, qty, sym, kind);
  if (b->seq != seq || b->price_q4 != px || b->qty != qty || b->symbol != sym || b->kind != kind) {
    HIP_TRY(hipEventSynchronize(h.ev_in), "hipEventSynchronize");
    const CopyPool::Piece cols[5] = {{seq, b->seq, 8 * n}, {px, b->price_q4, 8 * n}, {qty, b->qty, 4 * n},
                                     {sym, b->symbol, 4 * n}, {kind, b->kind, n}};
    if (n < 16384) {
      for (const auto& c : cols) memcpy(c.dst, c.src, c.bytes);
    } else {  // 64-KB pieces over the copy threads
      if (!e->copy_pool) {
        const char* v = getenv("ME_COPY_THREADS");
        const int nt = v ? std::max(1, std::min(32, atoi(v))) : 4;
        e->copy_pool.reset(new CopyPool(nt));
      }
      std::vector<CopyPool::Piece> pieces;
      for (const auto& c : cols)
        for (size_t o = 0; o < c.bytes; o += 65536)
          pieces.push_back({(char*)c.dst + o, (const char*)c.src + o, std::min<size_t>(65536, c.bytes - o)});
      e->copy_pool->run(pieces);
    }
  }
  // one H2D of the packed batch on the H2D stream; the engine stream waits for it before the launch
  // that buckets (or sorts) the batch
  HIP_TRY(hipMemcpyAsync(h.d_in, h.h_in, slot_in_bytes(n), hipMemcpyHostToDevice, e->s_h2d), "H2D host batch");
  HIP_TRY(hipEventRecord(h.ev_in, e->s_h2d), "hipEventRecord");
  HIP_TRY(hipStreamWaitEvent(e->stream, h.ev_in, 0), "hipStreamWaitEvent");
  h.ticket = e->next_ticket;
  h.n = (uint32_t)n;
  h.state = 1;
  h.big.clear();
  slot_soa(h.d_in, n, seq, px, qty, sym, kind);
  e->free_slots.pop_back();
  e->by_ticket[h.ticket] = slot;
  rc = enqueue_batch(e, seq, px, qty, sym, kind, (uint32_t)n, (uint32_t)n_rest, slot);
  if (rc) return rc;
  if (ticket) *ticket = e->next_ticket;
  e->next_ticket++;
  return ME_OK;
}

extern "C" int me_collect(me_engine* e, uint64_t ticket, const me_fill** fills, size_t* n_fills,
                          const me_order_result** results, size_t* n_results) {
  if (!e) return ME_E_INVALID;
  auto it = e->by_ticket.find(ticket);
  if (it == e->by_ticket.end()) return e->fail(ME_E_INVALID, "unknown or already collected ticket");
  const int slot = it->second;
  HostSlot& h = e->hs[slot];
  HIP_TRY(hipSetDevice(e->dev), "hipSetDevice");
  if (h.state == 1) {  // its group has not reached the tape job yet
    if (e->failed) return ME_E_STATE;
    int rc = flush_pipeline(e);
    if (rc) return rc;
  }
  if (h.state != 2) return e->fail(ME_E_STATE, "host batch outputs were never enqueued");
  HIP_TRY(hipEventSynchronize(h.ev_done), "hipEventSynchronize");
  h.state = 0;  // collected: the outputs stay readable until the next collect releases the slot
  e->by_ticket.erase(it);
  if (e->held_slot >= 0) e->free_slots.push_back(e->held_slot);
  e->held_slot = slot;
  const SlotMeta* m = (const SlotMeta*)h.h_out;
  {
    int rc = check_err_bits(e, m->err);
    if (rc) return rc;
  }
  const uint64_t cnt = m->count;
  me_fill* tape = (me_fill*)(h.h_out + slot_tape_off(e));
  if (cnt > e->hcap) {  // past the slot: the spill from scratch
    if (e->oset_gen[h.oset] != h.oset_gen) {  // this batch's output is lost; the books are intact (not sticky)
      e->err = "host batch tape (" + std::to_string(cnt) + " fills) outgrew host_tape_cap and its scratch was "
               "reused before me_collect: raise host_tape_cap or collect within 3 launch groups";
      return ME_E_CAPACITY;
    }
    const size_t extra = (size_t)(cnt - e->hcap);
    if (extra > e->spill_cap) {
      if (e->d_spill) HIP_TRY(hipFree(e->d_spill), "hipFree");
      e->d_spill = nullptr;
      e->spill_cap = 0;
      HIP_TRY(hipMalloc((void**)&e->d_spill, extra * sizeof(me_fill)), "hipMalloc spill");
      e->spill_cap = extra;
    }
    const auto& o = e->os[h.oset];
    hipError_t he = launch_tape_spill(e->stream, (const me_order_result*)(h.h_out_dev + slot_res_off(e)), o.fstart,
                                      h.n, o.scratch, e->hcap,
                                      e->d_spill);
    if (he != hipSuccess) return e->hip_fail(he, "spill launch");
    HIP_TRY(hipStreamSynchronize(e->stream), "hipStreamSynchronize");
    h.big.resize(cnt);
    memcpy(h.big.data(), tape, e->hcap * sizeof(me_fill));
    HIP_TRY(hipMemcpy(h.big.data() + e->hcap, e->d_spill, extra * sizeof(me_fill), hipMemcpyDeviceToHost),
            "D2H spill");
    tape = h.big.data();
  }
  if (fills) *fills = tape;
  if (n_fills) *n_fills = (size_t)cnt;
  if (results) *results = (const me_order_result*)(h.h_out + slot_res_off(e));
  if (n_results) *n_results = h.n;
  return ME_OK;
}

extern "C" int me_submit_batch(me_engine* e, const me_order_soa* b, size_t n, me_fill* out_fills,
                               size_t fills_cap, size_t* n_fills, me_order_result* out_results) {
  if (!e) return ME_E_INVALID;
  if (e->failed) return ME_E_STATE;
  if (n_fills) *n_fills = 0;
  if (n == 0) return ME_OK;
  uint64_t t = 0;
  int rc = me_submit_host(e, b, n, &t);
  if (rc) return rc;
  const me_fill* f = nullptr;
  const me_order_result* r = nullptr;
  size_t nf = 0, nr = 0;
  rc = me_collect(e, t, &f, &nf, &r, &nr);
  if (rc) return rc;
  if (n_fills) *n_fills = nf;
  if (out_results) memcpy(out_results, r, nr * sizeof(me_order_result));
  if (out_fills && nf) {
    if (nf > fills_cap) return e->fail(ME_E_INVALID, "fills_cap smaller than the tape");
    memcpy(out_fills, f, nf * sizeof(me_fill));
  }
  return ME_OK;
}

extern "C" int me_get_config(const me_engine* e, me_config* out) {
  if (!e || !out) return ME_E_INVALID;
  *out = e->cfg;
  return ME_OK;
}

extern "C" int me_copy_tape_device(me_engine* e, void* dst, size_t cap_fills, size_t* n_fills) {
  if (!e) return ME_E_INVALID;
  if (e->last_host) return e->fail(ME_E_INVALID, "the most recent batch was a host batch: its outputs come from me_collect");
  int rc = me_sync(e);
  if (rc) return rc;
  unsigned long long cnt = 0;
  if (e->last_n)
    HIP_TRY(hipMemcpy(&cnt, e->d_tape_count + e->last_tape, 8, hipMemcpyDeviceToHost), "read tape count");
  if (n_fills) *n_fills = (size_t)cnt;
  if (cnt > cap_fills) return e->fail(ME_E_INVALID, "cap_fills smaller than the tape");
  if (cnt) HIP_TRY(hipMemcpyAsync(dst, e->d_tape + (size_t)e->last_tape * e->tape_cap, cnt * sizeof(me_fill),
                                  hipMemcpyDeviceToDevice, e->stream),
                   "D2D tape");
  return ME_OK;
}

extern "C" int me_copy_results_device(me_engine* e, void* dst, size_t n_results) {
  if (!e) return ME_E_INVALID;
  if (e->last_host) return e->fail(ME_E_INVALID, "the most recent batch was a host batch: its outputs come from me_collect");
  if (e->failed) return ME_E_STATE;
  if (n_results > e->last_n) return e->fail(ME_E_INVALID, "n_results exceeds last batch size");
  if (n_results && !dst) return e->fail(ME_E_INVALID, "null destination");
  HIP_TRY(hipSetDevice(e->dev), "hipSetDevice");
  {
    int rc = flush_pipeline(e);
    if (rc) return rc;
  }
  if (n_results)
    HIP_TRY(hipMemcpyAsync(dst, e->os[e->last_set].res, n_results * sizeof(me_order_result), hipMemcpyDeviceToDevice,
                           e->stream),
            "D2D results");
  return ME_OK;
}

extern "C" int me_device_alloc(me_engine* e, size_t bytes, void** dptr) {
  if (!e || !dptr) return ME_E_INVALID;
  HIP_TRY(hipSetDevice(e->dev), "hipSetDevice");
  HIP_TRY(hipMalloc(dptr, std::max<size_t>(bytes, 1)), "hipMalloc");
  e->user_allocs.push_back(*dptr);
  return ME_OK;
}

extern "C" int me_device_free(me_engine* e, void* dptr) {
  if (!e) return ME_E_INVALID;
  auto it = std::find(e->user_allocs.begin(), e->user_allocs.end(), dptr);
  if (it == e->user_allocs.end()) return e->fail(ME_E_INVALID, "pointer not allocated by me_device_alloc");
  e->user_allocs.erase(it);
  HIP_TRY(hipSetDevice(e->dev), "hipSetDevice");
  if (!e->failed) {  // a submitted batch may still live in this buffer: finish it first
    int rc = flush_pipeline(e);
    if (rc) return rc;
  }
  HIP_TRY(hipStreamSynchronize(e->stream), "hipStreamSynchronize");
  HIP_TRY(hipFree(dptr), "hipFree");
  return ME_OK;
}

extern "C" int me_memcpy_h2d(me_engine* e, void* dst, const void* src, size_t bytes) {
  if (!e) return ME_E_INVALID;
  HIP_TRY(hipSetDevice(e->dev), "hipSetDevice");
  HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice), "hipMemcpy H2D");
  return ME_OK;
}

extern "C" int me_set_stream(me_engine* e, void* s) {
  if (!e) return ME_E_INVALID;
  if (!e->failed) {
    int rc = flush_pipeline(e);
    if (rc) return rc;
  }
  HIP_TRY(hipStreamSynchronize(e->stream), "hipStreamSynchronize");
  e->stream = s ? (hipStream_t)s : e->own_stream;
  return ME_OK;
}

// ---- book inspection (GetOrderBook / test dumps): device snapshot kernel (me_snapshot.hip) ------
// Run k_book_snapshot over syms[0..nsym) (host array), depth levels per side, orders into regions of
// ocap per (symbol, side) (0: levels only). Results stay in e->snap.
static int run_snapshot(me_engine* e, const uint32_t* syms, uint32_t nsym, uint32_t depth, uint64_t ocap) {
  auto& sb = e->snap;
  auto grow = [&](void** p, size_t& cap, size_t need, size_t elem) -> int {
    if (need <= cap) return ME_OK;
    if (*p) HIP_TRY(hipFree(*p), "hipFree");
    *p = nullptr;
    cap = 0;
    HIP_TRY(hipMalloc(p, std::max<size_t>(need, 1) * elem), "hipMalloc snapshot");
    cap = need;
    return ME_OK;
  };
  int rc;
  if ((rc = grow((void**)&sb.sym, sb.sym_cap, nsym, 4)) || (rc = grow((void**)&sb.nlv, sb.n_cap, 2ull * nsym, 4)) ||
      (rc = grow((void**)&sb.nord, sb.nord_cap, 2ull * nsym, 8)) ||
      (rc = grow((void**)&sb.lv, sb.lv_cap, 2ull * nsym * depth, sizeof(me_level))) ||
      (rc = grow((void**)&sb.ord, sb.ord_cap, 2ull * nsym * ocap, sizeof(me_book_entry))) ||
      (rc = grow((void**)&sb.err, sb.err_cap, 1, 4)))
    return rc;
  HIP_TRY(hipMemcpyAsync(sb.sym, syms, nsym * 4ull, hipMemcpyHostToDevice, e->stream), "H2D snapshot symbols");
  HIP_TRY(hipMemsetAsync(sb.err, 0, 4, e->stream), "hipMemset");
  SnapReq rq{};
  rq.sym = sb.sym;
  rq.nsym = nsym;
  rq.depth = depth;
  rq.lv = sb.lv;
  rq.nlv = sb.nlv;
  rq.ord = ocap ? sb.ord : nullptr;
  rq.ocap = ocap;
  rq.nord = sb.nord;
  rq.err = sb.err;
  hipError_t he = launch_book_snapshot(e->stream, e->bk, rq);
  if (he != hipSuccess) return e->hip_fail(he, "snapshot launch");
  uint32_t bad = 0;
  HIP_TRY(hipMemcpyAsync(&bad, sb.err, 4, hipMemcpyDeviceToHost, e->stream), "D2H snapshot error");
  HIP_TRY(hipStreamSynchronize(e->stream), "hipStreamSynchronize");
  if (bad) return e->fail(ME_E_STATE, "corrupt FIFO chain");
  return ME_OK;
}

extern "C" int me_book_orders(me_engine* e, uint32_t symbol, uint32_t depth, me_book_entry* bids, size_t bids_cap,
                              size_t* n_bids, me_book_entry* asks, size_t asks_cap, size_t* n_asks,
                              me_level* bid_levels, me_level* ask_levels, size_t* n_bid_levels,
                              size_t* n_ask_levels) {
  if (!e) return ME_E_INVALID;
  if (symbol >= e->bk.S) return e->fail(ME_E_INVALID, "symbol out of range");
  int rc = me_sync(e);
  if (rc) return rc;
  const bool want_orders = bids || asks || n_bids || n_asks;
  uint64_t ocap = 0;
  SymState ss;
  HIP_TRY(hipMemcpy(&ss, e->bk.sym + symbol, sizeof ss, hipMemcpyDeviceToHost), "D2H symbol");
  if (want_orders) ocap = std::max<uint64_t>(ss.resting, 1);  // bounds either side's orders
  // a side has at most L window levels and its far levels: any larger depth (0xFFFFFFFF: the whole book)
  // is that
  depth = (uint32_t)std::min<uint64_t>(depth, (uint64_t)e->bk.L + std::max(ss.nfar[0], ss.nfar[1]));
  if (!depth) {
    if (n_bids) *n_bids = 0;
    if (n_asks) *n_asks = 0;
    if (n_bid_levels) *n_bid_levels = 0;
    if (n_ask_levels) *n_ask_levels = 0;
    return ME_OK;
  }
  if ((rc = run_snapshot(e, &symbol, 1, depth, ocap))) return rc;
  auto& sb = e->snap;
  uint32_t nl[2];
  unsigned long long no[2];
  HIP_TRY(hipMemcpy(nl, sb.nlv, sizeof nl, hipMemcpyDeviceToHost), "D2H snapshot counts");
  HIP_TRY(hipMemcpy(no, sb.nord, sizeof no, hipMemcpyDeviceToHost), "D2H snapshot counts");
  me_level* lo[2] = {bid_levels, ask_levels};
  size_t* nlo[2] = {n_bid_levels, n_ask_levels};
  me_book_entry* oo[2] = {bids, asks};
  const size_t ocaps[2] = {bids_cap, asks_cap};
  size_t* noo[2] = {n_bids, n_asks};
  for (int k = 0; k < 2; ++k) {
    if (nlo[k]) *nlo[k] = nl[k];
    if (lo[k] && nl[k])
      HIP_TRY(hipMemcpy(lo[k], sb.lv + (size_t)k * depth, nl[k] * sizeof(me_level), hipMemcpyDeviceToHost),
              "D2H snapshot levels");
    if (noo[k]) *noo[k] = (size_t)no[k];
    const size_t m = std::min<size_t>({(size_t)no[k], ocaps[k], (size_t)ocap});
    if (oo[k] && m)
      HIP_TRY(hipMemcpy(oo[k], sb.ord + (size_t)k * ocap, m * sizeof(me_book_entry), hipMemcpyDeviceToHost),
              "D2H snapshot orders");
  }
  return ME_OK;
}

extern "C" int me_book_levels_all(me_engine* e, uint32_t depth, me_level* levels, uint32_t* counts) {
  if (!e) return ME_E_INVALID;
  int rc = me_sync(e);
  if (rc) return rc;
  if (!depth) return ME_OK;
  std::vector<uint32_t> syms(e->bk.S);
  for (uint32_t k = 0; k < e->bk.S; ++k) syms[k] = k;
  if ((rc = run_snapshot(e, syms.data(), e->bk.S, depth, 0))) return rc;
  auto& sb = e->snap;
  std::vector<uint32_t> cnt(2ull * e->bk.S);
  HIP_TRY(hipMemcpy(cnt.data(), sb.nlv, cnt.size() * 4, hipMemcpyDeviceToHost), "D2H snapshot counts");
  if (counts) memcpy(counts, cnt.data(), cnt.size() * 4);
  if (levels) {
    HIP_TRY(hipMemcpy(levels, sb.lv, 2ull * e->bk.S * depth * sizeof(me_level), hipMemcpyDeviceToHost),
            "D2H snapshot levels");
    for (size_t r = 0; r < cnt.size(); ++r)  // rows end in zeros past their levels
      memset(levels + r * depth + cnt[r], 0, (depth - cnt[r]) * sizeof(me_level));
  }
  return ME_OK;
}

extern "C" int me_book_snapshot(me_engine* e, uint32_t symbol, me_level* bids, me_level* asks, size_t depth,
                                size_t* n_bids, size_t* n_asks) {
  if (!e) return ME_E_INVALID;
  const uint32_t d = (uint32_t)std::min<size_t>(depth, 0xFFFFFFFFu);
  return me_book_orders(e, symbol, d, nullptr, 0, nullptr, nullptr, 0, nullptr, bids, asks, n_bids, n_asks);
}

extern "C" int me_book_dump(me_engine* e, uint32_t symbol, me_book_entry* out, size_t cap, size_t* n) {
  if (!e) return ME_E_INVALID;
  if (symbol >= e->bk.S) return e->fail(ME_E_INVALID, "symbol out of range");
  int rc = me_sync(e);
  if (rc) return rc;
  SymState ss;
  HIP_TRY(hipMemcpy(&ss, e->bk.sym + symbol, sizeof ss, hipMemcpyDeviceToHost), "D2H symbol");
  // every level of both sides (the whole window plus the far arrays), bids then asks
  std::vector<me_book_entry> side[2];
  side[0].resize(ss.resting + 1);
  side[1].resize(ss.resting + 1);
  size_t nb = 0, na = 0;
  rc = me_book_orders(e, symbol, 0xFFFFFFFFu, side[0].data(), side[0].size(), &nb, side[1].data(),
                      side[1].size(), &na, nullptr, nullptr, nullptr, nullptr);
  if (rc) return rc;
  if (out) {
    memcpy(out, side[0].data(), std::min(nb, cap) * sizeof(me_book_entry));
    if (cap > nb) memcpy(out + nb, side[1].data(), std::min(na, cap - nb) * sizeof(me_book_entry));
  }
  if (n) *n = nb + na;
  return ME_OK;
}

extern "C" int me_resting_count(me_engine* e, uint64_t* n) {
  if (!e || !n) return ME_E_INVALID;
  int rc = me_sync(e);
  if (rc) return rc;
  std::vector<SymState> ss(e->bk.S);
  HIP_TRY(hipMemcpy(ss.data(), e->bk.sym, ss.size() * sizeof(SymState), hipMemcpyDeviceToHost), "D2H symbols");
  uint64_t t = 0;
  for (auto& s : ss) t += s.resting;
  *n = t;
  return ME_OK;
}

extern "C" int me_timing_enable(me_engine* e, int enable) {
  if (!e) return ME_E_INVALID;
  if (!e->failed) {
    int rc = flush_pipeline(e);
    if (rc) return rc;
  }
  HIP_TRY(hipStreamSynchronize(e->stream), "hipStreamSynchronize");
  e->timed.clear();
  e->ev_used = 0;
  e->nlaunch = 0;
  e->nbat = 0;
  HIP_TRY(hipMemsetAsync(e->d_fills_acc, 0, 8, e->stream), "reset fill counter");
  HIP_TRY(hipStreamSynchronize(e->stream), "hipStreamSynchronize");
  e->timing = enable > 0 ? enable : 0;
  return ME_OK;
}

extern "C" int me_timing_read(me_engine* e, double* match_ms, double* pipeline_ms, uint64_t* launches,
                              uint64_t* fills, uint64_t* orders) {
  if (!e) return ME_E_INVALID;
  if (!e->failed) {
    int rc = flush_pipeline(e);
    if (rc) return rc;
  }
  HIP_TRY(hipStreamSynchronize(e->stream), "hipStreamSynchronize");
  double m = 0, p = 0;
  uint64_t o = 0;
  for (auto& t : e->timed) {
    float a = 0;
    HIP_TRY(hipEventElapsedTime(&a, t.m0, t.m1), "hipEventElapsedTime");
    m += a;
    o += t.orders;
  }
  if (e->timed.size() >= 2 && e->timed.back().idx > e->timed.front().idx) {
    // device time per batch: start-to-start of the first and last timed launches over the batches between
    float b = 0;
    HIP_TRY(hipEventElapsedTime(&b, e->timed.front().m0, e->timed.back().m0), "hipEventElapsedTime");
    p = b / (double)(e->timed.back().idx - e->timed.front().idx);
  }
  if (match_ms) *match_ms = m;
  if (pipeline_ms) *pipeline_ms = p;
  if (launches) *launches = e->timed.size();
  unsigned long long f = 0;
  HIP_TRY(hipMemcpy(&f, e->d_fills_acc, 8, hipMemcpyDeviceToHost), "read fill counter");
  if (orders) *orders = o;
  if (fills) *fills = f;
  return ME_OK;
}

extern "C" int me_stats_read(me_engine* e, uint64_t* handoffs) {
  if (!e) return ME_E_INVALID;
  int rc = me_sync(e);
  if (rc) return rc;
  unsigned long long v[ME_STATS];
  HIP_TRY(hipMemcpy(v, e->bk.stats, sizeof v, hipMemcpyDeviceToHost), "D2H stats");
  if (handoffs) *handoffs = v[ST_HANDOFFS];
  return ME_OK;
}

extern "C" int me_far_stats(me_engine* e, uint64_t* moves, uint64_t* collections, uint64_t* arena_used) {
  if (!e) return ME_E_INVALID;
  int rc = me_sync(e);
  if (rc) return rc;
  unsigned long long v[ME_STATS], ctl[FC_N];
  HIP_TRY(hipMemcpy(v, e->bk.stats, sizeof v, hipMemcpyDeviceToHost), "D2H stats");
  HIP_TRY(hipMemcpy(ctl, e->bk.far_ctl, sizeof ctl, hipMemcpyDeviceToHost), "D2H far arena");
  if (moves) *moves = v[ST_FAR_GROW];
  if (collections) *collections = v[ST_FAR_GC];
  if (arena_used) *arena_used = ctl[ctl[FC_HALF] & 1];
  return ME_OK;
}

extern "C" int me_chunk_stats(me_engine* e, uint64_t* reclaims, uint64_t* high_water, uint64_t* pool) {
  if (!e) return ME_E_INVALID;
  int rc = me_sync(e);
  if (rc) return rc;
  unsigned long long v[ME_STATS];
  uint32_t cp[CP_N], top = 0;
  HIP_TRY(hipMemcpy(v, e->bk.stats, sizeof v, hipMemcpyDeviceToHost), "D2H stats");
  HIP_TRY(hipMemcpy(cp, e->bk.cpool, sizeof cp, hipMemcpyDeviceToHost), "D2H chunk pool");
  HIP_TRY(hipMemcpy(&top, e->bk.chunk_top, 4, hipMemcpyDeviceToHost), "D2H chunk top");
  const uint64_t hw = top > cp[CP_NRECL] ? (uint64_t)cp[CP_FRESH] + (top - cp[CP_NRECL]) : cp[CP_FRESH];
  if (reclaims) *reclaims = v[ST_CHUNK_GC];
  if (high_water) *high_water = std::min<uint64_t>(hw, e->bk.nchunks);
  if (pool) *pool = e->bk.nchunks;
  return ME_OK;
}

extern "C" int me_paths_read(const me_engine* e, uint32_t* flags) {
  if (!e || !flags) return ME_E_INVALID;
  *flags = (e->hot.agg_reg ? ME_PATH_GROUPED_AGG : 0u) | (e->bk.hot_min && e->hot.agg ? ME_PATH_HOT_AGG : 0u) |
           (e->hot.agg_reg && e->hot.ag.gw_cx ? ME_PATH_GROUPED_CANCELS : 0u);
  return ME_OK;
}

extern "C" int me_last_error(const me_engine* e, char* buf, size_t cap) {
  std::string s;
  if (e) {
    s = e->err;
  } else {
    std::lock_guard<std::mutex> lk(g_err_mu);
    s = g_create_err;
  }
  if (buf && cap) {
    size_t k = std::min(cap - 1, s.size());
    memcpy(buf, s.data(), k);
    buf[k] = 0;
  }
  return (int)s.size();
}

#ifdef ME_STAMPS
// Diagnostic builds only: per-symbol phase cycles of the last k_match launch ([S][16]).
extern "C" int me_debug_stamps(me_engine* e, unsigned long long* out, size_t n) {
  if (!e || !e->bk.dbg) return ME_E_INVALID;
  HIP_TRY(hipStreamSynchronize(e->stream), "sync");
  size_t k = std::min(n, (size_t)e->bk.S * 24);
  HIP_TRY(hipMemcpy(out, e->bk.dbg, k * 8, hipMemcpyDeviceToHost), "D2H stamps");
  return ME_OK;
}
#endif

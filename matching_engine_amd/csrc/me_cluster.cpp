// me_cluster.cpp — the sharded deployment behind the C-ABI (include/me_cluster.h): one process per
// GPU, symbols hash-partitioned with me_shard_of, RCCL over xGMI (or a TCP star for the CPU tests)
// used only to scatter each slice's parts and to bring tapes, results, books and level snapshots back
// to the persistence root. Matching never crosses GPUs.
//
// The protocol is written once over a small Transport interface:
//   small host values  bcast / all-reduce MIN and SUM / gather of int64 words (commands, sizes, votes)
//   bulk payloads      scatterv from rank 0 / gatherv to rank 0 over transport buffers — HBM for RCCL
//                      (grouped ncclSend / ncclRecv, rank 0 included through a send to itself, so a
//                      one-GPU box runs every RCCL call of the protocol), host memory for TCP.
// librccl is opened at run time (dlopen), so the library carries no link-time RCCL dependency and the
// CPU tests never touch HIP.
#include <arpa/inet.h>
#include <dlfcn.h>
#include <errno.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "me_cluster.h"
#include "me_engine.h"

namespace {

std::mutex g_err_mu;
std::string g_create_err;

constexpr size_t kRec = 8 + 8 + 4 + 4 + 1;  // packed slice record: seq, price_q4, qty, symbol, kind
enum : int64_t { CMD_SUBMIT = 1, CMD_COLLECT = 2, CMD_BOOK = 3, CMD_SNAPSHOT = 4, CMD_STOP = 5 };
constexpr int kMaxInflight = 2;
// rank 0's time per protocol phase (me_cluster_phases)
enum { PH_SPLIT, PH_CTRL, PH_SCATTER, PH_VOTE, PH_MATCH, PH_COLLECT, PH_GATHER, PH_MERGE, PH_SPLIT_COUNT, PH_SPLIT_SLOT, PH_N };

inline size_t round8(size_t x) { return (x + 7) & ~(size_t)7; }

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// A persistent pool of up to 15 host threads for the parallel regions below (created on first use, parked
// on a condition variable between regions): a region used to start and join its threads, ~0.5-1 ms of the
// 5 ms rank 0 spends per 1M-order slice at W = 8. One region runs at a time (regions from the service's
// flusher and persister threads queue on `run_mu_`).
class ParPool {
 public:
  static ParPool& get() {
    static ParPool p;
    return p;
  }
  // job(t) for t in [0, T); the caller runs its share too
  void run(size_t T, const std::function<void(size_t)>& job) {
    std::lock_guard<std::mutex> rl(run_mu_);
    std::unique_lock<std::mutex> lk(mu_);
    while (th_.size() + 1 < T) th_.emplace_back([this] { worker(); });
    job_ = &job;
    T_ = T;
    next_.store(0);
    done_ = 0;
    ++gen_;
    cv_.notify_all();
    lk.unlock();
    size_t mine = 0;
    for (size_t t; (t = next_.fetch_add(1)) < T;) {
      job(t);
      ++mine;
    }
    lk.lock();
    done_ += mine;
    done_cv_.wait(lk, [&] { return done_ == T_; });
    job_ = nullptr;
  }
  ~ParPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }

 private:
  void worker() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      const std::function<void(size_t)>* job = job_;
      const size_t T = T_;
      lk.unlock();
      size_t mine = 0;
      for (size_t t; job && (t = next_.fetch_add(1)) < T;) {
        (*job)(t);
        ++mine;
      }
      lk.lock();
      done_ += mine;
      if (done_ == T_) done_cv_.notify_all();
    }
  }
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> th_;
  const std::function<void(size_t)>* job_ = nullptr;
  size_t T_ = 0, done_ = 0;
  std::atomic<size_t> next_{0};
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// f(t, lo, hi) over [0, n) in T contiguous chunks on T threads of the pool (the caller takes chunks too);
// one thread below `grain` records per chunk. The host halves of a large slice (split, pack, merge) are
// memory-bound loops.
template <class F>
void par_chunks(size_t n, size_t grain, F f) {
  const size_t hw = std::max<unsigned>(1u, std::thread::hardware_concurrency());
  const size_t T = std::max<size_t>(1, std::min<size_t>({hw, (size_t)16, n / std::max<size_t>(grain, 1)}));
  if (T <= 1) {
    f(0, 0, n);
    return;
  }
  const std::function<void(size_t)> job = [&](size_t t) { f(t, n * t / T, n * (t + 1) / T); };
  ParPool::get().run(T, job);
}
size_t par_threads(size_t n, size_t grain) {
  const size_t hw = std::max<unsigned>(1u, std::thread::hardware_concurrency());
  return std::max<size_t>(1, std::min<size_t>({hw, (size_t)16, n / std::max<size_t>(grain, 1)}));
}
constexpr size_t kGrain = 65536;  // records per host thread at least

// ---- sockets ----------------------------------------------------------------------------------
bool send_all(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n) {
    const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}
bool recv_all(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n) {
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}
void tune(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  int buf = 8 << 20;
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof buf);
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof buf);
}

// The star around rank 0: rank 0 accepts world - 1 connections (each names its rank first), every
// other rank connects to it (retrying until the timeout: rank 0 may start listening later).
bool star_connect(const me_cluster_config& c, std::vector<int>& fds, std::string& err) {
  const uint32_t tmo = c.timeout_ms ? c.timeout_ms : 60000;
  fds.assign(c.world, -1);
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons((uint16_t)c.port);
  if (inet_pton(AF_INET, c.addr ? c.addr : "127.0.0.1", &sa.sin_addr) != 1) {
    err = "bootstrap: addr is not an IPv4 address";
    return false;
  }
  const auto t0 = std::chrono::steady_clock::now();
  auto left_ms = [&]() {
    const long long e =
        std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
    return (long long)tmo - e;
  };
  if (c.rank == 0) {
    if (c.world == 1) return true;
    const int ls = ::socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    if (ls < 0 || ::bind(ls, (sockaddr*)&sa, sizeof sa) != 0 || ::listen(ls, (int)c.world) != 0) {
      err = std::string("bootstrap: rank 0 cannot listen: ") + strerror(errno);
      if (ls >= 0) ::close(ls);
      return false;
    }
    for (uint32_t got = 1; got < c.world;) {
      pollfd p{ls, POLLIN, 0};
      const long long lm = left_ms();
      if (lm <= 0 || ::poll(&p, 1, (int)lm) <= 0) {
        err = "bootstrap: timed out waiting for the other ranks";
        ::close(ls);
        return false;
      }
      const int fd = ::accept(ls, nullptr, nullptr);
      if (fd < 0) continue;
      uint32_t r = 0;
      if (!recv_all(fd, &r, 4) || r == 0 || r >= c.world || fds[r] >= 0) {
        ::close(fd);
        continue;
      }
      tune(fd);
      fds[r] = fd;
      ++got;
    }
    ::close(ls);
    return true;
  }
  for (;;) {
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd >= 0 && ::connect(fd, (sockaddr*)&sa, sizeof sa) == 0) {
      tune(fd);
      if (!send_all(fd, &c.rank, 4)) {
        ::close(fd);
        err = "bootstrap: lost rank 0";
        return false;
      }
      fds[0] = fd;
      return true;
    }
    if (fd >= 0) ::close(fd);
    if (left_ms() <= 0) {
      err = "bootstrap: cannot reach rank 0";
      return false;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

// ---- transports -------------------------------------------------------------------------------
class Transport {
 public:
  virtual ~Transport() = default;
  virtual bool device() const = 0;
  // small host values (int64 words)
  virtual bool bcast(int64_t* v, size_t n) = 0;
  virtual bool allreduce(int64_t* v, size_t n, bool min) = 0;
  virtual bool gather(const int64_t* mine, size_t n, int64_t* all) = 0;  // rank 0 receives world * n
  // bulk: transport buffers (HBM for RCCL, host for TCP); sizes per rank known on every rank
  virtual bool scatterv(const char* send, const std::vector<size_t>& bytes, char* recv) = 0;
  virtual bool gatherv(const char* send, const std::vector<size_t>& bytes, char* recv) = 0;
  virtual char* alloc(size_t bytes) = 0;
  virtual void release(char* p) = 0;
  virtual bool put(char* dst, const void* src, size_t n) = 0;  // host -> transport buffer
  virtual bool get(void* dst, const char* src, size_t n) = 0;  // transport buffer -> host (synchronous)
  virtual std::string error() const { return err; }
  uint64_t moved = 0;
  uint32_t rank = 0, world = 1;

 protected:
  std::string err;
};

class TcpTransport : public Transport {
 public:
  std::vector<int> fds;
  ~TcpTransport() override {
    for (int fd : fds)
      if (fd >= 0) ::close(fd);
  }
  bool device() const override { return false; }
  bool fail(const char* what) {
    err = std::string("tcp transport: ") + what;
    return false;
  }
  bool bcast(int64_t* v, size_t n) override {
    if (rank == 0) {
      for (uint32_t r = 1; r < world; ++r)
        if (!send_all(fds[r], v, 8 * n)) return fail("send");
    } else if (!recv_all(fds[0], v, 8 * n)) {
      return fail("recv");
    }
    moved += 8 * n;
    return true;
  }
  bool gather(const int64_t* mine, size_t n, int64_t* all) override {
    if (rank == 0) {
      memcpy(all, mine, 8 * n);
      for (uint32_t r = 1; r < world; ++r)
        if (!recv_all(fds[r], all + r * n, 8 * n)) return fail("recv");
    } else if (!send_all(fds[0], mine, 8 * n)) {
      return fail("send");
    }
    moved += 8 * n;
    return true;
  }
  bool allreduce(int64_t* v, size_t n, bool min) override {
    std::vector<int64_t> all(rank == 0 ? world * n : 0);
    if (!gather(v, n, all.data())) return false;
    if (rank == 0)
      for (uint32_t r = 1; r < world; ++r)
        for (size_t i = 0; i < n; ++i) v[i] = min ? std::min(v[i], all[r * n + i]) : v[i] + all[r * n + i];
    return bcast(v, n);
  }
  bool scatterv(const char* send, const std::vector<size_t>& bytes, char* recv) override {
    if (rank == 0) {
      size_t off = bytes[0];
      if (bytes[0]) memcpy(recv, send, bytes[0]);
      for (uint32_t r = 1; r < world; ++r) {
        if (bytes[r] && !send_all(fds[r], send + off, bytes[r])) return fail("send");
        off += bytes[r];
      }
    } else if (bytes[rank] && !recv_all(fds[0], recv, bytes[rank])) {
      return fail("recv");
    }
    moved += bytes[rank];
    return true;
  }
  bool gatherv(const char* send, const std::vector<size_t>& bytes, char* recv) override {
    if (rank == 0) {
      size_t off = bytes[0];
      if (bytes[0]) memcpy(recv, send, bytes[0]);
      for (uint32_t r = 1; r < world; ++r) {
        if (bytes[r] && !recv_all(fds[r], recv + off, bytes[r])) return fail("recv");
        off += bytes[r];
      }
    } else if (bytes[rank] && !send_all(fds[0], send, bytes[rank])) {
      return fail("send");
    }
    moved += bytes[rank];
    return true;
  }
  char* alloc(size_t bytes) override { return (char*)malloc(std::max<size_t>(bytes, 8)); }
  void release(char* p) override { free(p); }
  bool put(char* dst, const void* src, size_t n) override {
    if (n) memcpy(dst, src, n);
    return true;
  }
  bool get(void* dst, const char* src, size_t n) override {
    if (n) memcpy(dst, src, n);
    return true;
  }
};

// RCCL entry points, resolved from librccl at run time (types from rccl.h).
struct Rccl {
  void* h = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*Broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  bool load(std::string& err) {
    if (h) return true;
    // RTLD_NOLOAD first: a process that already holds an RCCL (torch's) keeps one copy
    for (const char* n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      h = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
      if (h) break;
    }
    if (!h)
      for (const char* n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
        h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
        if (h) break;
      }
    if (!h) {
      err = "librccl not found";
      return false;
    }
#define RS(f)                                                             \
  f = reinterpret_cast<decltype(f)>(dlsym(h, "nccl" #f));                 \
  if (!f) {                                                               \
    err = "librccl lacks nccl" #f;                                        \
    return false;                                                         \
  }
    RS(GetUniqueId);
    RS(CommInitRank);
    RS(CommDestroy);
    RS(CommAbort);
    RS(Broadcast);
    RS(AllReduce);
    RS(AllGather);
    RS(Send);
    RS(Recv);
    RS(GroupStart);
    RS(GroupEnd);
    RS(GetErrorString);
#undef RS
    return true;
  }
};
Rccl g_rccl;
std::mutex g_rccl_mu;

// RCCL for the bulk payloads (device buffers over xGMI); the small host values (commands, votes, sizes)
// go over the TCP star the bootstrap opened — a host word needs no H2D / collective / D2H round trip.
class RcclTransport : public Transport {
 public:
  ncclComm_t comm = nullptr;
  hipStream_t st = nullptr;
  TcpTransport ctl;            // the control plane
  ~RcclTransport() override {
    if (st) (void)hipStreamSynchronize(st);
    if (comm) g_rccl.CommDestroy(comm);
    if (st) (void)hipStreamDestroy(st);
  }
  bool device() const override { return true; }
  bool nfail(ncclResult_t r, const char* what) {
    err = std::string("rccl ") + what + ": " + (g_rccl.GetErrorString ? g_rccl.GetErrorString(r) : "error");
    return false;
  }
  bool hfail(hipError_t e, const char* what) {
    err = std::string(what) + ": " + hipGetErrorString(e);
    return false;
  }
  bool sync() {
    const hipError_t e = hipStreamSynchronize(st);
    return e == hipSuccess || hfail(e, "hipStreamSynchronize");
  }
  bool ctl_ok(bool ok) {
    if (!ok) err = ctl.error();
    return ok;
  }
  bool bcast(int64_t* v, size_t n) override { return ctl_ok(ctl.bcast(v, n)); }
  bool allreduce(int64_t* v, size_t n, bool min) override { return ctl_ok(ctl.allreduce(v, n, min)); }
  bool gather(const int64_t* mine, size_t n, int64_t* all) override { return ctl_ok(ctl.gather(mine, n, all)); }
  bool scatterv(const char* send, const std::vector<size_t>& bytes, char* recv) override {
    ncclResult_t r = g_rccl.GroupStart();
    if (r != ncclSuccess) return nfail(r, "group start");
    if (rank == 0) {
      size_t off = 0;
      for (uint32_t p = 0; p < world; ++p) {
        if (bytes[p] && (r = g_rccl.Send(send + off, bytes[p], ncclUint8, (int)p, comm, st)) != ncclSuccess)
          return nfail(r, "send");
        off += bytes[p];
      }
    }
    if (bytes[rank] && (r = g_rccl.Recv(recv, bytes[rank], ncclUint8, 0, comm, st)) != ncclSuccess)
      return nfail(r, "recv");
    if ((r = g_rccl.GroupEnd()) != ncclSuccess) return nfail(r, "group end");
    moved += bytes[rank];
    return sync();
  }
  bool gatherv(const char* send, const std::vector<size_t>& bytes, char* recv) override {
    ncclResult_t r = g_rccl.GroupStart();
    if (r != ncclSuccess) return nfail(r, "group start");
    if (bytes[rank] && (r = g_rccl.Send(send, bytes[rank], ncclUint8, 0, comm, st)) != ncclSuccess)
      return nfail(r, "send");
    if (rank == 0) {
      size_t off = 0;
      for (uint32_t p = 0; p < world; ++p) {
        if (bytes[p] && (r = g_rccl.Recv(recv + off, bytes[p], ncclUint8, (int)p, comm, st)) != ncclSuccess)
          return nfail(r, "recv");
        off += bytes[p];
      }
    }
    if ((r = g_rccl.GroupEnd()) != ncclSuccess) return nfail(r, "group end");
    moved += bytes[rank];
    return sync();
  }
  char* alloc(size_t bytes) override {
    void* p = nullptr;
    return hipMalloc(&p, std::max<size_t>(bytes, 8)) == hipSuccess ? (char*)p : nullptr;
  }
  void release(char* p) override {
    if (p) (void)hipFree(p);
  }
  bool put(char* dst, const void* src, size_t n) override {
    if (!n) return true;
    const hipError_t e = hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, st);
    return e == hipSuccess || hfail(e, "H2D");
  }
  bool get(void* dst, const char* src, size_t n) override {
    if (!n) return true;
    const hipError_t e = hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, st);
    if (e != hipSuccess) return hfail(e, "D2H");
    return sync();
  }
  // bootstrap over the TCP star: rank 0's unique id to every rank, then ncclCommInitRank
  bool init(const me_cluster_config& c, std::string& e) {
    {
      std::lock_guard<std::mutex> lk(g_rccl_mu);
      if (!g_rccl.load(e)) return false;
    }
    hipError_t he = hipSetDevice(c.device);
    if (he != hipSuccess) return (e = std::string("hipSetDevice: ") + hipGetErrorString(he)), false;
    if ((he = hipStreamCreateWithFlags(&st, hipStreamNonBlocking)) != hipSuccess)
      return (e = std::string("rccl transport: ") + hipGetErrorString(he)), false;
    std::vector<int>& fds = ctl.fds;
    if (!star_connect(c, fds, e)) return false;
    ctl.rank = c.rank;
    ctl.world = c.world;
    ncclUniqueId id;
    memset(&id, 0, sizeof id);
    bool ok = true;
    if (c.rank == 0) {
      ncclResult_t r = g_rccl.GetUniqueId(&id);
      if (r != ncclSuccess) {
        e = std::string("ncclGetUniqueId: ") + g_rccl.GetErrorString(r);
        ok = false;
      }
      for (uint32_t p = 1; p < c.world; ++p) ok = send_all(fds[p], &id, sizeof id) && ok;
    } else {
      ok = recv_all(fds[0], &id, sizeof id);
      if (!ok) e = "bootstrap: no unique id from rank 0";
    }
    if (!ok) return false;
    const ncclResult_t r = g_rccl.CommInitRank(&comm, (int)c.world, id, (int)c.rank);
    if (r != ncclSuccess) {
      comm = nullptr;
      e = std::string("ncclCommInitRank: ") + g_rccl.GetErrorString(r);
      return false;
    }
    return true;
  }
};

// One rank's share of an in-flight slice (slot = ticket & 1).
struct Part {
  bool used = false;
  uint64_t ticket = 0;
  size_t n = 0;         // records
  uint64_t nl = 0;      // LIMIT records (admission)
  size_t nf = 0;        // fills after the match
  char* in = nullptr;   // transport buffer: the packed part
  char* out = nullptr;  // transport buffer (device mode): tape, then results
  uint64_t eng_ticket = 0;       // engine over TCP: me_submit_host's ticket
  std::vector<char> h_out;       // host mode: tape, then results
};

// Rank 0's bookkeeping of a submitted slice.
struct Ticket {
  uint64_t t = 0;
  size_t n = 0;
  std::vector<size_t> pos_off;    // rank r's records are [pos_off[r], pos_off[r + 1]) of the parts laid end to end
  std::vector<uint16_t> srank;    // per slice record: its rank ...
  std::vector<uint32_t> sidx;     // ... and its index in that rank's part (merge gathers in slice order)
};

// The packed part of n records at p: seq[n] px[n] qty[n] sym[n] kind[n].
struct PackView {
  uint64_t* seq;
  int64_t* px;
  int32_t* qty;
  uint32_t* sym;
  uint8_t* kind;
  PackView(char* p, size_t n)
      : seq((uint64_t*)p), px((int64_t*)(p + 8 * n)), qty((int32_t*)(p + 16 * n)), sym((uint32_t*)(p + 20 * n)),
        kind((uint8_t*)(p + 24 * n)) {}
};

// Rank 0's split of a slice by owner, stable (each part keeps slice order = seq order), in two passes:
// split_count — per-chunk counts of records and of NEW LIMITs per rank (counted in each thread's own
// arrays, published once: the threads' rows share cache lines — at world 1 all sixteen in one line: 66 ms
// per 1M-record slice of false sharing, profiles/r4/r4e); split_pack — every chunk packs its records at its
// offsets into the parts' views and records where each came from. An unknown global id goes to rank 0 out
// of range (BAD_SYMBOL there).
struct SplitCounts {
  size_t T = 0;
  std::vector<uint64_t> cnt, lim;  // [T][W]
  std::vector<uint64_t> per_rank, lim_rank;  // [W]
};
void split_count(const uint32_t* owner, uint32_t W, uint32_t S, const me_order_soa* b, size_t n, SplitCounts& sc) {
  sc.T = par_threads(n, kGrain);
  sc.cnt.assign(sc.T * W, 0);
  sc.lim.assign(sc.T * W, 0);
  par_chunks(n, kGrain, [&](size_t i, size_t lo, size_t hi) {
    std::vector<uint64_t> ci(W, 0), li(W, 0);
    for (size_t k = lo; k < hi; ++k) {
      const uint32_t s = b->symbol[k];
      const uint32_t r = s < S ? owner[s] : 0;
      ci[r]++;
      li[r] += (b->kind[k] & 0x0Cu) == 0u;  // NEW LIMIT: may rest
    }
    std::copy(ci.begin(), ci.end(), sc.cnt.begin() + i * W);
    std::copy(li.begin(), li.end(), sc.lim.begin() + i * W);
  });
  sc.per_rank.assign(W, 0);
  sc.lim_rank.assign(W, 0);
  for (uint32_t r = 0; r < W; ++r)
    for (size_t i = 0; i < sc.T; ++i) {
      sc.per_rank[r] += sc.cnt[i * W + r];
      sc.lim_rank[r] += sc.lim[i * W + r];
    }
}
void split_pack(const uint32_t* owner, const uint32_t* local, uint32_t W, uint32_t S, const me_order_soa* b, size_t n,
                const SplitCounts& sc, std::vector<PackView>& dst, Ticket& tk) {
  tk.pos_off.assign(W + 1, 0);
  for (uint32_t r = 0; r < W; ++r) tk.pos_off[r + 1] = tk.pos_off[r] + sc.per_rank[r];
  tk.srank.resize(n);
  tk.sidx.resize(n);
  // chunk i's first record of rank r lands at base[i][r] within the part
  std::vector<uint64_t> base(sc.T * W, 0);
  for (uint32_t r = 0; r < W; ++r) {
    uint64_t x = 0;
    for (size_t i = 0; i < sc.T; ++i) {
      base[i * W + r] = x;
      x += sc.cnt[i * W + r];
    }
  }
  par_chunks(n, kGrain, [&](size_t i, size_t lo, size_t hi) {
    std::vector<uint64_t> at(base.begin() + i * W, base.begin() + (i + 1) * W);
    for (size_t k = lo; k < hi; ++k) {
      const uint32_t s = b->symbol[k];
      const uint32_t r = s < S ? owner[s] : 0;
      const uint64_t j = at[r]++;
      PackView& v = dst[r];
      v.seq[j] = b->seq[k];
      v.px[j] = b->price_q4[k];
      v.qty[j] = b->qty[k];
      v.sym[j] = s < S ? local[s] : 0xFFFFFFFFu;
      v.kind[j] = b->kind[k];
      tk.srank[k] = (uint16_t)r;
      tk.sidx[k] = (uint32_t)j;
    }
  });
}

// Rank 0's merge of the shards' outputs: results back to slice order, the merged tape in slice order (= taker
// seq order: every taker's fills are consecutive on its one shard, at its result's tape offset there). tr[r] /
// tf[r] / nf[r]: shard r's results (its part's order), tape and fill count. Every shard's results must account
// for its tape exactly (fill counts summing to its fills, each run inside the tape) — the copy trusts them;
// false (bad = the shard) otherwise.
// The check runs over the parts laid end to end, everything else in slice order — results gathered from the
// parts (W sequential read streams, sequential writes), the tape copied taker by taker — and every pass is one
// parallel region over the whole slice, so its threads do not shrink as W grows (a region per part, with the
// results and fills scattered to their slice positions, took 24.7 ms per 1M-record slice at W = 8,
// profiles/r5/rank0).
template <class G>
void part_runs(const Ticket& tk, size_t a, size_t b, G&& g) {  // g(r, first, last) in rank r's own indices
  uint32_t r = (uint32_t)(std::upper_bound(tk.pos_off.begin(), tk.pos_off.end(), a) - tk.pos_off.begin()) - 1u;
  for (size_t i = a; i < b;) {
    while (tk.pos_off[r + 1] <= i) ++r;
    const size_t e = std::min(b, tk.pos_off[r + 1]);
    g(r, i - tk.pos_off[r], e - tk.pos_off[r]);
    i = e;
  }
}
bool merge_parts(uint32_t W, const Ticket& tk, const std::vector<const me_order_result*>& tr,
                 const std::vector<const me_fill*>& tf, const std::vector<size_t>& nf, std::vector<me_order_result>& res_v,
                 std::vector<me_fill>& tape_v, uint32_t* bad) {
  const size_t n = tk.n, T = par_threads(n, kGrain);
  std::vector<uint64_t> psum(T * W, 0);
  std::vector<uint8_t> pout(T * W, 0);
  par_chunks(n, kGrain, [&](size_t t, size_t a, size_t b) {
    part_runs(tk, a, b, [&](uint32_t r, size_t ka, size_t kb) {
      const me_order_result* rr = tr[r];
      const size_t nfr = nf[r];
      uint64_t x = 0;
      bool o = false;
      for (size_t k = ka; k < kb; ++k) {
        x += rr[k].fill_count;
        o |= rr[k].fill_count && (uint64_t)rr[k].tape_offset + rr[k].fill_count > nfr;
      }
      psum[t * W + r] += x;
      pout[t * W + r] |= o;
    });
  });
  for (uint32_t r = 0; r < W; ++r) {
    uint64_t x = 0;
    bool o = false;
    for (size_t t = 0; t < T; ++t) {
      x += psum[t * W + r];
      o |= pout[t * W + r] != 0;
    }
    if (o || x != nf[r]) {
      if (bad) *bad = r;
      return false;
    }
  }
  res_v.resize(n);
  me_order_result* res = res_v.data();
  const uint16_t* srank = tk.srank.data();
  const uint32_t* sidx = tk.sidx.data();
  // results in slice order (tape_offset still the shard's) + each chunk's fill count
  std::vector<uint64_t> csum(T + 1, 0);
  par_chunks(n, kGrain, [&](size_t t, size_t a, size_t b) {
    uint64_t x = 0;
    for (size_t k = a; k < b; ++k) {
      res[k] = tr[srank[k]][sidx[k]];
      x += res[k].fill_count;
    }
    csum[t + 1] = x;
  });
  for (size_t t = 0; t < T; ++t) csum[t + 1] += csum[t];
  tape_v.resize(csum[T]);
  me_fill* tape = tape_v.data();
  // merged tape offsets (exclusive scan in slice order = taker seq order) and each taker's fills from its shard
  par_chunks(n, kGrain, [&](size_t t, size_t a, size_t b) {
    uint64_t o = csum[t];
    for (size_t k = a; k < b; ++k) {
      const uint32_t fc = res[k].fill_count;
      if (fc) memcpy(tape + o, tf[srank[k]] + res[k].tape_offset, fc * sizeof(me_fill));
      res[k].tape_offset = (uint32_t)o;
      o += fc;
    }
  });
  return true;
}

}  // namespace

struct me_cluster {
  me_cluster_config cfg{};
  std::unique_ptr<Transport> tp;
  me_engine* eng = nullptr;  // owned
  me_shard_ops ops{};
  bool use_ops = false;
  std::vector<uint32_t> owner, local;  // global symbol -> rank, local id
  std::vector<std::vector<uint32_t>> members;
  uint64_t tape_cap = 0;  // fills one part can produce at most (engine: me_fill_bound(max_batch))
  Part part[kMaxInflight];
  // rank 0
  std::deque<Ticket> tickets;
  uint64_t next_ticket = 0;
  std::vector<char> h_send;
  char* t_send = nullptr;  // transport buffer: every part, rank order
  char* t_gather = nullptr;
  size_t t_gather_cap = 0;
  std::vector<char> h_gather;
  std::vector<me_fill> tape;
  std::vector<me_order_result> res;
  // rank 0 with an engine: its own part goes straight into the engine's pinned host slots (me_host_inputs,
  // me_submit_host, me_collect) — no pack copy, scatter or gather for it; at world 1 collect hands out the
  // slot's outputs as they are (one shard: its tape and results are the slice's)
  bool direct0 = false;
  me_order_soa w0{};  // the slot inputs rank 0's part was packed into (SUBMIT in flight)
  const me_fill* out_tape = nullptr;
  size_t out_nf = 0;
  const me_order_result* out_res = nullptr;
  double ph[PH_N] = {};
  uint64_t max_resting_total = 0;
  bool failed = false;
  bool stopped = false;
  uint64_t slices = 0;
  std::string err;

  int fail(int code, const std::string& m) {
    err = m;
    return code;
  }
  int tfail(const char* what) {
    failed = true;
    return fail(ME_E_STATE, std::string(what) + ": " + tp->error());
  }
  size_t hdr_words() const { return 6 + 2 * (size_t)cfg.world; }
};

static int set_create_err(const std::string& s) {
  std::lock_guard<std::mutex> lk(g_err_mu);
  g_create_err = s;
  return 0;
}

static std::string eng_err(me_engine* e) {
  char b[512];
  me_last_error(e, b, sizeof b);
  return b;
}

extern "C" size_t me_cluster_shard_symbols(uint32_t num_symbols, uint32_t world, uint32_t rank, uint32_t* out,
                                           size_t cap) {
  size_t k = 0;
  if (!world) return 0;
  for (uint32_t s = 0; s < num_symbols; ++s)
    if (me_shard_of(s, world) == rank) {
      if (out && k < cap) out[k] = s;
      ++k;
    }
  return k;
}

static void free_cluster(me_cluster* c) {
  if (c->tp) {
    for (auto& p : c->part) {
      c->tp->release(p.in);
      c->tp->release(p.out);
    }
    c->tp->release(c->t_send);
    c->tp->release(c->t_gather);
  }
  c->tp.reset();
  if (c->eng) me_destroy(c->eng);
  c->eng = nullptr;
}

extern "C" me_cluster* me_cluster_create(const me_cluster_config* cfg, const me_config* engine_cfg,
                                         const me_shard_ops* ops) {
  if (!cfg || !cfg->world || cfg->rank >= cfg->world || !cfg->num_symbols || !cfg->max_batch ||
      (cfg->transport != ME_TRANSPORT_RCCL && cfg->transport != ME_TRANSPORT_TCP) ||
      (!ops && (!engine_cfg || !engine_cfg->base_price)) || (ops && !ops->match) || cfg->world > 1024) {
    set_create_err("me_cluster_create: invalid config (world >= 1, rank < world, num_symbols, max_batch, a "
                   "transport, and either shard ops with match or an engine config with base prices)");
    return nullptr;
  }
  std::unique_ptr<me_cluster> c(new me_cluster());
  c->cfg = *cfg;
  const uint32_t S = cfg->num_symbols, W = cfg->world;
  c->owner.resize(S);
  c->local.resize(S);
  c->members.resize(W);
  for (uint32_t s = 0; s < S; ++s) {
    const uint32_t r = me_shard_of(s, W);
    c->owner[s] = r;
    c->local[s] = (uint32_t)c->members[r].size();
    c->members[r].push_back(s);
  }
  const std::vector<uint32_t>& mine = c->members[cfg->rank];
  uint64_t my_resting = 0;
  if (ops) {
    c->ops = *ops;
    c->use_ops = true;
    my_resting = ops->max_resting;
    c->tape_cap = ops->max_resting + 2ull * cfg->max_batch;
  } else {
    // this rank's engine: its share of the symbols, their window bases, their global ids in me_fill
    me_config ec = *engine_cfg;
    std::vector<int64_t> base(std::max<size_t>(mine.size(), 1));
    std::vector<uint32_t> ids(std::max<size_t>(mine.size(), 1), 0);
    for (size_t k = 0; k < mine.size(); ++k) {
      base[k] = engine_cfg->base_price[mine[k]];
      ids[k] = mine[k];
    }
    if (mine.empty()) base[0] = engine_cfg->base_price[0];
    ec.num_symbols = (uint32_t)std::max<size_t>(mine.size(), 1);  // an empty shard keeps one idle book
    ec.base_price = base.data();
    ec.symbol_ids = ids.data();
    ec.device = cfg->device;
    ec.max_batch = cfg->max_batch;
    c->eng = me_create(&ec);
    if (!c->eng) {
      char b[512];
      me_last_error(nullptr, b, sizeof b);
      set_create_err(std::string("me_cluster_create: shard engine: ") + b);
      return nullptr;
    }
    my_resting = ec.max_resting;
    c->tape_cap = me_fill_bound(c->eng, cfg->max_batch);
  }
  std::string e;
  if (cfg->transport == ME_TRANSPORT_TCP) {
    auto t = std::make_unique<TcpTransport>();
    if (!star_connect(*cfg, t->fds, e)) {
      free_cluster(c.get());
      set_create_err("me_cluster_create: " + e);
      return nullptr;
    }
    c->tp = std::move(t);
  } else {
    auto t = std::make_unique<RcclTransport>();
    if (!t->init(*cfg, e)) {
      c->tp = std::move(t);
      free_cluster(c.get());
      set_create_err("me_cluster_create: " + e);
      return nullptr;
    }
    c->tp = std::move(t);
    if (c->eng) me_set_stream(c->eng, static_cast<RcclTransport*>(c->tp.get())->st);  // one ordered stream
  }
  c->tp->rank = cfg->rank;
  c->tp->world = W;
  // the shards' capacity, summed: the fill bound the service sizes its buffers with
  int64_t tot = (int64_t)my_resting;
  if (!c->tp->allreduce(&tot, 1, false)) {
    set_create_err("me_cluster_create: " + c->tp->error());
    free_cluster(c.get());
    return nullptr;
  }
  c->max_resting_total = (uint64_t)tot;
  const bool dev = c->tp->device();
  for (auto& p : c->part) {
    p.in = c->tp->alloc(kRec * cfg->max_batch);
    if (dev && !c->use_ops) p.out = c->tp->alloc(c->tape_cap * sizeof(me_fill) + (size_t)cfg->max_batch * 20 + 64);
    if (!p.in || (dev && !c->use_ops && !p.out)) {
      set_create_err("me_cluster_create: transport buffers");
      free_cluster(c.get());
      return nullptr;
    }
  }
  {  // ME_CLUSTER_DIRECT=0: rank 0's part through the transport like the others' (tests of the RCCL calls)
    const char* v = getenv("ME_CLUSTER_DIRECT");
    c->direct0 = cfg->rank == 0 && !c->use_ops && c->eng && !(v && atoi(v) == 0);
  }
  // ranks that match through the engine's pinned host slots (rank 0's direct part, every rank on a host
  // transport) allocate them now: a slot's first use would otherwise pin ~100 MB inside a slice's split
  // (config 3's 1M-record slices: 51 ms per slice over 16 slices, profiles/r4/r4c)
  // (the protocol's slots only: kMaxInflight tickets, the slot the last collect holds, one spare — not the
  // engine's 4G + 1, which at 1M-record slices would pin ~14 GB)
  if (c->eng && (c->direct0 || !dev) && me_host_reserve(c->eng, kMaxInflight + 2) != ME_OK) {
    set_create_err("me_cluster_create: host slots: " + eng_err(c->eng));
    free_cluster(c.get());
    return nullptr;
  }
  if (cfg->rank == 0) {
    c->t_send = c->tp->alloc(kRec * cfg->max_batch);
    if (!c->t_send) {
      set_create_err("me_cluster_create: transport buffers");
      free_cluster(c.get());
      return nullptr;
    }
  }
  return c.release();
}

extern "C" void me_cluster_destroy(me_cluster* c) {
  if (!c) return;
  free_cluster(c);
  delete c;
}

// ---- the commands (every rank runs the same code for each; hdr came from rank 0) ----------------
// Status agreement: MIN over ranks of each rank's code (0 ok, negative = an ME_E_* error).
static bool agree(me_cluster* c, int& rc) {
  int64_t v = rc;
  if (!c->tp->allreduce(&v, 1, true)) return false;
  rc = (int)v;
  return true;
}

static int run_submit(me_cluster* c, const int64_t* hdr) {
  const uint32_t W = c->cfg.world, me = c->cfg.rank;
  const uint64_t ticket = (uint64_t)hdr[1];
  Part& p = c->part[ticket & 1];
  const bool direct = me == 0 && c->direct0;  // rank 0's part is already in its engine's slot inputs
  p.used = false;
  p.ticket = ticket;
  p.n = (size_t)hdr[6 + me];
  p.nl = (uint64_t)hdr[6 + W + me];
  p.nf = 0;
  p.eng_ticket = 0;
  std::vector<size_t> bytes(W);
  for (uint32_t r = 0; r < W; ++r) bytes[r] = kRec * (size_t)hdr[6 + r];
  if (direct) bytes[0] = 0;
  double t = now_s();
  size_t tot = 0;
  for (size_t b : bytes) tot += b;
  // a rank with nothing to send or receive stays out of the scatter (sends and receives pair up per rank)
  if (me == 0 ? tot > 0 : bytes[me] > 0) {
    if (me == 0 && !c->tp->put(c->t_send, c->h_send.data(), tot)) return c->tfail("scatter");
    if (!c->tp->scatterv(c->t_send, bytes, p.in)) return c->tfail("scatter");
  }
  if (me == 0) c->ph[PH_SCATTER] += now_s() - t;
  // all-or-none: every shard's admission control first
  int rc = ME_OK, ok = 1;
  if (p.n && !c->failed) {
    if (c->use_ops) {
      if (c->ops.admit) rc = c->ops.admit(c->ops.ctx, p.nl, &ok);
    } else {
      rc = me_admission_check(c->eng, p.nl, &ok);
    }
  }
  t = now_s();
  int64_t vote[2] = {rc != ME_OK || c->failed ? 0 : ok, c->failed ? ME_E_STATE : rc};
  if (!c->tp->allreduce(vote, 2, true)) return c->tfail("admission vote");
  if (me == 0) c->ph[PH_VOTE] += now_s() - t;
  if (vote[1] != ME_OK) return c->fail((int)vote[1], "a shard failed its admission check");
  if (vote[0] == 0) return c->fail(ME_E_CAPACITY, "a shard's max_resting refused its part; no book changed");
  // match this rank's part
  t = now_s();
  rc = ME_OK;
  if (p.n) {
    if (c->use_ops) {
      PackView v(p.in, p.n);
      me_order_soa b{v.seq, v.px, v.qty, v.sym, v.kind};
      const me_fill* f = nullptr;
      const me_order_result* r = nullptr;
      size_t nf = 0;
      rc = c->ops.match(c->ops.ctx, &b, p.n, &f, &nf, &r);
      if (rc == ME_OK) {
        p.nf = nf;
        p.h_out.resize(round8(nf * sizeof(me_fill) + p.n * sizeof(me_order_result)));
        if (nf) memcpy(p.h_out.data(), f, nf * sizeof(me_fill));
        memcpy(p.h_out.data() + nf * sizeof(me_fill), r, p.n * sizeof(me_order_result));
      }
    } else if (direct) {  // the pipelined host path: collected at COLLECT, outputs in pinned memory
      rc = me_submit_host(c->eng, &c->w0, p.n, &p.eng_ticket);
    } else if (c->tp->device()) {  // device batch; outputs into the staging buffer, HBM to HBM
      PackView v(p.in, p.n);
      me_order_soa b{v.seq, v.px, v.qty, v.sym, v.kind};
      rc = me_submit_device_limits(c->eng, &b, p.n, p.nl);
      size_t nf = 0;
      if (rc == ME_OK) rc = me_copy_tape_device(c->eng, p.out, c->tape_cap, &nf);
      if (rc == ME_OK) rc = me_copy_results_device(c->eng, p.out + nf * sizeof(me_fill), p.n);
      p.nf = nf;
    } else {  // host batch through the engine's pinned slots: collected at COLLECT
      PackView v(p.in, p.n);
      me_order_soa b{v.seq, v.px, v.qty, v.sym, v.kind};
      rc = me_submit_host(c->eng, &b, p.n, &p.eng_ticket);
    }
  }
  if (me == 0) c->ph[PH_MATCH] += now_s() - t;
  if (!agree(c, rc)) return c->tfail("status");
  if (rc != ME_OK) {
    c->failed = true;  // some shard may have applied its part: the slice is lost
    return c->fail(ME_E_STATE, "a shard failed to match its part" + (c->eng ? ": " + eng_err(c->eng) : std::string()));
  }
  p.used = true;
  return ME_OK;
}

static int run_collect(me_cluster* c, const int64_t* hdr) {
  const uint32_t W = c->cfg.world, me = c->cfg.rank;
  const uint64_t ticket = (uint64_t)hdr[1];
  Part& p = c->part[ticket & 1];
  const bool direct = me == 0 && c->direct0;
  int rc = (p.used && p.ticket == ticket) ? ME_OK : ME_E_STATE;
  const char* send = nullptr;
  const me_fill* f0 = nullptr;  // rank 0's own outputs (direct: the engine slot's pinned memory)
  const me_order_result* r0 = nullptr;
  double t = now_s();
  if (rc == ME_OK && !c->use_ops && (direct || !c->tp->device()) && p.n) {  // host-slot batches: collect now
    const me_fill* f = nullptr;
    const me_order_result* r = nullptr;
    size_t nf = 0, nr = 0;
    rc = me_collect(c->eng, p.eng_ticket, &f, &nf, &r, &nr);
    if (rc == ME_OK) {
      p.nf = nf;
      if (direct) {
        f0 = f;
        r0 = r;
      } else {
        p.h_out.resize(round8(nf * sizeof(me_fill) + p.n * sizeof(me_order_result)));
        if (nf) memcpy(p.h_out.data(), f, nf * sizeof(me_fill));
        memcpy(p.h_out.data() + nf * sizeof(me_fill), r, p.n * sizeof(me_order_result));
      }
    }
  }
  if (me == 0) c->ph[PH_COLLECT] += now_s() - t;
  if (!agree(c, rc)) return c->tfail("status");
  p.used = false;
  if (rc != ME_OK) {
    c->failed = true;
    return c->fail(ME_E_STATE, "a shard lost its part of the slice");
  }
  t = now_s();
  // payloads padded to 8 B, so every rank's tape starts aligned in rank 0's gather buffer (rank 0's own
  // outputs, direct, stay where the engine put them)
  const size_t mine = direct ? 0 : round8(p.nf * sizeof(me_fill) + p.n * sizeof(me_order_result));
  char* staged = nullptr;  // a host payload (shard ops) on a device transport
  if (!mine) {
  } else if (c->tp->device() && !c->use_ops) {
    send = p.out;  // HBM to HBM: the engine's tape and results never left the device
  } else if (c->tp->device()) {
    staged = c->tp->alloc(mine);
    if (!staged || !c->tp->put(staged, p.h_out.data(), mine)) {
      c->tp->release(staged);
      return c->tfail("stage");
    }
    send = staged;
  } else {
    send = p.h_out.data();
  }
  // sizes to rank 0 (a rank needs only its own to post its send), then the payloads
  int64_t sz[2] = {(int64_t)p.nf, (int64_t)mine};
  std::vector<int64_t> szs(2 * W, 0);
  if (!c->tp->gather(sz, 2, szs.data())) {
    c->tp->release(staged);
    return c->tfail("size gather");
  }
  if (me != 0) szs[2 * me + 1] = (int64_t)mine;
  std::vector<size_t> bytes(W);
  size_t tot = 0;
  for (uint32_t r = 0; r < W; ++r) tot += (bytes[r] = (size_t)szs[2 * r + 1]);
  if (me == 0 && tot > c->t_gather_cap) {
    c->tp->release(c->t_gather);
    c->t_gather = c->tp->alloc(tot);
    c->t_gather_cap = c->t_gather ? tot : 0;
    if (!c->t_gather) {  // the protocol cannot go on: the others are already in the gather
      c->tp->release(staged);
      return c->tfail("gather buffer");
    }
  }
  const bool gok = (me == 0 ? tot == 0 : mine == 0) || c->tp->gatherv(send, bytes, c->t_gather);
  c->tp->release(staged);
  if (!gok) return c->tfail("gather");
  if (me != 0) return ME_OK;
  c->h_gather.resize(tot);
  if (tot && !c->tp->get(c->h_gather.data(), c->t_gather, tot)) return c->tfail("gather D2H");
  c->ph[PH_GATHER] += now_s() - t;
  t = now_s();
  const Ticket& tk = c->tickets.front();
  if (W == 1 && direct) {  // one shard: its tape and results are the slice's, in place
    c->out_tape = f0;
    c->out_nf = p.nf;
    c->out_res = r0;
  } else {
    std::vector<const me_fill*> tf(W);
    std::vector<const me_order_result*> tr(W);
    std::vector<size_t> nfs(W);
    size_t off = 0;
    for (uint32_t r = 0; r < W; ++r) {
      nfs[r] = (size_t)szs[2 * r];
      if (r == 0 && direct) {
        tf[0] = f0;
        tr[0] = r0;
      } else {
        tf[r] = (const me_fill*)(c->h_gather.data() + off);
        tr[r] = (const me_order_result*)(c->h_gather.data() + off + nfs[r] * sizeof(me_fill));
        off += bytes[r];
      }
    }
    uint32_t bad = 0;
    if (!merge_parts(W, tk, tr, tf, nfs, c->res, c->tape, &bad)) {
      c->failed = true;
      return c->fail(ME_E_STATE, "shard " + std::to_string(bad) + "'s results do not account for its tape");
    }
    const me_fill* tape = c->tape.data();
    const me_order_result* res = c->res.data();
    c->out_tape = tape;
    c->out_nf = c->tape.size();
    c->out_res = res;
  }
  c->ph[PH_MERGE] += now_s() - t;
  c->tickets.pop_front();
  c->slices++;
  return ME_OK;
}

// Payload of BOOK / SNAPSHOT from each rank to rank 0 (host bytes in, host bytes out on rank 0).
static bool gather_host(me_cluster* c, const std::vector<char>& mine, std::vector<char>& all,
                        std::vector<size_t>& bytes) {
  const uint32_t W = c->cfg.world;
  int64_t sz = (int64_t)round8(mine.size());
  std::vector<int64_t> szs(W, 0);
  if (!c->tp->gather(&sz, 1, szs.data())) return false;
  szs[c->cfg.rank] = sz;
  bytes.resize(W);
  size_t tot = 0;
  for (uint32_t r = 0; r < W; ++r) tot += (bytes[r] = (size_t)szs[r]);
  std::vector<char> padded(mine);
  padded.resize((size_t)sz);
  char* tbuf = c->tp->alloc((size_t)sz);
  if (!tbuf || !c->tp->put(tbuf, padded.data(), (size_t)sz)) {
    c->tp->release(tbuf);
    return false;
  }
  const char* send = tbuf;
  char* rbuf = nullptr;
  if (c->cfg.rank == 0) {
    rbuf = c->tp->alloc(tot);
    if (!rbuf) {
      c->tp->release(tbuf);
      return false;
    }
  }
  bool ok = c->tp->gatherv(send, bytes, rbuf);
  if (ok && c->cfg.rank == 0) {
    all.resize(tot);
    ok = c->tp->get(all.data(), rbuf, tot);
  }
  c->tp->release(tbuf);
  c->tp->release(rbuf);
  return ok;
}

struct BookReq {  // rank 0's caller buffers for BOOK
  me_book_entry* bids;
  size_t bids_cap;
  size_t* n_bids;
  me_book_entry* asks;
  size_t asks_cap;
  size_t* n_asks;
  me_level* bl;
  me_level* al;
  size_t* nbl;
  size_t* nal;
};

static int run_book(me_cluster* c, const int64_t* hdr, const BookReq* q) {
  const uint32_t sym = (uint32_t)hdr[3], depth = (uint32_t)hdr[4];
  const bool known = sym < c->cfg.num_symbols;
  const uint32_t own = known ? c->owner[sym] : 0;
  std::vector<char> mine;
  int rc = ME_OK;
  if (known && own == c->cfg.rank && !c->failed) {
    const uint32_t ls = c->local[sym];
    uint32_t d = depth;
    if (!d && !c->use_ops) d = 0xFFFFFFFFu;  // the whole book: every window level plus the far levels
    auto call = [&](me_book_entry* b, size_t bc, size_t* nb, me_book_entry* a, size_t ac, size_t* na, me_level* bl,
                    me_level* al, size_t* nbl, size_t* nal) {
      return c->use_ops ? c->ops.book(c->ops.ctx, ls, d, b, bc, nb, a, ac, na, bl, al, nbl, nal)
                        : me_book_orders(c->eng, ls, d, b, bc, nb, a, ac, na, bl, al, nbl, nal);
    };
    size_t nb = 0, na = 0, nbl = 0, nal = 0;
    rc = c->use_ops && !c->ops.book ? ME_E_INVALID : call(nullptr, 0, &nb, nullptr, 0, &na, nullptr, nullptr, &nbl, &nal);
    if (rc == ME_OK) {
      std::vector<me_book_entry> eb(std::max<size_t>(nb, 1)), ea(std::max<size_t>(na, 1));
      // (level buffers as long as the first call's counts: d may be 0xFFFFFFFF, "the whole book")
      std::vector<me_level> lb(std::max<size_t>(std::min<size_t>(nbl, d), 1)), la(std::max<size_t>(std::min<size_t>(nal, d), 1));
      rc = call(eb.data(), nb, &nb, ea.data(), na, &na, d ? lb.data() : nullptr, d ? la.data() : nullptr, &nbl, &nal);
      nbl = std::min<size_t>(nbl, d);
      nal = std::min<size_t>(nal, d);
      if (rc == ME_OK) {
        const int64_t h4[4] = {(int64_t)nb, (int64_t)na, (int64_t)nbl, (int64_t)nal};
        mine.resize(32 + (nb + na) * sizeof(me_book_entry) + (nbl + nal) * sizeof(me_level));
        char* w = mine.data();
        memcpy(w, h4, 32);
        w += 32;
        memcpy(w, eb.data(), nb * sizeof(me_book_entry));
        w += nb * sizeof(me_book_entry);
        memcpy(w, ea.data(), na * sizeof(me_book_entry));
        w += na * sizeof(me_book_entry);
        memcpy(w, lb.data(), nbl * sizeof(me_level));
        w += nbl * sizeof(me_level);
        memcpy(w, la.data(), nal * sizeof(me_level));
      }
    }
  }
  if (!agree(c, rc)) return c->tfail("status");
  if (rc != ME_OK) return c->fail(rc, "the owning shard failed the book read");
  std::vector<char> all;
  std::vector<size_t> bytes;
  if (!gather_host(c, mine, all, bytes)) return c->tfail("book gather");
  if (c->cfg.rank != 0) return ME_OK;
  size_t n4[4] = {0, 0, 0, 0};
  const char* r = nullptr;
  if (known) {
    size_t off = 0;
    for (uint32_t k = 0; k < own; ++k) off += bytes[k];
    r = all.data() + off;
    int64_t h4[4];
    memcpy(h4, r, 32);
    for (int k = 0; k < 4; ++k) n4[k] = (size_t)h4[k];
    r += 32;
  }
  if (q->n_bids) *q->n_bids = n4[0];
  if (q->n_asks) *q->n_asks = n4[1];
  if (q->nbl) *q->nbl = n4[2];
  if (q->nal) *q->nal = n4[3];
  if (!known) return ME_OK;
  if (q->bids) memcpy(q->bids, r, std::min(n4[0], q->bids_cap) * sizeof(me_book_entry));
  r += n4[0] * sizeof(me_book_entry);
  if (q->asks) memcpy(q->asks, r, std::min(n4[1], q->asks_cap) * sizeof(me_book_entry));
  r += n4[1] * sizeof(me_book_entry);
  if (depth && q->bl) memcpy(q->bl, r, n4[2] * sizeof(me_level));  // at most depth levels each
  r += n4[2] * sizeof(me_level);
  if (depth && q->al) memcpy(q->al, r, n4[3] * sizeof(me_level));
  return ME_OK;
}

static int run_snapshot(me_cluster* c, const int64_t* hdr, me_level* levels, uint32_t* counts) {
  const uint32_t depth = (uint32_t)hdr[3];
  const std::vector<uint32_t>& mine_ids = c->members[c->cfg.rank];
  const size_t ns = mine_ids.size();
  std::vector<char> mine;
  int rc = ME_OK;
  if (ns && depth && !c->failed) {
    std::vector<me_level> lv(ns * 2 * depth);
    std::vector<uint32_t> cnt(ns * 2);
    if (c->use_ops)
      rc = c->ops.levels_all ? c->ops.levels_all(c->ops.ctx, depth, lv.data(), cnt.data()) : ME_E_INVALID;
    else
      rc = me_book_levels_all(c->eng, depth, lv.data(), cnt.data());
    if (rc == ME_OK) {
      mine.resize(lv.size() * sizeof(me_level) + cnt.size() * 4);
      memcpy(mine.data(), lv.data(), lv.size() * sizeof(me_level));
      memcpy(mine.data() + lv.size() * sizeof(me_level), cnt.data(), cnt.size() * 4);
    }
  }
  if (!agree(c, rc)) return c->tfail("status");
  if (rc != ME_OK) return c->fail(rc, "a shard failed its level snapshot");
  std::vector<char> all;
  std::vector<size_t> bytes;
  if (!gather_host(c, mine, all, bytes)) return c->tfail("snapshot gather");
  if (c->cfg.rank != 0 || !depth) return ME_OK;
  const size_t S = c->cfg.num_symbols;
  if (levels) memset(levels, 0, S * 2 * depth * sizeof(me_level));
  if (counts) memset(counts, 0, S * 2 * 4);
  size_t off = 0;
  for (uint32_t r = 0; r < c->cfg.world; ++r) {
    const auto& ids = c->members[r];
    if (ids.size() && bytes[r]) {
      const me_level* lv = (const me_level*)(all.data() + off);
      const uint32_t* cnt = (const uint32_t*)(all.data() + off + ids.size() * 2 * depth * sizeof(me_level));
      for (size_t k = 0; k < ids.size(); ++k) {
        if (levels) memcpy(levels + (size_t)ids[k] * 2 * depth, lv + k * 2 * depth, 2 * depth * sizeof(me_level));
        if (counts) memcpy(counts + (size_t)ids[k] * 2, cnt + k * 2, 8);
      }
    }
    off += bytes[r];
  }
  return ME_OK;
}

static int dispatch(me_cluster* c, const int64_t* hdr, const BookReq* q, me_level* levels, uint32_t* counts) {
  switch (hdr[0]) {
    case CMD_SUBMIT:
      return run_submit(c, hdr);
    case CMD_COLLECT:
      return run_collect(c, hdr);
    case CMD_BOOK:
      return run_book(c, hdr, q);
    case CMD_SNAPSHOT:
      return run_snapshot(c, hdr, levels, counts);
    case CMD_STOP:
      c->stopped = true;
      return ME_OK;
  }
  return c->fail(ME_E_STATE, "unknown command");
}

extern "C" int me_cluster_serve(me_cluster* c) {
  if (!c) return ME_E_INVALID;
  if (c->cfg.rank == 0) return c->fail(ME_E_INVALID, "rank 0 issues the commands; it does not serve");
  std::vector<int64_t> hdr(c->hdr_words());
  while (!c->stopped) {
    if (!c->tp->bcast(hdr.data(), hdr.size())) return c->tfail("command channel");
    BookReq none{};
    (void)dispatch(c, hdr.data(), &none, nullptr, nullptr);  // failures are agreed on inside
  }
  return ME_OK;
}

static int issue(me_cluster* c, std::vector<int64_t>& hdr, const BookReq* q = nullptr, me_level* levels = nullptr,
                 uint32_t* counts = nullptr) {
  if (c->cfg.rank != 0) return c->fail(ME_E_INVALID, "only rank 0 issues commands");
  if (c->stopped) return c->fail(ME_E_STATE, "cluster stopped");
  const double t = now_s();
  if (!c->tp->bcast(hdr.data(), hdr.size())) return c->tfail("command channel");
  c->ph[PH_CTRL] += now_s() - t;
  BookReq none{};
  return dispatch(c, hdr.data(), q ? q : &none, levels, counts);
}

extern "C" int me_cluster_submit(me_cluster* c, const me_order_soa* b, size_t n, uint64_t* ticket) {
  if (!c || !b || !ticket) return ME_E_INVALID;
  if (c->failed) return c->fail(ME_E_STATE, "cluster failed: " + c->err);
  if (n == 0 || n > c->cfg.max_batch) return c->fail(ME_E_INVALID, "slice size must be in [1, max_batch]");
  if (c->tickets.size() >= (size_t)kMaxInflight) return c->fail(ME_E_STATE, "two slices in flight: collect first");
  const uint32_t W = c->cfg.world, S = c->cfg.num_symbols;
  double t = now_s();
  Ticket tk;
  tk.t = c->next_ticket;
  tk.n = n;
  std::vector<int64_t> hdr(c->hdr_words(), 0);
  hdr[0] = CMD_SUBMIT;
  hdr[1] = (int64_t)tk.t;
  hdr[2] = (int64_t)n;
  SplitCounts sc;
  split_count(c->owner.data(), W, S, b, n, sc);
  for (uint32_t r = 0; r < W; ++r) {
    hdr[6 + r] = (int64_t)sc.per_rank[r];
    hdr[6 + W + r] = (int64_t)sc.lim_rank[r];
  }
  c->ph[PH_SPLIT_COUNT] += now_s() - t;
  // where each rank's part goes: rank 0's into its engine's slot inputs (direct), the others' packed into
  // h_send in rank order
  const size_t n0 = (size_t)hdr[6];
  std::vector<PackView> dst;
  dst.reserve(W);
  c->h_send.resize(kRec * n);
  {
    size_t off = 0;
    for (uint32_t r = 0; r < W; ++r) {
      const size_t nr = (size_t)hdr[6 + r];
      if (r == 0 && c->direct0 && n0) {
        me_order_soa_w w{};
        const double ts = now_s();
        if (me_host_inputs(c->eng, n0, &w) != ME_OK) return c->fail(ME_E_STATE, "rank 0 slot inputs: " + eng_err(c->eng));
        c->ph[PH_SPLIT_SLOT] += now_s() - ts;
        PackView v(c->h_send.data(), 0);
        v.seq = w.seq;
        v.px = w.price_q4;
        v.qty = w.qty;
        v.sym = w.symbol;
        v.kind = w.kind;
        dst.push_back(v);
        c->w0 = me_order_soa{w.seq, w.price_q4, w.qty, w.symbol, w.kind};
        continue;
      }
      if (r == 0 && c->direct0) {
        dst.push_back(PackView(c->h_send.data(), 0));
        continue;
      }
      dst.push_back(PackView(c->h_send.data() + off, nr));
      off += kRec * nr;
    }
  }
  split_pack(c->owner.data(), c->local.data(), W, S, b, n, sc, dst, tk);
  c->ph[PH_SPLIT] += now_s() - t;
  const int rc = issue(c, hdr);
  if (rc != ME_OK) return rc;
  c->tickets.push_back(std::move(tk));
  *ticket = c->next_ticket++;
  return ME_OK;
}

extern "C" int me_cluster_collect(me_cluster* c, uint64_t ticket, const me_fill** fills, size_t* n_fills,
                                  const me_order_result** results) {
  if (!c) return ME_E_INVALID;
  if (c->tickets.empty() || c->tickets.front().t != ticket)
    return c->fail(ME_E_INVALID, "tickets are collected in submission order");
  std::vector<int64_t> hdr(c->hdr_words(), 0);
  hdr[0] = CMD_COLLECT;
  hdr[1] = (int64_t)ticket;
  const int rc = issue(c, hdr);
  if (rc != ME_OK) return rc;
  if (fills) *fills = c->out_tape;
  if (n_fills) *n_fills = c->out_nf;
  if (results) *results = c->out_res;
  return ME_OK;
}

extern "C" int me_cluster_match(me_cluster* c, const me_order_soa* b, size_t n, const me_fill** fills,
                                size_t* n_fills, const me_order_result** results) {
  uint64_t t = 0;
  const int rc = me_cluster_submit(c, b, n, &t);
  if (rc != ME_OK) return rc;
  return me_cluster_collect(c, t, fills, n_fills, results);
}

extern "C" int me_cluster_book(me_cluster* c, uint32_t symbol, uint32_t depth, me_book_entry* bids, size_t bids_cap,
                               size_t* n_bids, me_book_entry* asks, size_t asks_cap, size_t* n_asks,
                               me_level* bid_levels, me_level* ask_levels, size_t* n_bid_levels,
                               size_t* n_ask_levels) {
  if (!c) return ME_E_INVALID;
  std::vector<int64_t> hdr(c->hdr_words(), 0);
  hdr[0] = CMD_BOOK;
  hdr[3] = symbol;
  hdr[4] = depth;
  BookReq q{bids, bids_cap, n_bids, asks, asks_cap, n_asks, bid_levels, ask_levels, n_bid_levels, n_ask_levels};
  return issue(c, hdr, &q);
}

extern "C" int me_cluster_snapshot(me_cluster* c, uint32_t depth, me_level* levels, uint32_t* counts) {
  if (!c) return ME_E_INVALID;
  std::vector<int64_t> hdr(c->hdr_words(), 0);
  hdr[0] = CMD_SNAPSHOT;
  hdr[3] = depth;
  return issue(c, hdr, nullptr, levels, counts);
}

extern "C" int me_cluster_stop(me_cluster* c) {
  if (!c) return ME_E_INVALID;
  std::vector<int64_t> hdr(c->hdr_words(), 0);
  hdr[0] = CMD_STOP;
  return issue(c, hdr);
}

// ---- the service's matcher ------------------------------------------------------------------------
static int m_match(void* ctx, const me_order_soa* b, size_t n, const me_fill** f, size_t* nf,
                   const me_order_result** r) {
  return me_cluster_match((me_cluster*)ctx, b, n, f, nf, r);
}
static int m_book(void* ctx, uint32_t s, uint32_t d, me_book_entry* b, size_t bc, size_t* nb, me_book_entry* a,
                  size_t ac, size_t* na, me_level* bl, me_level* al, size_t* nbl, size_t* nal) {
  return me_cluster_book((me_cluster*)ctx, s, d, b, bc, nb, a, ac, na, bl, al, nbl, nal);
}
static int m_submit(void* ctx, const me_order_soa* b, size_t n, uint64_t* t) {
  return me_cluster_submit((me_cluster*)ctx, b, n, t);
}
static int m_collect(void* ctx, uint64_t t, const me_fill** f, size_t* nf, const me_order_result** r) {
  return me_cluster_collect((me_cluster*)ctx, t, f, nf, r);
}

extern "C" int me_cluster_matcher(me_cluster* c, me_matcher* out) {
  if (!c || !out) return ME_E_INVALID;
  if (c->cfg.rank != 0) return c->fail(ME_E_INVALID, "the matcher lives on rank 0");
  memset(out, 0, sizeof *out);
  out->ctx = c;
  out->num_symbols = c->cfg.num_symbols;
  out->max_batch = c->cfg.max_batch;
  out->max_resting = c->max_resting_total;  // every shard's resting orders can sweep into one slice
  out->match = m_match;
  out->book = m_book;
  out->submit = m_submit;
  out->collect = m_collect;
  return ME_OK;
}

extern "C" int me_cluster_stats(const me_cluster* c, uint64_t* slices, uint64_t* bytes) {
  if (!c) return ME_E_INVALID;
  if (slices) *slices = c->slices;
  if (bytes) *bytes = c->tp ? c->tp->moved : 0;
  return ME_OK;
}

extern "C" int me_cluster_phases(const me_cluster* c, double* seconds, size_t n) {
  if (!c) return ME_E_INVALID;
  for (size_t k = 0; k < n && k < (size_t)PH_N; ++k) seconds[k] = c->ph[k];
  return PH_N;
}

extern "C" int me_cluster_last_error(const me_cluster* c, char* buf, size_t cap) {
  std::string s;
  if (c) {
    s = c->err;
  } else {
    std::lock_guard<std::mutex> lk(g_err_mu);
    s = g_create_err;
  }
  if (buf && cap) {
    const size_t k = std::min(cap - 1, s.size());
    memcpy(buf, s.data(), k);
    buf[k] = 0;
  }
  return (int)s.size();
}

// Rank 0's host work per slice at `world` shards without any GPU or transport (does rank 0
// keep up with 100M orders/s at W = 8?): the exact split (split_count + split_pack into packed parts, the
// path of every rank but a direct rank 0) and merge (merge_parts) code of me_cluster_submit / collect, over
// `slice` with synthetic shard outputs — each record of a part gets floor((k + 1) F) - floor(k F) fills
// (mean F = fills_per_order), tapes laid out as a shard returns them. seconds[0..3] = per-slice mean of the
// owner-count pass, the pack, the merge, and the merged tape's length (fills).
extern "C" int me_cluster_host_probe(uint32_t world, uint32_t num_symbols, const me_order_soa* slice, size_t n,
                                     double fills_per_order, uint32_t iters, double* seconds) {
  if (!world || !num_symbols || !slice || !n || !iters || !seconds || fills_per_order < 0) return ME_E_INVALID;
  const uint32_t W = world, S = num_symbols;
  std::vector<uint32_t> owner(S), local(S), cntl(W, 0);
  for (uint32_t s = 0; s < S; ++s) {
    owner[s] = me_shard_of(s, W);
    local[s] = cntl[owner[s]]++;
  }
  std::vector<char> h_send(kRec * n);
  // synthetic shard outputs, sized from a first split
  SplitCounts sc;
  split_count(owner.data(), W, S, slice, n, sc);
  std::vector<std::vector<me_order_result>> rres(W);
  std::vector<std::vector<me_fill>> rtape(W);
  std::vector<const me_order_result*> tr(W);
  std::vector<const me_fill*> tf(W);
  std::vector<size_t> nf(W);
  for (uint32_t r = 0; r < W; ++r) {
    const size_t np = sc.per_rank[r];
    rres[r].assign(np, me_order_result{});
    uint64_t o = 0;
    for (size_t k = 0; k < np; ++k) {
      const uint32_t fc = (uint32_t)(std::floor((k + 1) * fills_per_order) - std::floor(k * fills_per_order));
      rres[r][k].fill_count = fc;
      rres[r][k].tape_offset = (uint32_t)o;
      rres[r][k].status = fc ? ME_ST_FILLED : ME_ST_NEW;
      o += fc;
    }
    rtape[r].assign(o, me_fill{});
    for (uint64_t f = 0; f < o; ++f) rtape[r][f].qty = 1;
    tr[r] = rres[r].data();
    tf[r] = rtape[r].data();
    nf[r] = o;
  }
  std::vector<me_order_result> res;
  std::vector<me_fill> tape;
  double t_count = 0, t_pack = 0, t_merge = 0;
  for (uint32_t it = 0; it < iters; ++it) {
    Ticket tk;
    tk.n = n;
    double t = now_s();
    SplitCounts c2;
    split_count(owner.data(), W, S, slice, n, c2);
    t_count += now_s() - t;
    std::vector<PackView> dst;
    size_t off = 0;
    for (uint32_t r = 0; r < W; ++r) {
      dst.push_back(PackView(h_send.data() + off, c2.per_rank[r]));
      off += kRec * c2.per_rank[r];
    }
    split_pack(owner.data(), local.data(), W, S, slice, n, c2, dst, tk);
    t_pack += now_s() - t;
    t = now_s();
    uint32_t bad = 0;
    if (!merge_parts(W, tk, tr, tf, nf, res, tape, &bad)) return ME_E_STATE;
    t_merge += now_s() - t;
  }
  seconds[0] = t_count / iters;
  seconds[1] = (t_pack - t_count) / iters;
  seconds[2] = t_merge / iters;
  seconds[3] = (double)tape.size();
  return ME_OK;
}

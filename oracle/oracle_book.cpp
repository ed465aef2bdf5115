// oracle_book.cpp — CPU ORACLE. TEST INFRASTRUCTURE ONLY.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
// and only as the checker / the timed CPU baseline — never as part of the product path.
//
// What it restates:
//  * orc_submit_order: the reference SubmitOrder handler, src/server/matching_engine_service.cpp:41-121
//      validation order + strings :66-83, OID allocation :85 / :29-32 (consumed even when
//      normalization throws), Order::FromRaw -> normalize_to_q4 include/domain/price.hpp:15-29,
//      persist Storage::insert_new_order src/storage/storage.cpp:78-123 (side CHECK -> "DB insert
//      failed", order_id still returned :107-111), persisted row incl. the order_type=1 quirk :106.
//  * orc_submit: the matching core. The reference has NO matcher (include/engine/model.hpp is 0
//      bytes), so fills are "parity unpinned" by the reference; this scalar price-time book is the
//      golden model defined in DESIGN.md §2 (derived from the declared-but-unimplemented contract:
//      OrderUpdate.Status proto/matching_engine.proto:79-85, FillRow include/storage/storage.hpp:11-17).
//      It deliberately shares no data structure and no limit with the GPU design: std::map price
//      levels over the whole int64 Q4 range (include/domain/price.hpp:6), std::deque FIFOs, and an
//      unbounded seq -> order map (OIDs are an unbounded u64, matching_engine_service.cpp:29-32).
//      The only admission rules are the domain's: BAD_QTY, BAD_SIDE (storage.cpp:32 CHECK),
//      BAD_SYMBOL, and seq 0 (no OID is ever 0: the counter starts at 1, storage.cpp:254-267).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <deque>
#include <functional>
#include <map>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../include/me_engine.h"

namespace {

struct Entry {
  uint64_t seq;
  int32_t qty;  // 0 = dead (cancelled or filled, awaiting pop)
};

struct Level {
  int64_t total = 0;
  std::deque<Entry> q;
};

struct Book {
  std::map<int64_t, Level, std::greater<int64_t>> bids;  // best (highest) first
  std::map<int64_t, Level> asks;                          // best (lowest) first
};

struct Where {
  uint32_t sym;
  uint8_t side;
  int64_t price;
  Entry* e;
};

}  // namespace

struct orc {
  uint32_t S;
  std::vector<Book> books;
  std::unordered_map<uint64_t, Where> where;  // live resting orders only
  uint64_t resting = 0;
};

extern "C" orc* orc_create(uint32_t S) {
  orc* o = new orc();
  o->S = S;
  o->books.resize(S);
  o->where.reserve(1 << 20);
  return o;
}

extern "C" void orc_destroy(orc* o) { delete o; }

extern "C" uint64_t orc_resting(const orc* o) { return o->resting; }

template <class Map>
static int64_t match_side(orc* o, Map& side, uint32_t sym, bool market, int64_t limit, bool buy, uint64_t taker,
                          int64_t want, std::vector<me_fill>& tape, uint32_t gsym) {
  int64_t rem = want;
  while (rem > 0 && !side.empty()) {
    auto it = side.begin();
    const int64_t px = it->first;
    if (!market && (buy ? px > limit : px < limit)) break;
    Level& lv = it->second;
    while (rem > 0 && !lv.q.empty()) {
      Entry& m = lv.q.front();
      if (m.qty == 0) {
        lv.q.pop_front();
        continue;
      }
      const int64_t f = rem < m.qty ? rem : m.qty;
      tape.push_back(me_fill{taker, m.seq, px, (int32_t)f, gsym});
      m.qty -= (int32_t)f;
      lv.total -= f;
      rem -= f;
      if (m.qty == 0) {
        o->where.erase(m.seq);
        lv.q.pop_front();
        o->resting--;
      }
    }
    if (lv.total == 0) side.erase(it);
  }
  (void)sym;
  return want - rem;
}

// One batch in seq order into res_out[n]; its fills appended to `tape` in taker order.
static void submit_core(orc* o, size_t n, const uint64_t* seq, const int64_t* px, const int32_t* qty,
                        const uint32_t* sym, const uint8_t* kind, const uint32_t* gsym_map, me_order_result* res_out,
                        std::vector<me_fill>& tape) {
  for (size_t i = 0; i < n; ++i) {
    me_order_result r{};
    r.tape_offset = (uint32_t)tape.size();
    const uint32_t s = sym[i];
    const uint32_t k = kind[i];
    const uint32_t side = k & 3u;
    const bool market = (k >> 2) & 1u;
    const bool cancel = (k >> 3) & 1u;
    const int32_t q = qty[i];
    if (s >= o->S) {
      r.status = ME_ST_REJECTED;
      r.reason = ME_RJ_BAD_SYMBOL;
      res_out[i] = r;
      continue;
    }
    if (cancel) {
      auto it = o->where.find((uint64_t)px[i]);
      if (it == o->where.end() || it->second.sym != s) {
        r.status = ME_ST_REJECTED;
        r.reason = ME_RJ_UNKNOWN_ORDER;
      } else {
        Where w = it->second;
        const int32_t got = w.e->qty;
        w.e->qty = 0;
        o->where.erase(it);
        o->resting--;
        Book& b = o->books[s];
        if (w.side == ME_SIDE_BUY) {
          auto lit = b.bids.find(w.price);
          lit->second.total -= got;
          if (lit->second.total == 0) b.bids.erase(lit);
        } else {
          auto lit = b.asks.find(w.price);
          lit->second.total -= got;
          if (lit->second.total == 0) b.asks.erase(lit);
        }
        r.status = ME_ST_CANCELED;
        r.remaining_qty = got;
      }
      res_out[i] = r;
      continue;
    }
    if (q <= 0) {
      r.status = ME_ST_REJECTED;
      r.reason = ME_RJ_BAD_QTY;
      res_out[i] = r;
      continue;
    }
    r.remaining_qty = q;
    if (side != ME_SIDE_BUY && side != ME_SIDE_SELL) {
      r.status = ME_ST_REJECTED;
      r.reason = ME_RJ_BAD_SIDE;
      res_out[i] = r;
      continue;
    }
    if (seq[i] == 0) {
      r.status = ME_ST_REJECTED;
      r.reason = ME_RJ_BAD_SEQ;
      res_out[i] = r;
      continue;
    }
    const bool buy = side == ME_SIDE_BUY;
    const uint32_t gs = gsym_map ? gsym_map[s] : s;
    Book& b = o->books[s];
    const size_t t0 = tape.size();
    const int64_t filled = buy ? match_side(o, b.asks, s, market, px[i], true, seq[i], q, tape, gs)
                               : match_side(o, b.bids, s, market, px[i], false, seq[i], q, tape, gs);
    const int32_t rem = q - (int32_t)filled;
    r.filled_qty = (int32_t)filled;
    r.remaining_qty = rem;
    r.fill_count = (uint32_t)(tape.size() - t0);
    if (market) {
      r.status = rem == 0 ? ME_ST_FILLED : ME_ST_CANCELED;
    } else {
      if (rem > 0) {
        Level& lv = buy ? b.bids[px[i]] : b.asks[px[i]];
        lv.q.push_back(Entry{seq[i], rem});
        lv.total += rem;
        o->where[seq[i]] = Where{s, (uint8_t)side, px[i], &lv.q.back()};
        o->resting++;
      }
      r.status = rem == 0 ? ME_ST_FILLED : (filled > 0 ? ME_ST_PARTIALLY_FILLED : ME_ST_NEW);
    }
    res_out[i] = r;
  }
}

// One batch in seq order. res_out[n]; fills appended in taker order.
extern "C" int orc_submit(orc* o, size_t n, const uint64_t* seq, const int64_t* px, const int32_t* qty,
                          const uint32_t* sym, const uint8_t* kind, const uint32_t* gsym_map, me_order_result* res_out,
                          me_fill* fills_out, size_t fills_cap, size_t* nfills) {
  std::vector<me_fill> tape;
  tape.reserve(n * 2);
  submit_core(o, n, seq, px, qty, sym, kind, gsym_map, res_out, tape);
  if (nfills) *nfills = tape.size();
  if (fills_out) {
    if (tape.size() > fills_cap) return -3;
    memcpy(fills_out, tape.data(), tape.size() * sizeof(me_fill));
  }
  return 0;
}

// Resting state of one symbol: bids best-first, then asks best-first, FIFO inside a level.
extern "C" size_t orc_dump(const orc* o, uint32_t s, me_book_entry* out, size_t cap) {
  size_t k = 0;
  const Book& b = o->books[s];
  auto put = [&](int64_t px, const Entry& e, uint8_t side) {
    if (e.qty <= 0) return;
    if (out && k < cap) {
      me_book_entry be{};
      be.seq = e.seq;
      be.price_q4 = px;
      be.qty = e.qty;
      be.side = side;
      out[k] = be;
    }
    ++k;
  };
  for (auto& kv : b.bids)
    for (auto& e : kv.second.q) put(kv.first, e, ME_SIDE_BUY);
  for (auto& kv : b.asks)
    for (auto& e : kv.second.q) put(kv.first, e, ME_SIDE_SELL);
  return k;
}

// Top `depth` levels per side (GetOrderBook restatement on the oracle book).
extern "C" int orc_snapshot(const orc* o, uint32_t s, me_level* bids, me_level* asks, size_t depth, size_t* nb,
                            size_t* na) {
  const Book& b = o->books[s];
  size_t i = 0;
  for (auto& kv : b.bids) {
    if (i >= depth) break;
    uint32_t c = 0;
    for (auto& e : kv.second.q) c += e.qty > 0;
    if (bids) bids[i] = me_level{kv.first, kv.second.total, c, 0};
    ++i;
  }
  *nb = i;
  i = 0;
  for (auto& kv : b.asks) {
    if (i >= depth) break;
    uint32_t c = 0;
    for (auto& e : kv.second.q) c += e.qty > 0;
    if (asks) asks[i] = me_level{kv.first, kv.second.total, c, 0};
    ++i;
  }
  *na = i;
  return 0;
}

// ---------------------------------------------------------------------------------------------
// SubmitOrder restatement (src/server/matching_engine_service.cpp:41-121) without gRPC/SQLite:
// returns the OrderResponse fields and the row Storage::insert_new_order would persist.
struct orc_service {
  uint64_t next_id = 1;  // seeded from load_next_oid_seq (storage.cpp:254-267): 1 on a fresh DB
};

extern "C" orc_service* orc_service_create(uint64_t next_id) {
  orc_service* s = new orc_service();
  s->next_id = next_id;
  return s;
}
extern "C" void orc_service_destroy(orc_service* s) { delete s; }

// grpc_status: 0 OK, 2 UNKNOWN (escaping exception: scale out of range / overflow).
// persisted: 1 when a row was inserted; row fields in *row_*.
extern "C" int orc_service_submit(orc_service* svc, const char* symbol, int32_t order_type, int32_t side,
                                  int64_t price, int32_t scale, int32_t quantity, char* order_id, size_t oid_cap,
                                  int* success, char* error_message, size_t err_cap, int* grpc_status,
                                  int* persisted, int64_t* row_price, int32_t* row_order_type,
                                  int32_t* row_status, int64_t* row_remaining, int32_t* row_side) {
  auto put = [](char* dst, size_t cap, const std::string& v) {
    if (!dst || !cap) return;
    size_t k = v.size() < cap - 1 ? v.size() : cap - 1;
    memcpy(dst, v.data(), k);
    dst[k] = 0;
  };
  put(order_id, oid_cap, "");
  put(error_message, err_cap, "");
  *success = 0;
  *grpc_status = 0;
  *persisted = 0;
  // validation :66-83, first failing check wins, no OID allocated
  if (!symbol || !symbol[0]) {
    put(error_message, err_cap, "symbol is required");
    return 0;
  }
  if (quantity <= 0) {
    put(error_message, err_cap, "quantity must be > 0");
    return 0;
  }
  if (order_type == ME_TYPE_LIMIT && price <= 0) {
    put(error_message, err_cap, "price must be > 0 for LIMIT");
    return 0;
  }
  // OID :85 (allocated before normalization)
  const std::string oid = "OID-" + std::to_string(svc->next_id++);
  // Order::FromRaw -> normalize_to_q4 (include/domain/price.hpp:15-29), restated independently
  static const int64_t P10[19] = {1LL, 10LL, 100LL, 1000LL, 10000LL, 100000LL, 1000000LL, 10000000LL,
                                  100000000LL, 1000000000LL, 10000000000LL, 100000000000LL,
                                  1000000000000LL, 10000000000000LL, 100000000000000LL,
                                  1000000000000000LL, 10000000000000000LL, 100000000000000000LL,
                                  1000000000000000000LL};
  int64_t q4;
  if (scale < 0 || scale > 18) {
    *grpc_status = 2;
    put(error_message, err_cap, "scale out of range");
    return 0;
  }
  if (scale == 4) {
    q4 = price;
  } else if (scale < 4) {
    const int64_t mul = P10[4 - scale];
    if (price > 0 && price > INT64_MAX / mul) {
      *grpc_status = 2;
      put(error_message, err_cap, "overflow");
      return 0;
    }
    if (price < 0 && price < INT64_MIN / mul) {
      *grpc_status = 2;
      put(error_message, err_cap, "underflow");
      return 0;
    }
    q4 = price * mul;
  } else {
    q4 = price / P10[scale - 4];
  }
  // persist :99-104 -> storage.cpp:78-123; CHECK side IN (1,2) and quantity > 0 (schema :32,35)
  put(order_id, oid_cap, oid);
  const bool ok = (side == ME_SIDE_BUY || side == ME_SIDE_SELL);
  *success = ok ? 1 : 0;
  if (!ok) {
    put(error_message, err_cap, "DB insert failed");
    return 0;
  }
  *persisted = 1;
  *row_price = q4;
  *row_order_type = 1;  // storage.cpp:106 binds the constant 1 (quirk)
  *row_status = 0;      // NEW
  *row_remaining = quantity;
  *row_side = side;
  return 0;
}

// ---------------------------------------------------------------------------------------------
// The CPU baseline at the host's cores (bench.py cpu_baseline): T books, one per
// std::thread, each over its own pre-split batches (symbols hash-sharded across threads as across GPUs:
// independent books, no shared state), with no Python in the timed loop. Thread r runs book books[r]
// through nb[r] batches: records [boff[r][j], boff[r][j + 1]) of its SoA arrays, results into a reused
// buffer, fills into a reused tape (cleared per batch). Every thread allocates and touches its buffers
// first; the clock starts when all are ready (a spin barrier) and stops when the last one finishes.
// The first nwarm batches of every thread run before the barrier, untimed (the allocator's arenas warm up:
// first-touch page faults of many threads serialise on the process's memory map). Returns the wall
// seconds of the rest; fills_out (optional) receives each thread's fill count over the timed batches.
extern "C" double orc_run_sharded(uint32_t T, uint32_t nwarm, orc* const* books, const uint32_t* nb,
                                  const uint64_t* const* boff,
                                  const uint64_t* const* seq, const int64_t* const* px, const int32_t* const* qty,
                                  const uint32_t* const* sym, const uint8_t* const* kind, uint64_t* fills_out) {
  std::atomic<uint32_t> ready{0};
  std::atomic<bool> go{false};
  std::vector<double> end(T, 0.0);
  std::chrono::steady_clock::time_point t0;
  std::vector<std::thread> th;
  th.reserve(T);
  for (uint32_t r = 0; r < T; ++r) {
    th.emplace_back([&, r]() {
      size_t mx = 0;
      for (uint32_t j = 0; j < nb[r]; ++j) mx = std::max<size_t>(mx, boff[r][j + 1] - boff[r][j]);
      std::vector<me_order_result> res(mx + 1);
      std::vector<me_fill> tape;
      tape.reserve(2 * mx + 16);
      uint64_t nf = 0;
      auto run = [&](uint32_t j) {
        const uint64_t a = boff[r][j], n = boff[r][j + 1] - a;
        tape.clear();
        submit_core(books[r], n, seq[r] + a, px[r] + a, qty[r] + a, sym[r] + a, kind[r] + a, nullptr, res.data(),
                    tape);
      };
      const uint32_t w0 = std::min(nwarm, nb[r]);
      for (uint32_t j = 0; j < w0; ++j) run(j);
      ready.fetch_add(1);
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      for (uint32_t j = w0; j < nb[r]; ++j) {
        run(j);
        nf += tape.size();
      }
      end[r] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (fills_out) fills_out[r] = nf;
    });
  }
  while (ready.load() < T) std::this_thread::yield();
  t0 = std::chrono::steady_clock::now();
  go.store(true, std::memory_order_release);
  for (auto& t : th) t.join();
  double w = 0;
  for (double x : end) w = std::max(w, x);
  return w;
}

// TEST INFRASTRUCTURE (CPU baseline only): the reference's SubmitOrder path restated as it runs per
// order today — bench.py --workload c1 times it on one core beside the build's batched path. Never
// linked into the product.
//
// Per order, in the reference's order of operations:
//   src/server/matching_engine_service.cpp:41-121  steady-clock start, the request log line
//     (std::endl: one flush), validation (:66-83), gen_order_id "OID-<n>" (:29-32, :85), the
//     "validated" log, Order::FromRaw -> normalize_to_q4 (include/domain/price.hpp:15-29), the
//     write mutex (:101-104), the outcome and duration logs;
//   src/storage/storage.cpp:78-123  insert_new_order: SQLite::Transaction (BEGIN), the log block
//     (two std::endl flushes), a fresh SQLite::Statement (prepare) for the 11-column INSERT, binds,
//     exec, commit, statement finalize — one transaction per order;
//   storage.cpp:9-24  the connection: OPEN_READWRITE|CREATE|FULLMUTEX, busy timeout 5000 ms,
//     PRAGMA journal_mode=WAL, synchronous=NORMAL, foreign_keys=ON, then the schema (:26-69).
// The logs go to a caller-chosen file descriptor (bench.py: /dev/null) through an ostream whose
// std::endl flushes, so each flush is the write(2) the server pays; the terminal is not timed.
// SQLite is dlopen'ed (libsqlite3.so.0) like the product's service, so no sqlite3 header is needed.
#include <dlfcn.h>
#include <stdint.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <ostream>
#include <streambuf>
#include <string>

namespace {

struct sqlite3;
struct sqlite3_stmt;
using destructor_t = void (*)(void*);

struct Sql {
  void* h = nullptr;
  int (*open_v2)(const char*, sqlite3**, int, const char*);
  int (*close)(sqlite3*);
  int (*exec)(sqlite3*, const char*, void*, void*, char**);
  int (*prepare_v2)(sqlite3*, const char*, int, sqlite3_stmt**, const char**);
  int (*bind_int64)(sqlite3_stmt*, int, long long);
  int (*bind_int)(sqlite3_stmt*, int, int);
  int (*bind_text)(sqlite3_stmt*, int, const char*, int, destructor_t);
  int (*step)(sqlite3_stmt*);
  int (*finalize)(sqlite3_stmt*);
  int (*busy_timeout)(sqlite3*, int);
  bool load() {
    if (h) return true;
    h = dlopen("libsqlite3.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) return false;
    bool ok = true;
    auto get = [&](auto& f, const char* n) {
      f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, n));
      ok = ok && f;
    };
    get(open_v2, "sqlite3_open_v2");
    get(close, "sqlite3_close");
    get(exec, "sqlite3_exec");
    get(prepare_v2, "sqlite3_prepare_v2");
    get(bind_int64, "sqlite3_bind_int64");
    get(bind_int, "sqlite3_bind_int");
    get(bind_text, "sqlite3_bind_text");
    get(step, "sqlite3_step");
    get(finalize, "sqlite3_finalize");
    get(busy_timeout, "sqlite3_busy_timeout");
    return ok;
  }
} g;

const destructor_t kTransient = reinterpret_cast<destructor_t>(-1);

// An ostream over a file descriptor: buffered, flushed by std::endl (one write per flush), like
// std::cout redirected to a file.
class FdBuf : public std::streambuf {
 public:
  explicit FdBuf(int fd) : fd_(fd) { setp(buf_, buf_ + sizeof buf_); }
  ~FdBuf() override { sync(); }

 protected:
  int overflow(int c) override {
    if (sync() != 0) return traits_type::eof();
    if (c != traits_type::eof()) {
      *pptr() = (char)c;
      pbump(1);
    }
    return c;
  }
  int sync() override {
    const ptrdiff_t n = pptr() - pbase();
    if (n > 0 && ::write(fd_, pbase(), (size_t)n) != n) return -1;
    setp(buf_, buf_ + sizeof buf_);
    return 0;
  }

 private:
  int fd_;
  char buf_[4096];
};

int64_t now_ms() {
  using namespace std::chrono;
  return duration_cast<milliseconds>(system_clock::now().time_since_epoch()).count();
}

// include/domain/price.hpp:15-29 (restated): 0 ok, nonzero = the exception it throws.
int to_q4(int64_t price, int32_t scale, int64_t* out) {
  static const int64_t P10[19] = {1LL, 10LL, 100LL, 1000LL, 10000LL, 100000LL, 1000000LL, 10000000LL,
                                  100000000LL, 1000000000LL, 10000000000LL, 100000000000LL, 1000000000000LL,
                                  10000000000000LL, 100000000000000LL, 1000000000000000LL, 10000000000000000LL,
                                  100000000000000000LL, 1000000000000000000LL};
  if (scale < 0 || scale > 18) return 1;
  if (scale == 4) {
    *out = price;
    return 0;
  }
  if (scale < 4) {
    const int64_t mul = P10[4 - scale];
    if ((price > 0 && price > INT64_MAX / mul) || (price < 0 && price < INT64_MIN / mul)) return 2;
    *out = price * mul;
    return 0;
  }
  *out = price / P10[scale - 4];
  return 0;
}

const char* kSchema =
    "CREATE TABLE IF NOT EXISTS orders (order_id TEXT PRIMARY KEY, client_id TEXT NOT NULL, symbol TEXT NOT NULL,"
    " side INTEGER NOT NULL CHECK (side IN (1,2)), order_type INTEGER NOT NULL, price INTEGER,"
    " quantity INTEGER NOT NULL CHECK (quantity > 0), status INTEGER NOT NULL, remaining_quantity INTEGER NOT NULL,"
    " created_ts INTEGER NOT NULL, updated_ts INTEGER NOT NULL);"
    "CREATE INDEX IF NOT EXISTS idx_orders_symbol_side ON orders(symbol, side);"
    "CREATE INDEX IF NOT EXISTS idx_orders_client ON orders(client_id);"
    "CREATE TABLE IF NOT EXISTS fills (id INTEGER PRIMARY KEY AUTOINCREMENT, order_id TEXT NOT NULL,"
    " symbol TEXT NOT NULL, fill_price INTEGER NOT NULL, fill_quantity INTEGER NOT NULL, event_ts INTEGER NOT NULL,"
    " FOREIGN KEY(order_id) REFERENCES orders(order_id));"
    "CREATE INDEX IF NOT EXISTS idx_fills_order ON fills(order_id);";

}  // namespace

// Run n SubmitOrder calls (all from client_id / symbol) against a fresh SQLite DB at db_path, one
// transaction per accepted order. ok[i] = OrderResponse.success; returns the number of rows written
// or -1 when SQLite cannot be opened.
extern "C" long long ref_submit_run(const char* db_path, const char* client_id, const char* symbol, size_t n,
                                    const int32_t* order_type, const int32_t* side, const int64_t* price,
                                    const int32_t* scale, const int32_t* quantity, int log_fd, uint8_t* ok) {
  if (!g.load()) return -1;
  sqlite3* db = nullptr;
  if (g.open_v2(db_path, &db, 0x2 | 0x4 | 0x10000, nullptr) != 0) return -1;
  g.busy_timeout(db, 5000);
  g.exec(db, "PRAGMA journal_mode=WAL;", nullptr, nullptr, nullptr);
  g.exec(db, "PRAGMA synchronous=NORMAL;", nullptr, nullptr, nullptr);
  g.exec(db, "PRAGMA foreign_keys=ON;", nullptr, nullptr, nullptr);
  g.exec(db, kSchema, nullptr, nullptr, nullptr);
  FdBuf buf(log_fd);
  std::ostream out(&buf);
  std::atomic<uint64_t> next_oid{1};  // Impl::next_oid, seeded 1 on a fresh DB
  std::mutex write_mu;
  const std::string client(client_id), sym(symbol);
  long long rows = 0;
  for (size_t i = 0; i < n; ++i) {
    ok[i] = 0;
    const auto t0 = std::chrono::steady_clock::now();
    const bool limit = order_type[i] == 0;
    out << "[SERVER] [SubmitOrder] ============================================================= New Order\n"
        << " client_id=" << client << " symbol=" << sym << " side=" << (side[i] == 1 ? "BUY" : "SELL")
        << " type=" << (limit ? "LIMIT" : "MARKET") << " price=" << (limit ? std::to_string(price[i]) : "NULL")
        << " scale=" << scale[i] << " qty=" << quantity[i] << std::endl;
    if (sym.empty() || quantity[i] <= 0 || (limit && price[i] <= 0)) continue;  // in-band rejects
    const std::string oid = "OID-" + std::to_string(next_oid.fetch_add(1, std::memory_order_relaxed));
    out << "[SERVER] [SubmitOrder] oid=" << oid << " validated\n";
    int64_t q4 = 0;
    if (to_q4(price[i], scale[i], &q4)) continue;  // FromRaw throws: gRPC UNKNOWN
    bool good = false;
    {
      std::lock_guard<std::mutex> lk(write_mu);
      if (g.exec(db, "BEGIN", nullptr, nullptr, nullptr) == 0) {  // SQLite::Transaction
        const int64_t ts = now_ms();
        out << "[DB] [insert_new_order] ============================================================= "
            << std::endl
            << " order_id=" << oid << " client_id=" << client << " symbol=" << sym << " side=" << side[i]
            << " price_q4=" << q4 << " quantity=" << quantity[i] << " timse_stamp=" << ts << std::endl;
        sqlite3_stmt* st = nullptr;  // a fresh SQLite::Statement per call
        if (g.prepare_v2(db,
                         "INSERT INTO orders(  order_id, client_id, symbol, side, order_type,  price, quantity, "
                         "status, remaining_quantity,  created_ts, updated_ts) VALUES (?,?,?,?,?,?,?,?,?,?,?)",
                         -1, &st, nullptr) == 0) {
          g.bind_text(st, 1, oid.c_str(), -1, kTransient);
          g.bind_text(st, 2, client.c_str(), -1, kTransient);
          g.bind_text(st, 3, sym.c_str(), -1, kTransient);
          g.bind_int(st, 4, side[i]);
          g.bind_int(st, 5, 1);
          g.bind_int64(st, 6, q4);
          g.bind_int64(st, 7, quantity[i]);
          g.bind_int(st, 8, 0);
          g.bind_int64(st, 9, quantity[i]);
          g.bind_int64(st, 10, ts);
          g.bind_int64(st, 11, ts);
          good = g.step(st) == 101;  // SQLITE_DONE
          g.finalize(st);
        }
        good = good && g.exec(db, "COMMIT", nullptr, nullptr, nullptr) == 0;
        if (!good) g.exec(db, "ROLLBACK", nullptr, nullptr, nullptr);
      }
    }
    ok[i] = good;
    rows += good;
    if (good)
      out << "[SERVER] [SubmitOrder][ok] oid=" << oid << " inserted\n";
    const auto us =
        std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
    out << "[SERVER] [SubmitOrder] oid=" << oid << " done in " << us << "us\n";
  }
  out.flush();
  g.close(db);
  return rows;
}

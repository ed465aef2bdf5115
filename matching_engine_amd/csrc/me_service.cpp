// me_service.cpp — SubmitOrder re-hosted on the batched core (include/me_service.h).
//
// Per order (host, synchronous, the reference's exact contract):
//   validate (matching_engine_service.cpp:66-83) -> "OID-<n>" (:85, :29-32) -> normalize_to_q4
//   (:89-97, price.hpp:15-29) -> side CHECK (storage.cpp:32) -> response (:107-114)
// and the order joins the open time slice (SoA). me_service_flush matches the slice on the GPU
// engine and persists it in ONE SQLite transaction (the batched rewrite of storage.cpp:78-208):
// orders rows exactly as insert_new_order writes them (incl. order_type=1, storage.cpp:106),
// update_order_status-style updates for the matched outcome, and fills rows through the
// corrected add_fill statement (5 columns, 5 placeholders; the reference's has 6, storage.cpp:190).
//
// SQLite is loaded at run time (dlopen libsqlite3.so.0) so the library has no build-time
// dependency on a sqlite3 header.
#include <dlfcn.h>
#include <string.h>

#include <chrono>
#include <deque>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "me_engine.h"
#include "me_service.h"

namespace {

// ---- minimal sqlite3 C API (dlopen) -------------------------------------------------------
struct sqlite3;
struct sqlite3_stmt;
constexpr int SQLITE_OK = 0, SQLITE_ROW = 100, SQLITE_DONE = 101;
constexpr int SQLITE_OPEN_READWRITE = 0x2, SQLITE_OPEN_CREATE = 0x4, SQLITE_OPEN_FULLMUTEX = 0x10000;
using destructor_t = void (*)(void*);
const destructor_t SQLITE_TRANSIENT = reinterpret_cast<destructor_t>(-1);

struct Sql {
  void* h = nullptr;
  int (*open_v2)(const char*, sqlite3**, int, const char*) = nullptr;
  int (*close)(sqlite3*) = nullptr;
  int (*exec)(sqlite3*, const char*, void*, void*, char**) = nullptr;
  int (*prepare_v2)(sqlite3*, const char*, int, sqlite3_stmt**, const char**) = nullptr;
  int (*bind_int64)(sqlite3_stmt*, int, long long) = nullptr;
  int (*bind_text)(sqlite3_stmt*, int, const char*, int, destructor_t) = nullptr;
  int (*step)(sqlite3_stmt*) = nullptr;
  int (*reset)(sqlite3_stmt*) = nullptr;
  int (*finalize)(sqlite3_stmt*) = nullptr;
  long long (*column_int64)(sqlite3_stmt*, int) = nullptr;
  const char* (*errmsg)(sqlite3*) = nullptr;
  int (*busy_timeout)(sqlite3*, int) = nullptr;

  bool load(std::string& err) {
    if (h) return true;
    h = dlopen("libsqlite3.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("libsqlite3.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      err = "libsqlite3 not found";
      return false;
    }
#define SYM(f, n)                                  \
  f = reinterpret_cast<decltype(f)>(dlsym(h, n));  \
  if (!f) {                                        \
    err = std::string("sqlite symbol missing: ") + n; \
    return false;                                  \
  }
    SYM(open_v2, "sqlite3_open_v2");
    SYM(close, "sqlite3_close");
    SYM(exec, "sqlite3_exec");
    SYM(prepare_v2, "sqlite3_prepare_v2");
    SYM(bind_int64, "sqlite3_bind_int64");
    SYM(bind_text, "sqlite3_bind_text");
    SYM(step, "sqlite3_step");
    SYM(reset, "sqlite3_reset");
    SYM(finalize, "sqlite3_finalize");
    SYM(column_int64, "sqlite3_column_int64");
    SYM(errmsg, "sqlite3_errmsg");
    SYM(busy_timeout, "sqlite3_busy_timeout");
#undef SYM
    return true;
  }
};

Sql g_sql;
std::mutex g_sql_mu;

inline int64_t now_ms() {
  using namespace std::chrono;
  return duration_cast<milliseconds>(system_clock::now().time_since_epoch()).count();
}

// storage.cpp:26-69, verbatim schema semantics.
const char* kSchema =
    "CREATE TABLE IF NOT EXISTS orders ("
    "  order_id TEXT PRIMARY KEY, client_id TEXT NOT NULL, symbol TEXT NOT NULL,"
    "  side INTEGER NOT NULL CHECK (side IN (1,2)), order_type INTEGER NOT NULL, price INTEGER,"
    "  quantity INTEGER NOT NULL CHECK (quantity > 0), status INTEGER NOT NULL,"
    "  remaining_quantity INTEGER NOT NULL, created_ts INTEGER NOT NULL, updated_ts INTEGER NOT NULL);"
    "CREATE INDEX IF NOT EXISTS idx_orders_symbol_side ON orders(symbol, side);"
    "CREATE INDEX IF NOT EXISTS idx_orders_client ON orders(client_id);"
    "CREATE TABLE IF NOT EXISTS fills ("
    "  id INTEGER PRIMARY KEY AUTOINCREMENT, order_id TEXT NOT NULL, symbol TEXT NOT NULL,"
    "  fill_price INTEGER NOT NULL, fill_quantity INTEGER NOT NULL, event_ts INTEGER NOT NULL,"
    "  FOREIGN KEY(order_id) REFERENCES orders(order_id));"
    "CREATE INDEX IF NOT EXISTS idx_fills_order ON fills(order_id);";

struct Pending {
  std::string client;
  uint32_t symbol_id;
  std::string symbol;
  int32_t side;
  bool cancel;      // CancelOrder record (build extension): target = the order it removes
  uint64_t target;
};

// A resting order the OrderUpdate stream still reports on (owner + unfilled quantity).
struct Live {
  std::string client;
  std::string symbol;
  int32_t remaining;
};

constexpr size_t kMaxQueuedUpdates = size_t(1) << 24;  // oldest events are dropped beyond this

}  // namespace

struct me_service {
  me_engine* eng = nullptr;
  std::unordered_map<std::string, uint32_t> sym;
  std::vector<std::string> names;
  uint64_t next_id = 1;
  mutable std::mutex mu;
  // open time slice (SoA handed to the engine) + the host-only fields persistence needs
  std::vector<uint64_t> seq;
  std::vector<int64_t> px;
  std::vector<int32_t> qty;
  std::vector<uint32_t> sid;
  std::vector<uint8_t> kind;
  std::vector<Pending> meta;
  // StreamOrderUpdates: resting orders by seq, and the undrained events
  std::unordered_map<uint64_t, Live> live;
  std::deque<me_order_update> updates;
  uint64_t updates_dropped = 0;
  // persistence
  sqlite3* db = nullptr;
  sqlite3_stmt* st_ins = nullptr;
  sqlite3_stmt* st_upd = nullptr;
  sqlite3_stmt* st_fill = nullptr;
  sqlite3_stmt* st_maker = nullptr;
  std::string err;

  int fail(int code, const std::string& m) {
    err = m;
    return code;
  }
  bool sql_ok(int rc, const char* what) {
    if (rc == SQLITE_OK || rc == SQLITE_DONE || rc == SQLITE_ROW) return true;
    err = std::string(what) + ": " + (db ? g_sql.errmsg(db) : "no db");
    return false;
  }
};

static void close_db(me_service* s) {
  for (sqlite3_stmt* st : {s->st_ins, s->st_upd, s->st_fill, s->st_maker})
    if (st) g_sql.finalize(st);
  s->st_ins = s->st_upd = s->st_fill = s->st_maker = nullptr;
  if (s->db) g_sql.close(s->db);
  s->db = nullptr;
}

static bool open_db(me_service* s, const char* path) {
  {
    std::lock_guard<std::mutex> lk(g_sql_mu);
    if (!g_sql.load(s->err)) return false;
  }
  if (!s->sql_ok(g_sql.open_v2(path, &s->db, SQLITE_OPEN_READWRITE | SQLITE_OPEN_CREATE | SQLITE_OPEN_FULLMUTEX,
                               nullptr),
                 "open"))
    return false;
  g_sql.busy_timeout(s->db, 5000);  // storage.cpp:14
  // storage.cpp:17-24 pragmas, then the schema
  if (!s->sql_ok(g_sql.exec(s->db, "PRAGMA journal_mode=WAL;", nullptr, nullptr, nullptr), "pragma") ||
      !s->sql_ok(g_sql.exec(s->db, "PRAGMA synchronous=NORMAL;", nullptr, nullptr, nullptr), "pragma") ||
      !s->sql_ok(g_sql.exec(s->db, "PRAGMA foreign_keys=ON;", nullptr, nullptr, nullptr), "pragma") ||
      !s->sql_ok(g_sql.exec(s->db, kSchema, nullptr, nullptr, nullptr), "schema"))
    return false;
  // load_next_oid_seq (storage.cpp:254-267)
  sqlite3_stmt* q = nullptr;
  if (!s->sql_ok(g_sql.prepare_v2(s->db,
                                  "SELECT COALESCE(MAX(CAST(SUBSTR(order_id, 5) AS INTEGER)), 0) + 1 "
                                  "FROM orders WHERE order_id LIKE 'OID-%'",
                                  -1, &q, nullptr),
                 "prepare oid"))
    return false;
  if (g_sql.step(q) == SQLITE_ROW) s->next_id = (uint64_t)g_sql.column_int64(q, 0);
  g_sql.finalize(q);
  // cached statements (the reference prepares a fresh one per call, storage.cpp:95)
  const char* ins =
      "INSERT INTO orders(order_id, client_id, symbol, side, order_type, price, quantity, status,"
      " remaining_quantity, created_ts, updated_ts) VALUES (?,?,?,?,?,?,?,?,?,?,?)";
  const char* upd = "UPDATE orders SET status=?, remaining_quantity=?, updated_ts=? WHERE order_id=?";
  const char* fill = "INSERT INTO fills(order_id, symbol, fill_price, fill_quantity, event_ts) VALUES (?,?,?,?,?)";
  const char* maker =
      "UPDATE orders SET remaining_quantity=remaining_quantity-?, status=CASE WHEN remaining_quantity-?=0 "
      "THEN 2 ELSE 1 END, updated_ts=? WHERE order_id=?";
  return s->sql_ok(g_sql.prepare_v2(s->db, ins, -1, &s->st_ins, nullptr), "prepare insert") &&
         s->sql_ok(g_sql.prepare_v2(s->db, upd, -1, &s->st_upd, nullptr), "prepare update") &&
         s->sql_ok(g_sql.prepare_v2(s->db, fill, -1, &s->st_fill, nullptr), "prepare fill") &&
         s->sql_ok(g_sql.prepare_v2(s->db, maker, -1, &s->st_maker, nullptr), "prepare maker");
}

extern "C" me_service* me_service_create(me_engine* engine, const char* const* symbols, uint32_t num_symbols,
                                         const char* db_path) {
  me_service* s = new me_service();
  s->eng = engine;
  for (uint32_t i = 0; i < num_symbols; ++i) {
    s->names.emplace_back(symbols[i]);
    s->sym.emplace(s->names.back(), i);
  }
  if (db_path && !open_db(s, db_path)) {
    // keep the object so the caller can read the error; persistence is disabled
    close_db(s);
    s->err = "me_service_create: " + s->err;
  }
  return s;
}

extern "C" void me_service_destroy(me_service* s) {
  if (!s) return;
  close_db(s);
  delete s;
}

static void put(char* dst, size_t cap, const std::string& v) {
  size_t k = v.size() < cap - 1 ? v.size() : cap - 1;
  memcpy(dst, v.data(), k);
  dst[k] = 0;
}

extern "C" int me_service_submit_order(me_service* s, const me_order_request* r, me_order_response* resp) {
  memset(resp, 0, sizeof(*resp));
  const char* symbol = r->symbol ? r->symbol : "";
  // --- validation (:66-83): first failing check wins, no OID
  if (!symbol[0]) {
    put(resp->error_message, sizeof resp->error_message, "symbol is required");
    return 0;
  }
  if (r->quantity <= 0) {
    put(resp->error_message, sizeof resp->error_message, "quantity must be > 0");
    return 0;
  }
  if (r->order_type == ME_TYPE_LIMIT && r->price <= 0) {
    put(resp->error_message, sizeof resp->error_message, "price must be > 0 for LIMIT");
    return 0;
  }
  std::lock_guard<std::mutex> lk(s->mu);
  // --- OID (:85), consumed even if normalisation throws below
  const uint64_t id = s->next_id++;
  int64_t q4 = 0;
  const int nr = me_normalize_to_q4(r->price, r->scale, &q4);
  if (nr != 0) {  // exception escapes the handler -> gRPC UNKNOWN, no order_id in the response
    resp->grpc_status = 2;
    put(resp->error_message, sizeof resp->error_message,
        nr == 1 ? "scale out of range" : (nr == 2 ? "overflow" : "underflow"));
    return 0;
  }
  const std::string oid = "OID-" + std::to_string(id);
  put(resp->order_id, sizeof resp->order_id, oid);
  // --- the reference's DB CHECK side IN (1,2) (storage.cpp:32) -> "DB insert failed" (:109-111)
  if (r->side != ME_SIDE_BUY && r->side != ME_SIDE_SELL) {
    resp->success = 0;
    put(resp->error_message, sizeof resp->error_message, "DB insert failed");
    return 0;
  }
  resp->success = 1;
  // --- join the open time slice
  auto it = s->sym.find(symbol);
  const uint32_t sid = it == s->sym.end() ? (uint32_t)s->names.size() : it->second;  // unknown -> BAD_SYMBOL
  s->seq.push_back(id);
  s->px.push_back(q4);
  s->qty.push_back(r->quantity);
  s->sid.push_back(sid);
  s->kind.push_back(ME_KIND(r->side, r->order_type == ME_TYPE_LIMIT ? ME_TYPE_LIMIT : ME_TYPE_MARKET, ME_OP_NEW));
  s->meta.push_back(Pending{r->client_id ? r->client_id : "", sid, symbol, r->side, false, 0});
  return 0;
}

// "OID-<n>", n >= 1 with no trailing characters -> n; else 0.
static uint64_t parse_oid(const char* s) {
  if (!s || strncmp(s, "OID-", 4) != 0 || !s[4]) return 0;
  uint64_t v = 0;
  for (const char* p = s + 4; *p; ++p) {
    if (*p < '0' || *p > '9' || v > (UINT64_MAX - 9) / 10) return 0;
    v = v * 10 + (uint64_t)(*p - '0');
  }
  return v;
}

extern "C" int me_service_cancel_order(me_service* s, const me_cancel_request* r, me_order_response* resp) {
  memset(resp, 0, sizeof(*resp));
  const char* symbol = r->symbol ? r->symbol : "";
  if (!symbol[0]) {
    put(resp->error_message, sizeof resp->error_message, "symbol is required");
    return 0;
  }
  const uint64_t target = parse_oid(r->order_id);
  if (!target) {
    put(resp->error_message, sizeof resp->error_message, "order_id is invalid");
    return 0;
  }
  std::lock_guard<std::mutex> lk(s->mu);
  const uint64_t id = s->next_id++;  // the cancel's stream position (batch order == seq order)
  put(resp->order_id, sizeof resp->order_id, "OID-" + std::to_string(target));
  resp->success = 1;
  auto it = s->sym.find(symbol);
  const uint32_t sid = it == s->sym.end() ? (uint32_t)s->names.size() : it->second;
  s->seq.push_back(id);
  s->px.push_back((int64_t)target);
  s->qty.push_back(0);
  s->sid.push_back(sid);
  s->kind.push_back(ME_KIND(ME_SIDE_BUY, ME_TYPE_LIMIT, ME_OP_CANCEL));
  s->meta.push_back(Pending{r->client_id ? r->client_id : "", sid, symbol, 0, true, target});
  return 0;
}

extern "C" size_t me_service_pending(const me_service* s) {
  std::lock_guard<std::mutex> lk(s->mu);
  return s->seq.size();
}

extern "C" uint64_t me_service_next_oid(const me_service* s) {
  std::lock_guard<std::mutex> lk(s->mu);
  return s->next_id;
}

static void push_update(me_service* s, uint64_t oid, const std::string& client, const std::string& symbol,
                        int status, int64_t price, int32_t fq, int32_t remaining) {
  me_order_update u;
  memset(&u, 0, sizeof u);
  put(u.order_id, sizeof u.order_id, "OID-" + std::to_string(oid));
  put(u.client_id, sizeof u.client_id, client);
  put(u.symbol, sizeof u.symbol, symbol);
  u.status = status;
  u.scale = 4;
  u.fill_price = price;
  u.fill_quantity = fq;
  u.remaining_quantity = remaining;
  if (s->updates.size() >= kMaxQueuedUpdates) {
    s->updates.pop_front();
    s->updates_dropped++;
  }
  s->updates.push_back(u);
}

// OrderUpdate events of one matched slice (order documented in me_service.h), and the live-order
// table they are computed from (owner and unfilled quantity of every resting order).
static void emit_updates(me_service* s, size_t n, const me_order_result* res, const me_fill* tape) {
  for (size_t i = 0; i < n; ++i) {
    const Pending& m = s->meta[i];
    const me_order_result& r = res[i];
    if (m.cancel) {
      auto it = s->live.find(m.target);
      if (r.status == ME_ST_CANCELED && it != s->live.end()) {
        push_update(s, m.target, it->second.client, it->second.symbol, ME_ST_CANCELED, 0, 0, r.remaining_qty);
        s->live.erase(it);
      } else {
        push_update(s, m.target, m.client, m.symbol, r.status == ME_ST_CANCELED ? ME_ST_CANCELED : ME_ST_REJECTED,
                    0, 0, r.remaining_qty);
      }
      continue;
    }
    const uint64_t oid = s->seq[i];
    int32_t rem = s->qty[i];
    for (uint32_t f = 0; f < r.fill_count; ++f) {
      const me_fill& fl = tape[r.tape_offset + f];
      auto it = s->live.find(fl.maker_seq);
      if (it != s->live.end()) {
        Live& mk = it->second;
        mk.remaining -= fl.qty;
        push_update(s, fl.maker_seq, mk.client, mk.symbol,
                    mk.remaining > 0 ? ME_ST_PARTIALLY_FILLED : ME_ST_FILLED, fl.price_q4, fl.qty, mk.remaining);
        if (mk.remaining <= 0) s->live.erase(it);
      }
      rem -= fl.qty;
      push_update(s, oid, m.client, m.symbol, rem > 0 ? ME_ST_PARTIALLY_FILLED : ME_ST_FILLED, fl.price_q4,
                  fl.qty, rem);
    }
    const bool market = ((s->kind[i] >> 2) & 1u) != 0;
    if (r.status == ME_ST_REJECTED || r.status == ME_ST_CANCELED || (r.fill_count == 0 && r.status == ME_ST_NEW))
      push_update(s, oid, m.client, m.symbol, r.status, 0, 0, r.remaining_qty);
    if (!market && r.remaining_qty > 0 && (r.status == ME_ST_NEW || r.status == ME_ST_PARTIALLY_FILLED))
      s->live[oid] = Live{m.client, m.symbol, r.remaining_qty};
  }
}

extern "C" int me_service_updates(me_service* s, const char* client_id, me_order_update* out, size_t cap,
                                  size_t* n) {
  std::lock_guard<std::mutex> lk(s->mu);
  size_t k = 0;
  const bool all = !client_id || !client_id[0];
  if (all) {
    for (; k < cap && !s->updates.empty(); ++k) {
      if (out) out[k] = s->updates.front();
      s->updates.pop_front();
    }
  } else {  // one pass: this client's events out (up to cap), every other event kept in order
    std::deque<me_order_update> keep;
    for (auto& u : s->updates) {
      if (k < cap && strncmp(u.client_id, client_id, sizeof u.client_id) == 0) {
        if (out) out[k] = u;
        ++k;
      } else {
        keep.push_back(u);
      }
    }
    s->updates.swap(keep);
  }
  if (n) *n = k;
  return ME_OK;
}

static bool persist(me_service* s, size_t n, const me_order_result* res, const me_fill* tape, size_t nf) {
  if (!s->db) return true;
  const int64_t ts = now_ms();
  auto step = [&](sqlite3_stmt* st, const char* what) {
    const int rc = g_sql.step(st);
    g_sql.reset(st);
    return s->sql_ok(rc, what);
  };
  if (!s->sql_ok(g_sql.exec(s->db, "BEGIN", nullptr, nullptr, nullptr), "begin")) return false;
  bool ok = true;
  for (size_t i = 0; i < n && ok; ++i) {
    const Pending& m = s->meta[i];
    if (m.cancel) {  // no row of its own: the target's row becomes CANCELED
      if (res[i].status == ME_ST_CANCELED) {
        const std::string toid = "OID-" + std::to_string(m.target);
        sqlite3_stmt* up = s->st_upd;
        g_sql.bind_int64(up, 1, ME_ST_CANCELED);
        g_sql.bind_int64(up, 2, res[i].remaining_qty);  // the quantity the cancel removed
        g_sql.bind_int64(up, 3, ts);
        g_sql.bind_text(up, 4, toid.c_str(), -1, SQLITE_TRANSIENT);
        ok = step(up, "cancel order");
      }
      continue;
    }
    const std::string oid = "OID-" + std::to_string(s->seq[i]);
    sqlite3_stmt* st = s->st_ins;  // insert_new_order's row (storage.cpp:102-112)
    g_sql.bind_text(st, 1, oid.c_str(), -1, SQLITE_TRANSIENT);
    g_sql.bind_text(st, 2, m.client.c_str(), -1, SQLITE_TRANSIENT);
    g_sql.bind_text(st, 3, m.symbol.c_str(), -1, SQLITE_TRANSIENT);
    g_sql.bind_int64(st, 4, m.side);
    g_sql.bind_int64(st, 5, 1);  // order_type: the reference binds the constant 1 (storage.cpp:106)
    g_sql.bind_int64(st, 6, s->px[i]);
    g_sql.bind_int64(st, 7, s->qty[i]);
    g_sql.bind_int64(st, 8, 0);
    g_sql.bind_int64(st, 9, s->qty[i]);
    g_sql.bind_int64(st, 10, ts);
    g_sql.bind_int64(st, 11, ts);
    ok = step(st, "insert order");
    // makers hit by this taker (earlier rows, possibly in this same transaction)
    for (uint32_t f = 0; ok && f < res[i].fill_count; ++f) {
      const me_fill& fl = tape[res[i].tape_offset + f];
      const std::string moid = "OID-" + std::to_string(fl.maker_seq);
      sqlite3_stmt* mk = s->st_maker;
      g_sql.bind_int64(mk, 1, fl.qty);
      g_sql.bind_int64(mk, 2, fl.qty);
      g_sql.bind_int64(mk, 3, ts);
      g_sql.bind_text(mk, 4, moid.c_str(), -1, SQLITE_TRANSIENT);
      ok = step(mk, "update maker");
      for (int side = 0; ok && side < 2; ++side) {  // one FillRow per order of the trade
        sqlite3_stmt* fs = s->st_fill;
        g_sql.bind_text(fs, 1, side ? moid.c_str() : oid.c_str(), -1, SQLITE_TRANSIENT);
        g_sql.bind_text(fs, 2, m.symbol.c_str(), -1, SQLITE_TRANSIENT);
        g_sql.bind_int64(fs, 3, fl.price_q4);
        g_sql.bind_int64(fs, 4, fl.qty);
        g_sql.bind_int64(fs, 5, ts);
        ok = step(fs, "insert fill");
      }
    }
    if (ok && (res[i].status != ME_ST_NEW || res[i].remaining_qty != s->qty[i])) {
      sqlite3_stmt* up = s->st_upd;  // update_order_status (storage.cpp:160-181)
      g_sql.bind_int64(up, 1, res[i].status);
      g_sql.bind_int64(up, 2, res[i].remaining_qty);  // unfilled qty (0 once FILLED)
      g_sql.bind_int64(up, 3, ts);
      g_sql.bind_text(up, 4, oid.c_str(), -1, SQLITE_TRANSIENT);
      ok = step(up, "update order");
    }
  }
  (void)nf;
  if (!ok) {
    g_sql.exec(s->db, "ROLLBACK", nullptr, nullptr, nullptr);
    return false;
  }
  return s->sql_ok(g_sql.exec(s->db, "COMMIT", nullptr, nullptr, nullptr), "commit");
}

extern "C" int me_service_flush(me_service* s, me_fill* out_fills, size_t fills_cap, size_t* n_fills,
                                me_order_result* out_results, uint64_t* out_seq, size_t results_cap,
                                size_t* n_results) {
  std::lock_guard<std::mutex> lk(s->mu);
  const size_t n = s->seq.size();
  if (n_fills) *n_fills = 0;
  if (n_results) *n_results = n;
  if (n == 0) return ME_OK;
  if (!s->eng) return s->fail(ME_E_STATE, "me_service_flush: no engine (HIP device required)");
  std::vector<me_order_result> res(n);
  std::vector<me_fill> tape(me_fill_bound(s->eng, n));
  size_t nf = 0;
  me_order_soa b{s->seq.data(), s->px.data(), s->qty.data(), s->sid.data(), s->kind.data()};
  int rc = me_submit_batch(s->eng, &b, n, tape.data(), tape.size(), &nf, res.data());
  if (rc != ME_OK) {
    char e[512];
    me_last_error(s->eng, e, sizeof e);
    return s->fail(rc, std::string("engine: ") + e);
  }
  if (!persist(s, n, res.data(), tape.data(), nf)) return s->fail(ME_E_SQLITE, s->err);
  emit_updates(s, n, res.data(), tape.data());
  if (n_fills) *n_fills = nf;
  if (out_fills) {
    if (nf > fills_cap) return s->fail(ME_E_INVALID, "fills_cap smaller than the tape");
    memcpy(out_fills, tape.data(), nf * sizeof(me_fill));
  }
  if (out_results || out_seq) {
    if (n > results_cap) return s->fail(ME_E_INVALID, "results_cap smaller than the slice");
    if (out_results) memcpy(out_results, res.data(), n * sizeof(me_order_result));
    if (out_seq) memcpy(out_seq, s->seq.data(), n * sizeof(uint64_t));
  }
  s->seq.clear();
  s->px.clear();
  s->qty.clear();
  s->sid.clear();
  s->kind.clear();
  s->meta.clear();
  return ME_OK;
}

extern "C" int me_service_book(me_service* s, const char* symbol, me_level* bids, me_level* asks, size_t depth,
                               size_t* n_bids, size_t* n_asks) {
  if (n_bids) *n_bids = 0;
  if (n_asks) *n_asks = 0;
  auto it = s->sym.find(symbol ? symbol : "");
  if (it == s->sym.end()) return ME_OK;  // unknown symbol: empty book (the reference's stub is always empty)
  if (!s->eng) return s->fail(ME_E_STATE, "no engine");
  return me_book_snapshot(s->eng, it->second, bids, asks, depth, n_bids, n_asks);
}

extern "C" int me_service_market_data(me_service* s, const char* symbol, me_market_data* out) {
  memset(out, 0, sizeof(*out));
  out->scale = 4;
  auto it = s->sym.find(symbol ? symbol : "");
  if (it == s->sym.end()) return ME_OK;
  if (!s->eng) return s->fail(ME_E_STATE, "no engine");
  me_level b{}, a{};
  size_t nb = 0, na = 0;
  const int rc = me_book_snapshot(s->eng, it->second, &b, &a, 1, &nb, &na);
  if (rc != ME_OK) return rc;
  auto sat = [](int64_t v) { return (int32_t)(v > INT32_MAX ? INT32_MAX : v); };
  if (nb) {
    out->has_bid = 1;
    out->best_bid = b.price_q4;
    out->bid_size = sat(b.total_qty);
  }
  if (na) {
    out->has_ask = 1;
    out->best_ask = a.price_q4;
    out->ask_size = sat(a.total_qty);
  }
  return ME_OK;
}

extern "C" int me_service_last_error(const me_service* s, char* buf, size_t cap) {
  if (buf && cap) put(buf, cap, s->err);
  return (int)s->err.size();
}

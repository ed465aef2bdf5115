// me_service.cpp — SubmitOrder re-hosted on the batched core (include/me_service.h).
//
// Per order (host, synchronous, the reference's exact contract):
//   validate (matching_engine_service.cpp:66-83) -> "OID-<n>" (:85, :29-32) -> normalize_to_q4
//   (:89-97, price.hpp:15-29) -> side CHECK (storage.cpp:32) -> response (:107-114)
// and the order joins the open time slice (SoA). A slice closes when it reaches the slice size or
// (with the background flusher, me_service_start) when it is older than the interval; closed slices
// are matched on the engine and persisted, in stream order, OUTSIDE the submit lock — SubmitOrder
// only ever waits for another SubmitOrder. Persistence is ONE SQLite transaction per slice (the
// batched rewrite of storage.cpp:78-208): each order's row as insert_new_order writes it (incl.
// order_type=1, storage.cpp:106) carrying its matched status and remainder in the same INSERT,
// update_order_status-style updates for makers and cancel targets, and fills rows through the
// corrected add_fill statement (5 columns, 5 placeholders; the reference's has 6, storage.cpp:190).
//
// Two stages run concurrently: the flushing thread matches slice k+1 while the persister thread
// (which alone owns the DB) emits slice k's OrderUpdates and commits its transaction, so the engine
// (or the sharded matcher's gather) overlaps SQLite instead of waiting for it.
//
// Locks (always taken in this order, never the other way round):
//   flush_mu  one flusher at a time: slices are matched in stream order
//   eng_mu    every engine call (the engine is single-threaded): flush matching, book reads
//   mu        the open slice, the closed-slice queue, the symbol table, the OID counter
//   pq_mu     the matched-slice queue between the two stages
//   live_mu   resting orders' owners and remainders (cancel ownership, OrderUpdate bookkeeping)
//   upd_mu    the OrderUpdate queue
//   ref_mu    per-book reference counts (which books an idle symbol may hand over)
//   err_mu    the last error text
//
// The flusher keeps two slices in flight: slice k+1 is submitted to the backend (me_submit_host, or
// the matcher's submit) before slice k is collected, so the backend's work on k+1 overlaps the
// collect of k and its hand-off to the persister.
//
// SQLite is loaded at run time (dlopen libsqlite3.so.0) so the library has no build-time
// dependency on a sqlite3 header.
#include <dlfcn.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
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
  const unsigned char* (*column_text)(sqlite3_stmt*, int) = nullptr;
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
    SYM(column_text, "sqlite3_column_text");
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
inline int64_t mono_us() {
  using namespace std::chrono;
  return duration_cast<microseconds>(steady_clock::now().time_since_epoch()).count();
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
  std::string symbol;
  int32_t side;
  bool cancel;      // CancelOrder record (build extension): target = the order it removes
  uint64_t target;
};

// The symbol id of a cancel whose symbol holds no book: out of the backend's range, so the record is
// rejected (BAD_SYMBOL -> an OrderUpdate REJECTED) without taking a book for it.
constexpr uint32_t kNoBook = 0xFFFFFFFFu;

// One time slice: the SoA handed to the engine + the host-only fields persistence needs.
struct Slice {
  std::vector<uint64_t> seq;
  std::vector<int64_t> px;
  std::vector<int32_t> qty;
  std::vector<uint32_t> sid;
  std::vector<uint8_t> kind;
  std::vector<Pending> meta;
  int64_t opened_us = 0;
  bool recovery = false;  // resting orders replayed from the DB at create: their rows already exist
  size_t size() const { return seq.size(); }
  // The first k records become their own slice; this one keeps the rest.
  Slice take_prefix(size_t k) {
    Slice p;
    p.opened_us = opened_us;
    p.recovery = recovery;
    auto cut = [k](auto& src, auto& dst) {
      dst.assign(std::make_move_iterator(src.begin()), std::make_move_iterator(src.begin() + k));
      src.erase(src.begin(), src.begin() + k);
    };
    cut(seq, p.seq);
    cut(px, p.px);
    cut(qty, p.qty);
    cut(sid, p.sid);
    cut(kind, p.kind);
    cut(meta, p.meta);
    return p;
  }
};

// A matched slice on its way to the DB (outputs copied out of the engine's buffers). One whose
// transaction failed stays at the head of the queue, in order, until a later flush commits it.
struct Matched {
  Slice sl;
  std::vector<me_order_result> res;
  std::vector<me_fill> tape;
  int64_t ts;
};

// An order the OrderUpdate stream still reports on, and whose owner may cancel it: every accepted
// LIMIT order from SubmitOrder until it stops resting.
struct Live {
  std::string client;
  std::string symbol;
  int32_t remaining;
  uint32_t sid;  // its book (reference-counted: a book with live orders is never handed over)
};

constexpr size_t kMaxQueuedUpdates = size_t(1) << 24;  // oldest events are dropped beyond this
constexpr int kRows = 64;  // rows per multi-row INSERT (11 * 64 parameters < SQLite's 999 floor)
constexpr size_t kMaxMatchedAhead = 4;  // matched slices the flusher may run ahead of the persister

}  // namespace

struct me_service {
  me_engine* eng = nullptr;
  me_matcher m{};           // the matcher when the service fronts shards it does not own (m.match set)
  uint32_t sym_cap = UINT32_MAX;  // symbols the engine holds (local ids 0 .. sym_cap-1)
  size_t slice_max = 0;           // records per slice (the engine's max_batch)
  // --- mu
  std::mutex mu;
  std::unordered_map<std::string, uint32_t> sym;
  std::vector<std::string> names;
  uint64_t next_id = 1;
  Slice open;
  std::deque<Slice> closed;
  size_t closed_records = 0;
  size_t inflight_records = 0;  // taken off `closed`, not yet in pq (being matched)
  // --- flush_mu
  std::mutex flush_mu;
  // --- pq_mu: matched slices, oldest first, until committed (the persister thread owns the DB)
  std::mutex pq_mu;
  std::condition_variable pq_cv;
  std::deque<Matched> pq;
  size_t pq_emitted = 0;    // slices at the head of pq whose OrderUpdates are out
  size_t pq_records = 0;
  bool pq_stalled = false;  // the head's transaction failed: retried when the next flush starts
  bool pq_stop = false;
  std::string pq_err;
  std::thread persister;
  // --- eng_mu
  std::mutex eng_mu;
  // --- live_mu / upd_mu
  std::mutex live_mu;
  std::unordered_map<uint64_t, Live> live;
  std::mutex upd_mu;
  std::deque<me_order_update> updates;
  uint64_t updates_dropped = 0;
  // --- ref_mu: per book, live-table entries of its symbol + its records not yet emitted. A book at 0
  // holds no resting order and has nothing on its way: a new symbol may take it over.
  std::mutex ref_mu;
  std::vector<int64_t> sref;
  std::vector<uint32_t> idle;     // books whose count reached 0 (checked again when taken) ...
  std::vector<uint8_t> in_idle;   // ... each at most once: a book's count returns to 0 again and again
  uint64_t reclaimed = 0;
  uint64_t recovered = 0;
  // --- background flusher
  std::thread flusher;
  std::condition_variable cv;  // with mu
  bool stop = false;
  int64_t interval_us = 0;
  // --- persistence (the persister thread; create/destroy otherwise)
  sqlite3* db = nullptr;
  sqlite3_stmt* st_ins = nullptr;
  sqlite3_stmt* st_upd = nullptr;
  sqlite3_stmt* st_fill = nullptr;
  sqlite3_stmt* st_maker = nullptr;
  sqlite3_stmt* st_ins_k = nullptr;   // kRows-row INSERT INTO orders
  sqlite3_stmt* st_fill_k = nullptr;  // kRows-row INSERT INTO fills
  bool failed = false;  // the engine lost a slice it had accepted: nothing more can be matched
  // --- err_mu
  mutable std::mutex err_mu;
  std::string err;

  int fail(int code, const std::string& m) {
    std::lock_guard<std::mutex> lk(err_mu);
    err = m;
    return code;
  }
  std::string sql_err(const char* what) { return std::string(what) + ": " + (db ? g_sql.errmsg(db) : "no db"); }
};

static void close_db(me_service* s) {
  for (sqlite3_stmt* st : {s->st_ins, s->st_upd, s->st_fill, s->st_maker, s->st_ins_k, s->st_fill_k})
    if (st) g_sql.finalize(st);
  s->st_ins = s->st_upd = s->st_fill = s->st_maker = s->st_ins_k = s->st_fill_k = nullptr;
  if (s->db) g_sql.close(s->db);
  s->db = nullptr;
}

static void persister_main(me_service* s);
static bool has_backend(const me_service* s);

static bool sql_ok(int rc) { return rc == SQLITE_OK || rc == SQLITE_DONE || rc == SQLITE_ROW; }

static bool open_db(me_service* s, const char* path, std::string& err) {
  {
    std::lock_guard<std::mutex> lk(g_sql_mu);
    if (!g_sql.load(err)) return false;
  }
  auto chk = [&](int rc, const char* what) {
    if (sql_ok(rc)) return true;
    err = s->sql_err(what);
    return false;
  };
  if (!chk(g_sql.open_v2(path, &s->db, SQLITE_OPEN_READWRITE | SQLITE_OPEN_CREATE | SQLITE_OPEN_FULLMUTEX, nullptr),
           "open"))
    return false;
  g_sql.busy_timeout(s->db, 5000);  // storage.cpp:14
  // storage.cpp:17-24 pragmas, then the schema
  if (!chk(g_sql.exec(s->db, "PRAGMA journal_mode=WAL;", nullptr, nullptr, nullptr), "pragma") ||
      !chk(g_sql.exec(s->db, "PRAGMA synchronous=NORMAL;", nullptr, nullptr, nullptr), "pragma") ||
      !chk(g_sql.exec(s->db, "PRAGMA foreign_keys=ON;", nullptr, nullptr, nullptr), "pragma") ||
      !chk(g_sql.exec(s->db, kSchema, nullptr, nullptr, nullptr), "schema"))
    return false;
  // load_next_oid_seq (storage.cpp:254-267)
  sqlite3_stmt* q = nullptr;
  if (!chk(g_sql.prepare_v2(s->db,
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
  // multi-row forms: one statement step per kRows rows
  auto rows = [](const char* head, const char* tuple) {
    std::string q(head);
    for (int r = 0; r < kRows; ++r) q += (r ? "," : "") + std::string(tuple);
    return q;
  };
  const std::string ins_k = rows("INSERT INTO orders(order_id, client_id, symbol, side, order_type, price, quantity, "
                                 "status, remaining_quantity, created_ts, updated_ts) VALUES ",
                                 "(?,?,?,?,?,?,?,?,?,?,?)");
  const std::string fill_k =
      rows("INSERT INTO fills(order_id, symbol, fill_price, fill_quantity, event_ts) VALUES ", "(?,?,?,?,?)");
  return chk(g_sql.prepare_v2(s->db, ins, -1, &s->st_ins, nullptr), "prepare insert") &&
         chk(g_sql.prepare_v2(s->db, upd, -1, &s->st_upd, nullptr), "prepare update") &&
         chk(g_sql.prepare_v2(s->db, fill, -1, &s->st_fill, nullptr), "prepare fill") &&
         chk(g_sql.prepare_v2(s->db, maker, -1, &s->st_maker, nullptr), "prepare maker") &&
         chk(g_sql.prepare_v2(s->db, ins_k.c_str(), -1, &s->st_ins_k, nullptr), "prepare insert rows") &&
         chk(g_sql.prepare_v2(s->db, fill_k.c_str(), -1, &s->st_fill_k, nullptr), "prepare fill rows");
}

// ---- per-book reference counts ----------------------------------------------------------------
static void ref_add(me_service* s, uint32_t sid, int64_t d) {
  if (sid == kNoBook || d == 0) return;
  std::lock_guard<std::mutex> lr(s->ref_mu);
  if (sid >= s->sref.size()) return;
  int64_t& r = s->sref[sid];
  r += d;
  if (r == 0 && !s->in_idle[sid]) {
    s->in_idle[sid] = 1;
    s->idle.push_back(sid);
  }
}

// Symbol string -> local book id (mu held). The reference accepts any non-empty symbol
// (matching_engine_service.cpp:66-71) and keeps it forever; the backend holds sym_cap books. A new
// symbol takes the next unused book, else a book whose symbol has no live order and no record on its
// way (its count is 0 under ref_mu, and only this thread, holding mu, could raise it): the old symbol's
// book is empty, so handing it over changes no order's outcome; the window re-centres on the new
// symbol's first rest. False only when every book is in use.
static bool intern(me_service* s, const std::string& symbol, uint32_t& sid) {
  auto it = s->sym.find(symbol);
  if (it != s->sym.end()) {
    sid = it->second;
    return true;
  }
  std::lock_guard<std::mutex> lr(s->ref_mu);
  if (s->names.size() < s->sym_cap) {
    sid = (uint32_t)s->names.size();
    s->names.push_back(symbol);
    s->sym.emplace(symbol, sid);
    s->sref.push_back(0);
    s->in_idle.push_back(0);
    return true;
  }
  while (!s->idle.empty()) {
    const uint32_t c = s->idle.back();
    s->idle.pop_back();
    if (c < s->in_idle.size()) s->in_idle[c] = 0;
    if (c >= s->sref.size() || s->sref[c] != 0) continue;  // busy again since it went idle
    s->sym.erase(s->names[c]);
    s->names[c] = symbol;
    s->sym.emplace(symbol, c);
    s->reclaimed++;
    sid = c;
    return true;
  }
  return false;
}

static int flush_closed(me_service* s, bool take_open, size_t limit, struct FlushOut* out, bool wait);

// Restart recovery: the orders the DB shows resting (status NEW / PARTIALLY_FILLED, remaining > 0) as
// LIMIT records in OID order, with their remainders — replayed into the backend before any new
// order, so each keeps its place in its level's FIFO. Chunks of at most slice_max records spanning
// fewer than half the engine's seq ring, each matched alone (one launch group must span fewer seqs than
// the seq ring, and old resting orders can be sparse).
static bool load_resting(me_service* s, std::string& err) {
  sqlite3_stmt* q = nullptr;
  if (!sql_ok(g_sql.prepare_v2(s->db,
                               "SELECT order_id, client_id, symbol, side, price, remaining_quantity FROM orders "
                               "WHERE status IN (0, 1) AND remaining_quantity > 0 AND order_id LIKE 'OID-%' "
                               "ORDER BY CAST(SUBSTR(order_id, 5) AS INTEGER)",
                               -1, &q, nullptr))) {
    err = s->sql_err("prepare recovery");
    return false;
  }
  const size_t cap = s->slice_max ? s->slice_max : 65536;
  // a recovery chunk is matched alone (flush_closed collects it before the next submit), so one launch
  // group spans only its own OIDs: below half the engine's seq ring (a matcher: 2^20)
  uint64_t span = 1ull << 20;
  if (s->eng) {
    me_config c{};
    if (me_get_config(s->eng, &c) == ME_OK && c.seq_ring) span = std::max<uint64_t>(c.seq_ring / 2, 1);
  }
  bool ok = true;
  std::lock_guard<std::mutex> lk(s->mu);
  Slice cur;
  cur.recovery = true;
  auto close_chunk = [&] {
    if (!cur.size()) return;
    s->closed_records += cur.size();
    s->closed.push_back(std::move(cur));
    cur = Slice{};
    cur.recovery = true;
  };
  for (int rc; (rc = g_sql.step(q)) == SQLITE_ROW;) {
    const char* oid_s = (const char*)g_sql.column_text(q, 0);
    const char* cl = (const char*)g_sql.column_text(q, 1);
    const char* sy = (const char*)g_sql.column_text(q, 2);
    const uint64_t oid = oid_s ? strtoull(oid_s + 4, nullptr, 10) : 0;
    const int32_t side = (int32_t)g_sql.column_int64(q, 3);
    const int64_t px = g_sql.column_int64(q, 4);
    const long long rem = g_sql.column_int64(q, 5);
    if (!oid || (side != ME_SIDE_BUY && side != ME_SIDE_SELL) || rem <= 0 || rem > INT32_MAX) continue;
    const std::string symbol = sy ? sy : "";
    uint32_t sid = 0;
    if (!intern(s, symbol, sid)) {
      err = "restart recovery: the DB holds resting orders on more symbols than the backend has books";
      ok = false;
      break;
    }
    if (cur.size() >= cap || (cur.size() && oid - cur.seq.front() >= span)) close_chunk();
    cur.seq.push_back(oid);
    cur.px.push_back(px);
    cur.qty.push_back((int32_t)rem);
    cur.sid.push_back(sid);
    cur.kind.push_back(ME_KIND(side, ME_TYPE_LIMIT, ME_OP_NEW));
    cur.meta.push_back(Pending{cl ? cl : "", symbol, side, false, 0});
    {
      std::lock_guard<std::mutex> lv(s->live_mu);
      s->live[oid] = Live{cl ? cl : "", symbol, (int32_t)rem, sid};
    }
    ref_add(s, sid, 1);
    s->recovered++;
  }
  g_sql.finalize(q);
  close_chunk();
  return ok;
}

static me_service* create(me_engine* engine, const me_matcher* m, const char* const* symbols, uint32_t num_symbols,
                          const char* db_path) {
  me_service* s = new me_service();
  s->eng = engine;
  if (engine) {
    me_config c{};
    if (me_get_config(engine, &c) == ME_OK) {
      s->sym_cap = c.num_symbols;
      s->slice_max = c.max_batch;
    }
    // the flusher keeps two slices in flight, and me_collect holds the last collected slot back: three
    // warm pinned slots, so no slot is pinned inside the serving path
    me_host_reserve(engine, 3);
  } else if (m) {
    s->m = *m;
    s->sym_cap = m->num_symbols;
    s->slice_max = m->max_batch;
  }
  for (uint32_t i = 0; i < num_symbols; ++i) {
    s->names.emplace_back(symbols[i]);
    s->sym.emplace(s->names.back(), i);
    s->sref.push_back(0);
    s->in_idle.push_back(1);
  }
  for (uint32_t i = num_symbols; i-- > 0;) s->idle.push_back(i);  // nothing rests on them yet
  if (s->names.size() > s->sym_cap) s->fail(ME_E_INVALID, "me_service_create: more symbols than the engine holds");
  std::string err;
  if (db_path && !open_db(s, db_path, err)) {
    // keep the object so the caller can read the error; persistence is disabled
    close_db(s);
    s->fail(ME_E_SQLITE, "me_service_create: " + err);
  }
  s->persister = std::thread(persister_main, s);
  if (s->db && has_backend(s)) {  // rebuild the books from the DB before the first SubmitOrder
    if (!load_resting(s, err)) {
      s->failed = true;
      s->fail(ME_E_CAPACITY, "me_service_create: " + err);
    } else {
      std::lock_guard<std::mutex> lf(s->flush_mu);
      const int rc = flush_closed(s, false, SIZE_MAX, nullptr, true);
      if (rc != ME_OK) {
        s->failed = true;
        std::string e;
        {
          std::lock_guard<std::mutex> le(s->err_mu);
          e = s->err;
        }
        s->fail(rc, "me_service_create: restart recovery failed: " + e);
      }
    }
  }
  return s;
}

extern "C" me_service* me_service_create(me_engine* engine, const char* const* symbols, uint32_t num_symbols,
                                         const char* db_path) {
  return create(engine, nullptr, symbols, num_symbols, db_path);
}

extern "C" me_service* me_service_create_matcher(const me_matcher* m, const char* const* symbols,
                                                 uint32_t num_symbols, const char* db_path) {
  if (!m || !m->match || !m->book || !m->max_batch) return nullptr;
  return create(nullptr, m, symbols, num_symbols, db_path);
}

// The backend behind the service: its own engine, or the matcher of a sharded deployment.
static bool has_backend(const me_service* s) { return s->eng || s->m.match; }

static std::string backend_err(me_service* s) {
  if (!s->eng) return "matcher failed";
  char e[512];
  me_last_error(s->eng, e, sizeof e);
  return e;
}

// A slice handed to the backend and not collected yet.
struct Inflight {
  Slice sl;
  uint64_t ticket = 0;
  bool done = false;  // outputs already here (a matcher without submit / collect matches at once)
  std::vector<me_order_result> res;
  std::vector<me_fill> tape;
};

// Backends that take a slice now and hand its outputs back later: the engine (host slots and
// tickets) and matchers with submit / collect. The flusher keeps two slices in flight with them.
static bool backend_async(const me_service* s) { return s->eng || (s->m.submit && s->m.collect); }

// Hand one slice to the backend (eng_mu held). accepted = the backend took it (a later failure loses
// it); ME_E_CAPACITY with accepted false: refused, nothing of it was applied.
static int backend_submit(me_service* s, Inflight& f, bool& accepted) {
  Slice& sl = f.sl;
  const size_t n = sl.size();
  me_order_soa b{sl.seq.data(), sl.px.data(), sl.qty.data(), sl.sid.data(), sl.kind.data()};
  accepted = false;
  if (s->eng) {
    const int rc = me_submit_host(s->eng, &b, n, &f.ticket);
    accepted = rc == ME_OK;
    return rc;
  }
  if (s->m.submit && s->m.collect) {
    const int rc = s->m.submit(s->m.ctx, &b, n, &f.ticket);
    accepted = rc != ME_E_CAPACITY;
    return rc;
  }
  const me_fill* tape = nullptr;
  const me_order_result* res = nullptr;
  size_t nf = 0;
  const int rc = s->m.match(s->m.ctx, &b, n, &tape, &nf, &res);
  accepted = rc != ME_E_CAPACITY;
  if (rc != ME_OK) return rc;
  // the matcher's output views stay valid until its next call: copy them out under eng_mu
  f.res.assign(res, res + n);
  f.tape.assign(tape, tape + nf);
  f.done = true;
  return ME_OK;
}

// The outputs of an accepted slice (eng_mu held), copied out of the backend's buffers.
static int backend_collect(me_service* s, Inflight& f) {
  if (f.done) return ME_OK;
  const me_fill* tape = nullptr;
  const me_order_result* res = nullptr;
  size_t nf = 0, nr = 0;
  const int rc = s->eng ? me_collect(s->eng, f.ticket, &tape, &nf, &res, &nr)
                        : s->m.collect(s->m.ctx, f.ticket, &tape, &nf, &res);
  if (rc != ME_OK) return rc;
  f.res.assign(res, res + f.sl.size());
  f.tape.assign(tape, tape + nf);
  f.done = true;
  return ME_OK;
}

static int backend_book(me_service* s, uint32_t sid, uint32_t depth, me_book_entry* bids, size_t bids_cap,
                        size_t* n_bids, me_book_entry* asks, size_t asks_cap, size_t* n_asks, me_level* bl,
                        me_level* al, size_t* nbl, size_t* nal) {
  if (s->eng) {
    if (!depth) depth = 0xFFFFFFFFu;  // the whole book: every window level plus the far levels
    return me_book_orders(s->eng, sid, depth, bids, bids_cap, n_bids, asks, asks_cap, n_asks, bl, al, nbl, nal);
  }
  return s->m.book(s->m.ctx, sid, depth, bids, bids_cap, n_bids, asks, asks_cap, n_asks, bl, al, nbl, nal);
}

static void put(char* dst, size_t cap, const std::string& v) {
  size_t k = v.size() < cap - 1 ? v.size() : cap - 1;
  memcpy(dst, v.data(), k);
  dst[k] = 0;
}

// Close the open slice (mu held).
static void close_open(me_service* s) {
  if (!s->open.size()) return;
  s->closed_records += s->open.size();
  s->closed.push_back(std::move(s->open));
  s->open = Slice{};
  s->cv.notify_all();
}

// Append a record to the open slice (mu held); a full slice is closed and handed to the flusher.
static void append(me_service* s, uint64_t seq, int64_t px, int32_t qty, uint32_t sid, uint8_t kind, Pending&& m) {
  Slice& o = s->open;
  if (!o.size()) o.opened_us = mono_us();
  o.seq.push_back(seq);
  o.px.push_back(px);
  o.qty.push_back(qty);
  o.sid.push_back(sid);
  o.kind.push_back(kind);
  o.meta.push_back(std::move(m));
  if (s->slice_max && o.size() >= s->slice_max) close_open(s);
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
  const std::string sym(symbol);
  std::string client = r->client_id ? r->client_id : "";
  std::lock_guard<std::mutex> lk(s->mu);
  uint32_t sid = 0;
  if (!intern(s, sym, sid)) {  // the engine's books are all taken: RESOURCE_EXHAUSTED, no OID
    resp->grpc_status = 8;
    put(resp->error_message, sizeof resp->error_message, "symbol capacity exhausted");
    return 0;
  }
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
  const bool limit = r->order_type == ME_TYPE_LIMIT;
  if (limit) {  // its owner, for CancelOrder and the OrderUpdate stream
    std::lock_guard<std::mutex> lv(s->live_mu);
    s->live[id] = Live{client, sym, r->quantity, sid};
  }
  ref_add(s, sid, 1);  // a LIMIT's live entry, or a MARKET record on its way
  append(s, id, q4, r->quantity, sid, ME_KIND(r->side, limit ? ME_TYPE_LIMIT : ME_TYPE_MARKET, ME_OP_NEW),
         Pending{std::move(client), sym, r->side, false, 0});
  return 0;
}

extern "C" int me_service_submit_orders(me_service* s, const me_order_request* reqs, size_t n,
                                        me_order_response* resps) {
  for (size_t i = 0; i < n; ++i) me_service_submit_order(s, reqs + i, resps + i);
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
  const std::string client = r->client_id ? r->client_id : "";
  const std::string sym(symbol);
  std::lock_guard<std::mutex> lk(s->mu);
  {  // only the order's owner may cancel it
    std::lock_guard<std::mutex> lv(s->live_mu);
    auto it = s->live.find(target);
    if (it != s->live.end() && it->second.client != client) {
      put(resp->error_message, sizeof resp->error_message, "order belongs to another client");
      return 0;
    }
  }
  // A symbol with no book has no resting order: the record goes out with an id the backend rejects
  // (BAD_SYMBOL -> OrderUpdate REJECTED) and takes no book.
  auto it = s->sym.find(sym);
  const uint32_t sid = it != s->sym.end() ? it->second : kNoBook;
  // Stream position: the last OID allocated, consuming none (a cancel record may repeat the previous
  // record's seq, me_engine.h), so accepted orders keep the reference's gap-free OIDs (:29-32, :85).
  const uint64_t id = s->next_id - 1;
  put(resp->order_id, sizeof resp->order_id, "OID-" + std::to_string(target));
  resp->success = 1;
  ref_add(s, sid, 1);
  append(s, id, (int64_t)target, 0, sid, ME_KIND(ME_SIDE_BUY, ME_TYPE_LIMIT, ME_OP_CANCEL),
         Pending{client, sym, 0, true, target});
  return 0;
}

extern "C" size_t me_service_pending(const me_service* s) {
  me_service* m = const_cast<me_service*>(s);
  std::lock_guard<std::mutex> lk(m->mu);
  return m->open.size() + m->closed_records + m->inflight_records;
}

extern "C" uint64_t me_service_next_oid(const me_service* s) {
  me_service* m = const_cast<me_service*>(s);
  std::lock_guard<std::mutex> lk(m->mu);
  return m->next_id;
}

extern "C" size_t me_service_unpersisted(const me_service* s) {
  me_service* m = const_cast<me_service*>(s);
  std::lock_guard<std::mutex> lk(m->pq_mu);
  return m->pq_records;
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
  if (s->updates.size() >= kMaxQueuedUpdates) {  // nobody drains the stream: drop the oldest, loudly
    s->updates.pop_front();
    if (s->updates_dropped++ == 0)
      s->fail(ME_OK, "OrderUpdate queue full (2^24 undrained events): dropping the oldest; drain with me_service_updates");
  }
  s->updates.push_back(u);
}

// OrderUpdate events of one matched slice (order documented in me_service.h), and the live-order
// table they are computed from. Locks are taken per block of records so SubmitOrder / CancelOrder
// (which touch the live table) never wait for a whole slice.
// Book reference counts move here too: every record's own count is released once its events are
// out, and a live entry's when it stops resting (filled, cancelled, or never rested).
// A recovery slice (orders replayed from the DB at create) emits only what is new: fills and
// outcomes other than "still resting" (its NEW events went out in the earlier run).
static void emit_updates(me_service* s, const Slice& sl, const me_order_result* res, const me_fill* tape) {
  constexpr size_t kBlock = 512;
  for (size_t i0 = 0; i0 < sl.size(); i0 += kBlock) {
    std::lock_guard<std::mutex> lv(s->live_mu);
    std::lock_guard<std::mutex> lu(s->upd_mu);
    auto live_erase = [&](std::unordered_map<uint64_t, Live>::iterator it) {
      ref_add(s, it->second.sid, -1);
      s->live.erase(it);
    };
    for (size_t i = i0; i < sl.size() && i < i0 + kBlock; ++i) {
      const Pending& m = sl.meta[i];
      const me_order_result& r = res[i];
      if (m.cancel) {
        auto it = s->live.find(m.target);
        if (r.status == ME_ST_CANCELED && it != s->live.end()) {
          push_update(s, m.target, it->second.client, it->second.symbol, ME_ST_CANCELED, 0, 0, r.remaining_qty);
          live_erase(it);
        } else {
          push_update(s, m.target, m.client, m.symbol, r.status == ME_ST_CANCELED ? ME_ST_CANCELED : ME_ST_REJECTED,
                      0, 0, r.remaining_qty);
        }
        ref_add(s, sl.sid[i], -1);  // the cancel record itself
        continue;
      }
      const uint64_t oid = sl.seq[i];
      int32_t rem = sl.qty[i];
      for (uint32_t f = 0; f < r.fill_count; ++f) {
        const me_fill& fl = tape[r.tape_offset + f];
        auto it = s->live.find(fl.maker_seq);
        if (it != s->live.end()) {
          Live& mk = it->second;
          mk.remaining -= fl.qty;
          push_update(s, fl.maker_seq, mk.client, mk.symbol,
                      mk.remaining > 0 ? ME_ST_PARTIALLY_FILLED : ME_ST_FILLED, fl.price_q4, fl.qty, mk.remaining);
          if (mk.remaining <= 0) live_erase(it);
        }
        rem -= fl.qty;
        push_update(s, oid, m.client, m.symbol, rem > 0 ? ME_ST_PARTIALLY_FILLED : ME_ST_FILLED, fl.price_q4,
                    fl.qty, rem);
      }
      const bool market = ((sl.kind[i] >> 2) & 1u) != 0;
      if (r.status == ME_ST_REJECTED || r.status == ME_ST_CANCELED ||
          (r.fill_count == 0 && r.status == ME_ST_NEW && !sl.recovery))
        push_update(s, oid, m.client, m.symbol, r.status, 0, 0, r.remaining_qty);
      if (market) {
        ref_add(s, sl.sid[i], -1);  // the MARKET record (it never rests)
        continue;
      }
      // a LIMIT's count is its live entry, created at submit: it stays while the order rests
      if (r.remaining_qty > 0 && (r.status == ME_ST_NEW || r.status == ME_ST_PARTIALLY_FILLED)) {
        auto it = s->live.find(oid);
        if (it != s->live.end()) {
          it->second.remaining = r.remaining_qty;
        } else {
          s->live[oid] = Live{m.client, m.symbol, r.remaining_qty, sl.sid[i]};
          ref_add(s, sl.sid[i], 1);
        }
      } else {
        auto it = s->live.find(oid);
        if (it != s->live.end()) live_erase(it);
      }
    }
  }
}

extern "C" int me_service_updates(me_service* s, const char* client_id, me_order_update* out, size_t cap,
                                  size_t* n) {
  std::lock_guard<std::mutex> lk(s->upd_mu);
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

// One transaction for one matched slice (the persister thread). The rows end exactly as the reference's
// per-order statements would leave them — insert_new_order's row (storage.cpp:102-112, incl.
// order_type=1, storage.cpp:106), then update_order_status-style changes (storage.cpp:160-181) as
// later fills and cancels hit the order — but the slice's own orders are brought to their final
// state in memory first, so each is ONE multi-row INSERT entry and only orders of earlier slices
// take UPDATEs. Orders rows go in before fills rows (the fills' foreign key), fills rows in tape
// order (taker's row, then maker's), through the corrected add_fill statement (5 columns, 5
// placeholders; the reference's has 6, storage.cpp:190).
static bool persist(me_service* s, const Slice& sl, const me_order_result* res, const me_fill* tape, int64_t ts,
                    std::string& err) {
  if (!s->db) return true;
  const size_t n = sl.size();
  if (sl.recovery) {  // replayed resting orders: their rows exist; a consistent DB produces no change
    bool change = false;
    for (size_t i = 0; i < n && !change; ++i) change = res[i].fill_count || res[i].status != ME_ST_NEW;
    if (!change) return true;
  }
  // ---- final state of this slice's rows; changes to earlier slices' rows
  std::vector<int32_t> fst(n), frem(n);
  std::unordered_map<uint64_t, long long> ext_fill;       // earlier order -> quantity filled now
  std::vector<std::pair<uint64_t, int32_t>> ext_cancel;   // earlier order -> quantity the cancel removed
  auto find = [&](uint64_t q) -> long {  // row of order q in this slice (seqs ascend), or -1
    auto it = std::lower_bound(sl.seq.begin(), sl.seq.end(), q);
    if (it == sl.seq.end() || *it != q) return -1;
    const long j = (long)(it - sl.seq.begin());
    return sl.meta[j].cancel ? -1 : j;
  };
  size_t nfill = 0;
  for (size_t i = 0; i < n; ++i) {
    const Pending& m = sl.meta[i];
    if (m.cancel) {
      if (res[i].status != ME_ST_CANCELED) continue;
      const long j = find(m.target);
      if (j >= 0) {
        fst[j] = ME_ST_CANCELED;
        frem[j] = res[i].remaining_qty;
      } else {
        ext_cancel.emplace_back(m.target, res[i].remaining_qty);
      }
      continue;
    }
    fst[i] = res[i].status;
    frem[i] = res[i].remaining_qty;  // unfilled qty (0 once FILLED)
    for (uint32_t f = 0; f < res[i].fill_count; ++f) {
      const me_fill& fl = tape[res[i].tape_offset + f];
      const long j = find(fl.maker_seq);
      if (j >= 0) {
        frem[j] -= fl.qty;
        fst[j] = frem[j] == 0 ? ME_ST_FILLED : ME_ST_PARTIALLY_FILLED;
      } else {
        ext_fill[fl.maker_seq] += fl.qty;
      }
    }
    nfill += res[i].fill_count;
  }
  std::vector<std::string> oid(n);
  for (size_t i = 0; i < n; ++i)
    if (!sl.meta[i].cancel) oid[i] = "OID-" + std::to_string(sl.seq[i]);
  bool ok = true;
  auto step = [&](sqlite3_stmt* st, const char* what) {
    const int rc = g_sql.step(st);
    g_sql.reset(st);
    if (!sql_ok(rc)) {
      err = s->sql_err(what);
      ok = false;
    }
    return ok;
  };
  if (!sql_ok(g_sql.exec(s->db, "BEGIN", nullptr, nullptr, nullptr))) {
    err = s->sql_err("begin");
    return false;
  }
  // ---- orders rows, kRows per statement (a recovery slice's rows exist: they take UPDATEs)
  if (sl.recovery) {
    for (size_t i = 0; ok && i < n; ++i) {
      if (fst[i] == ME_ST_NEW && frem[i] == sl.qty[i]) continue;
      g_sql.bind_int64(s->st_upd, 1, fst[i]);
      g_sql.bind_int64(s->st_upd, 2, frem[i]);
      g_sql.bind_int64(s->st_upd, 3, ts);
      g_sql.bind_text(s->st_upd, 4, oid[i].c_str(), -1, SQLITE_TRANSIENT);
      step(s->st_upd, "update recovered order");
    }
  } else {
    std::vector<size_t> rows;
    rows.reserve(n);
    for (size_t i = 0; i < n; ++i)
      if (!sl.meta[i].cancel) rows.push_back(i);
    auto bind_row = [&](sqlite3_stmt* st, int b, size_t i) {
      const Pending& m = sl.meta[i];
      g_sql.bind_text(st, b + 1, oid[i].c_str(), -1, nullptr);
      g_sql.bind_text(st, b + 2, m.client.c_str(), -1, nullptr);
      g_sql.bind_text(st, b + 3, m.symbol.c_str(), -1, nullptr);
      g_sql.bind_int64(st, b + 4, m.side);
      g_sql.bind_int64(st, b + 5, 1);  // order_type: the reference binds the constant 1 (storage.cpp:106)
      g_sql.bind_int64(st, b + 6, sl.px[i]);
      g_sql.bind_int64(st, b + 7, sl.qty[i]);
      g_sql.bind_int64(st, b + 8, fst[i]);
      g_sql.bind_int64(st, b + 9, frem[i]);
      g_sql.bind_int64(st, b + 10, ts);
      g_sql.bind_int64(st, b + 11, ts);
    };
    size_t k = 0;
    for (; ok && k + kRows <= rows.size(); k += kRows) {
      for (int r = 0; r < kRows; ++r) bind_row(s->st_ins_k, 11 * r, rows[k + r]);
      step(s->st_ins_k, "insert orders");
    }
    for (; ok && k < rows.size(); ++k) {
      bind_row(s->st_ins, 0, rows[k]);
      step(s->st_ins, "insert order");
    }
  }
  // ---- earlier slices' rows: fills first (an order is filled before it can be canceled), then cancels
  for (auto it = ext_fill.begin(); ok && it != ext_fill.end(); ++it) {
    const std::string moid = "OID-" + std::to_string(it->first);
    g_sql.bind_int64(s->st_maker, 1, it->second);
    g_sql.bind_int64(s->st_maker, 2, it->second);
    g_sql.bind_int64(s->st_maker, 3, ts);
    g_sql.bind_text(s->st_maker, 4, moid.c_str(), -1, SQLITE_TRANSIENT);
    step(s->st_maker, "update maker");
  }
  for (size_t k = 0; ok && k < ext_cancel.size(); ++k) {
    const std::string toid = "OID-" + std::to_string(ext_cancel[k].first);
    g_sql.bind_int64(s->st_upd, 1, ME_ST_CANCELED);
    g_sql.bind_int64(s->st_upd, 2, ext_cancel[k].second);  // the quantity the cancel removed
    g_sql.bind_int64(s->st_upd, 3, ts);
    g_sql.bind_text(s->st_upd, 4, toid.c_str(), -1, SQLITE_TRANSIENT);
    step(s->st_upd, "cancel order");
  }
  // ---- fills rows: one FillRow per order of each trade, kRows per statement
  if (ok && nfill) {
    std::vector<std::string> moid(nfill);
    std::vector<std::pair<size_t, size_t>> fr;  // (taker row, fill index in the slice's fills)
    fr.reserve(nfill);
    size_t q = 0;
    for (size_t i = 0; i < n; ++i) {
      if (sl.meta[i].cancel) continue;
      for (uint32_t f = 0; f < res[i].fill_count; ++f, ++q) {
        moid[q] = "OID-" + std::to_string(tape[res[i].tape_offset + f].maker_seq);
        fr.emplace_back(i, res[i].tape_offset + f);
      }
    }
    auto bind_fill = [&](sqlite3_stmt* st, int b, size_t r) {  // row r: fill r / 2, taker (even) or maker
      const size_t i = fr[r / 2].first;
      const me_fill& fl = tape[fr[r / 2].second];
      const char* who = (r & 1) ? moid[r / 2].c_str() : oid[i].c_str();
      g_sql.bind_text(st, b + 1, who, -1, nullptr);
      g_sql.bind_text(st, b + 2, sl.meta[i].symbol.c_str(), -1, nullptr);
      g_sql.bind_int64(st, b + 3, fl.price_q4);
      g_sql.bind_int64(st, b + 4, fl.qty);
      g_sql.bind_int64(st, b + 5, ts);
    };
    const size_t nrows = 2 * nfill;
    size_t r = 0;
    for (; ok && r + kRows <= nrows; r += kRows) {
      for (int k = 0; k < kRows; ++k) bind_fill(s->st_fill_k, 5 * k, r + k);
      step(s->st_fill_k, "insert fills");
    }
    for (; ok && r < nrows; ++r) {
      bind_fill(s->st_fill, 0, r);
      step(s->st_fill, "insert fill");
    }
  }
  if (!ok) {
    g_sql.exec(s->db, "ROLLBACK", nullptr, nullptr, nullptr);
    return false;
  }
  if (!sql_ok(g_sql.exec(s->db, "COMMIT", nullptr, nullptr, nullptr))) {
    err = s->sql_err("commit");
    g_sql.exec(s->db, "ROLLBACK", nullptr, nullptr, nullptr);
    return false;
  }
  return true;
}

// The persister: emits each matched slice's OrderUpdates, then commits its transaction, oldest
// first. A failed transaction stalls the queue (later slices still get their updates) until the
// next flush clears pq_stalled; on stop it drains what it can and exits.
static void persister_main(me_service* s) {
  std::unique_lock<std::mutex> lk(s->pq_mu);
  for (;;) {
    s->pq_cv.wait(lk, [&] {
      return s->pq_stop || s->pq_emitted < s->pq.size() || (!s->pq_stalled && !s->pq.empty());
    });
    if (s->pq_emitted < s->pq.size()) {
      const Matched* m = &s->pq[s->pq_emitted];  // deque elements stay put under push_back
      lk.unlock();
      emit_updates(s, m->sl, m->res.data(), m->tape.data());
      lk.lock();
      ++s->pq_emitted;
      s->pq_cv.notify_all();
      continue;
    }
    if (!s->pq_stalled && !s->pq.empty()) {
      const Matched* m = &s->pq.front();
      lk.unlock();
      std::string err;
      const bool ok = persist(s, m->sl, m->res.data(), m->tape.data(), m->ts, err);
      lk.lock();
      if (ok) {
        s->pq_records -= m->sl.size();
        s->pq.pop_front();
        --s->pq_emitted;
      } else {
        s->pq_stalled = true;
        s->pq_err = err;
      }
      s->pq_cv.notify_all();
      continue;
    }
    if (s->pq_stop) break;
  }
}

// Where a flush's caller wants the matched outputs (any pointer may be NULL). The capacities are
// checked against the pending records before anything is matched; a slice whose outputs still would
// not fit (a matcher exceeding its own fill bound) is not copied: `short_buf`, ME_E_INVALID at the end.
struct FlushOut {
  me_fill* fills = nullptr;
  size_t fills_cap = 0;
  size_t nf = 0;
  me_order_result* res = nullptr;
  uint64_t* seq = nullptr;
  size_t res_cap = 0;
  size_t nr = 0;
  bool short_buf = false;
};

// A matched slice: its outputs to the caller, the slice to the persister (stream order).
static void deliver(me_service* s, Slice&& sl, std::vector<me_order_result>&& res, std::vector<me_fill>&& tape,
                    FlushOut* out) {
  const size_t n = sl.size(), nf = tape.size();
  if (out && !out->short_buf) {
    if ((out->fills && out->nf + nf > out->fills_cap) || ((out->res || out->seq) && out->nr + n > out->res_cap)) {
      out->short_buf = true;
    } else {
      if (out->fills) memcpy(out->fills + out->nf, tape.data(), nf * sizeof(me_fill));
      if (out->res)
        for (size_t i = 0; i < n; ++i) {
          out->res[out->nr + i] = res[i];
          out->res[out->nr + i].tape_offset += (uint32_t)out->nf;
        }
      if (out->seq) memcpy(out->seq + out->nr, sl.seq.data(), n * sizeof(uint64_t));
      out->nf += nf;
      out->nr += n;
    }
  }
  Matched mt;
  mt.ts = now_ms();
  mt.sl = std::move(sl);
  mt.res = std::move(res);
  mt.tape = std::move(tape);
  {
    std::lock_guard<std::mutex> lq(s->pq_mu);
    s->pq.push_back(std::move(mt));
    s->pq_records += n;
    s->pq_cv.notify_all();
  }
  std::lock_guard<std::mutex> lk(s->mu);  // after the push: pending + unpersisted never dips to 0 early
  s->inflight_records -= n;
}

// The backend refused a slice (its books near max_resting; nothing of it applied). Rather than
// retrying the same slice forever — nothing could free capacity, since every later record (cancels
// included) is queued behind it — it is split and its halves go back to the head of the queue; a
// single LIMIT that still does not fit is answered in-band (REJECTED, ME_RJ_CAPACITY). `taken` counts
// the records of this flush's budget handed out so far.
static int on_refused(me_service* s, Slice&& sl, FlushOut* out, size_t& taken) {
  const size_t n = sl.size();
  if (sl.recovery) {  // the DB's resting orders do not fit the books: nothing sensible to do
    s->failed = true;
    {
      std::lock_guard<std::mutex> lk(s->mu);
      s->inflight_records -= n;
    }
    return s->fail(ME_E_CAPACITY, "the backend's max_resting is below the resting orders the DB holds: " +
                                      backend_err(s));
  }
  if (n == 1 && (sl.kind[0] & 0x0Cu) == 0u) {  // one LIMIT and no room to rest it
    me_order_result r{};
    r.remaining_qty = sl.qty[0];
    r.status = ME_ST_REJECTED;
    r.reason = ME_RJ_CAPACITY;
    deliver(s, std::move(sl), std::vector<me_order_result>{r}, std::vector<me_fill>{}, out);
    return ME_OK;
  }
  std::lock_guard<std::mutex> lk(s->mu);
  s->inflight_records -= n;
  s->closed_records += n;
  taken -= n;
  if (n == 1) {  // a record that cannot rest, refused by a matcher: kept queued for the next flush
    s->closed.push_front(std::move(sl));
    return s->fail(ME_E_CAPACITY, "the matcher refused a record that cannot rest; it stays queued");
  }
  Slice head = sl.take_prefix(n / 2);
  s->closed.push_front(std::move(sl));
  s->closed.push_front(std::move(head));
  return ME_OK;
}

// Flush the closed slices (and the open one when take_open), oldest first, two in flight: slice k+1 is
// submitted before slice k is collected. `rec_limit` bounds the records taken (those present when the
// caller checked its output capacity). With `wait`, returns once the persister has emitted every
// matched slice and committed them (or stalled on a failed transaction: ME_E_SQLITE, the slices kept
// in order for the next flush).
static int flush_closed(me_service* s, bool take_open, size_t rec_limit, FlushOut* out, bool wait) {
  if (s->failed) return s->fail(ME_E_STATE, "service failed: the engine lost an accepted slice");
  if (!has_backend(s)) {
    std::lock_guard<std::mutex> lk(s->mu);
    if (s->open.size() || !s->closed.empty())
      return s->fail(ME_E_STATE, "me_service_flush: no engine (HIP device required)");
  }
  {  // every flush retries the kept slices first
    std::lock_guard<std::mutex> lq(s->pq_mu);
    if (s->pq_stalled) {
      s->pq_stalled = false;
      s->pq_cv.notify_all();
    }
  }
  if (take_open) {
    std::lock_guard<std::mutex> lk(s->mu);
    close_open(s);
  }
  std::deque<Inflight> fl;  // submitted, not collected (at most two)
  auto lost = [&](int r, const std::string& what) {
    s->failed = true;
    size_t n = 0;
    for (auto& f : fl) n += f.sl.size();
    std::lock_guard<std::mutex> lk(s->mu);
    s->inflight_records -= n;
    return s->fail(r, what + backend_err(s));
  };
  auto finish_oldest = [&]() -> int {
    int r;
    {
      std::lock_guard<std::mutex> le(s->eng_mu);
      r = backend_collect(s, fl.front());
    }
    if (r != ME_OK) return lost(r, "engine lost an accepted slice: ");
    Inflight& f = fl.front();
    deliver(s, std::move(f.sl), std::move(f.res), std::move(f.tape), out);
    fl.pop_front();
    return ME_OK;
  };
  size_t taken = 0;
  while (taken < rec_limit) {
    Inflight f;
    {
      std::lock_guard<std::mutex> lk(s->mu);
      if (s->closed.empty()) break;
      f.sl = std::move(s->closed.front());
      s->closed.pop_front();
      s->closed_records -= f.sl.size();
      s->inflight_records += f.sl.size();
    }
    taken += f.sl.size();
    {  // bounded run-ahead: at most kMaxMatchedAhead slices wait for the DB (unless it is stalled)
      std::unique_lock<std::mutex> lq(s->pq_mu);
      s->pq_cv.wait(lq, [&] { return s->pq_stalled || s->pq.size() < kMaxMatchedAhead; });
    }
    bool accepted = false;
    int r;
    {
      std::lock_guard<std::mutex> le(s->eng_mu);
      r = backend_submit(s, f, accepted);
    }
    if (r != ME_OK && !accepted) {  // refused: the slices before it go first, then it is split
      while (!fl.empty())
        if ((r = finish_oldest()) != ME_OK) return r;
      if ((r = on_refused(s, std::move(f.sl), out, taken)) != ME_OK) return r;
      continue;
    }
    if (r != ME_OK) {  // accepted and lost: the books may hold the slice, the service cannot go on
      fl.push_back(std::move(f));
      return lost(r, "engine lost an accepted slice: ");
    }
    fl.push_back(std::move(f));
    if (fl.size() > 1 || !backend_async(s))
      if ((r = finish_oldest()) != ME_OK) return r;
    if (!fl.empty() && fl.back().sl.recovery)  // a recovery chunk is matched alone (load_resting)
      while (!fl.empty())
        if ((r = finish_oldest()) != ME_OK) return r;
  }
  while (!fl.empty()) {
    const int r = finish_oldest();
    if (r != ME_OK) return r;
  }
  if (out && out->short_buf)
    return s->fail(ME_E_INVALID, "output buffers too small for the matched slices (they were matched and persisted; "
                                 "outputs truncated to the slices that fit)");
  if (!wait) return ME_OK;
  std::unique_lock<std::mutex> lq(s->pq_mu);
  s->pq_cv.wait(lq, [&] { return s->pq_emitted == s->pq.size() && (s->pq.empty() || s->pq_stalled); });
  if (s->pq_stalled)
    return s->fail(ME_E_SQLITE, "persistence deferred (" + s->pq_err +
                                    "); the matched slices are kept and retried at the next flush");
  return ME_OK;
}

extern "C" int me_service_flush(me_service* s, me_fill* out_fills, size_t fills_cap, size_t* n_fills,
                                me_order_result* out_results, uint64_t* out_seq, size_t results_cap,
                                size_t* n_results) {
  if (n_fills) *n_fills = 0;
  if (n_results) *n_results = 0;
  std::lock_guard<std::mutex> lf(s->flush_mu);
  size_t total = 0;
  {  // the open slice closes in the same critical section that counts it: SubmitOrders after this point go
     // into a new open slice (the next flush's), so `total` is exactly what this flush matches
    std::lock_guard<std::mutex> lk(s->mu);
    close_open(s);
    total = s->closed_records;  // inflight is 0 here (flush_mu held)
  }
  // the caller's buffers are checked before anything is matched
  if ((out_results || out_seq) && total > results_cap)
    return s->fail(ME_E_INVALID, "results_cap smaller than the pending records");
  const uint64_t bound = s->eng ? me_fill_bound(s->eng, total) : s->m.max_resting + 2 * (uint64_t)total;
  if (out_fills && has_backend(s) && fills_cap < bound)
    return s->fail(ME_E_INVALID, "fills_cap smaller than me_fill_bound(pending records)");
  FlushOut out;
  out.fills = out_fills;
  out.fills_cap = fills_cap;
  out.res = out_results;
  out.seq = out_seq;
  out.res_cap = results_cap;
  const int rc = flush_closed(s, false, total, &out, true);
  if (n_fills) *n_fills = out.nf;
  if (n_results) *n_results = out.nr;
  return rc;
}

// The background flusher: closes the open slice once it is interval old (or the submit path closed
// it at the slice size) and flushes the closed ones.
static void flusher_main(me_service* s) {
  std::unique_lock<std::mutex> lk(s->mu);
  // after a failed flush (e.g. a matcher kept refusing a record): retry after 1 ms, doubling to 100 ms
  int64_t backoff_us = 0, retry_at = 0;
  while (!s->stop) {
    const int64_t now = mono_us();
    const bool due = s->open.size() && now - s->open.opened_us >= s->interval_us;
    if (due) close_open(s);
    const bool blocked = backoff_us && now < retry_at;
    if (s->closed.empty() || blocked) {
      int64_t wait = s->open.size() ? s->open.opened_us + s->interval_us - now : s->interval_us;
      if (blocked) wait = std::min(wait, retry_at - now);
      s->cv.wait_for(lk, std::chrono::microseconds(wait > 0 ? wait : 1));
      continue;
    }
    lk.unlock();
    int rc;
    {
      std::lock_guard<std::mutex> lf(s->flush_mu);
      rc = flush_closed(s, false, SIZE_MAX, nullptr, false);  // errors land in me_service_last_error
    }
    lk.lock();
    if (s->failed) break;
    if (rc == ME_OK) {
      backoff_us = 0;
    } else {
      backoff_us = std::min<int64_t>(std::max<int64_t>(2 * backoff_us, 1000), 100000);
      retry_at = mono_us() + backoff_us;
    }
  }
}

extern "C" int me_service_start(me_service* s, uint32_t interval_us, uint32_t slice_orders) {
  if (!s || !has_backend(s)) return ME_E_STATE;
  std::lock_guard<std::mutex> lk(s->mu);
  if (s->flusher.joinable()) return s->fail(ME_E_STATE, "flusher already running");
  uint32_t mb = s->m.max_batch;
  if (s->eng) {
    me_config c{};
    me_get_config(s->eng, &c);
    mb = c.max_batch;
  }
  s->slice_max = slice_orders && slice_orders < mb ? slice_orders : mb;
  s->interval_us = interval_us ? interval_us : 1000;
  s->stop = false;
  s->flusher = std::thread(flusher_main, s);
  return ME_OK;
}

extern "C" int me_service_stop(me_service* s) {
  if (!s) return ME_E_INVALID;
  {
    std::lock_guard<std::mutex> lk(s->mu);
    s->stop = true;
    s->cv.notify_all();
  }
  if (s->flusher.joinable()) s->flusher.join();
  // what the flusher matched is out (updates emitted, committed or stalled) when stop returns
  std::unique_lock<std::mutex> lq(s->pq_mu);
  s->pq_cv.wait(lq, [&] { return s->pq_emitted == s->pq.size() && (s->pq.empty() || s->pq_stalled); });
  return ME_OK;
}

extern "C" void me_service_destroy(me_service* s) {
  if (!s) return;
  me_service_stop(s);
  {  // the persister commits what it can (a stalled head is given one more try), then exits
    std::lock_guard<std::mutex> lq(s->pq_mu);
    s->pq_stalled = false;
    s->pq_stop = true;
    s->pq_cv.notify_all();
  }
  if (s->persister.joinable()) s->persister.join();
  close_db(s);
  delete s;
}

extern "C" int me_service_book(me_service* s, const char* symbol, me_level* bids, me_level* asks, size_t depth,
                               size_t* n_bids, size_t* n_asks) {
  if (n_bids) *n_bids = 0;
  if (n_asks) *n_asks = 0;
  if (depth == 0) return ME_OK;  // no levels asked for (the backend would read 0 as "the whole book")
  uint32_t sid = 0;
  {
    std::lock_guard<std::mutex> lk(s->mu);
    auto it = s->sym.find(symbol ? symbol : "");
    if (it == s->sym.end()) return ME_OK;  // unknown symbol: empty book (the reference's stub is always empty)
    sid = it->second;
  }
  if (!has_backend(s)) return s->fail(ME_E_STATE, "no engine");
  std::lock_guard<std::mutex> le(s->eng_mu);
  const int rc = backend_book(s, sid, (uint32_t)std::min<size_t>(depth, 0xFFFFFFFFu), nullptr, 0, nullptr, nullptr,
                              0, nullptr, bids, asks, n_bids, n_asks);
  if (rc != ME_OK) return s->fail(rc, "engine: " + backend_err(s));
  return ME_OK;
}

extern "C" int me_service_order_book(me_service* s, const char* symbol, uint32_t depth, me_book_order* bids,
                                     size_t bids_cap, size_t* n_bids, me_book_order* asks, size_t asks_cap,
                                     size_t* n_asks) {
  if (n_bids) *n_bids = 0;
  if (n_asks) *n_asks = 0;
  uint32_t sid = 0;
  {
    std::lock_guard<std::mutex> lk(s->mu);
    auto it = s->sym.find(symbol ? symbol : "");
    if (it == s->sym.end()) return ME_OK;
    sid = it->second;
  }
  if (!has_backend(s)) return s->fail(ME_E_STATE, "no engine");
  std::vector<me_book_entry> side[2];
  size_t n[2] = {0, 0};
  {
    std::lock_guard<std::mutex> le(s->eng_mu);
    side[0].resize(std::max<size_t>(bids_cap, 1));
    side[1].resize(std::max<size_t>(asks_cap, 1));
    const int rc = backend_book(s, sid, depth, bids ? side[0].data() : nullptr, bids ? side[0].size() : 0, &n[0],
                                asks ? side[1].data() : nullptr, asks ? side[1].size() : 0, &n[1], nullptr, nullptr,
                                nullptr, nullptr);
    if (rc != ME_OK) return s->fail(rc, "engine: " + backend_err(s));
  }
  me_book_order* out[2] = {bids, asks};
  const size_t caps[2] = {bids_cap, asks_cap};
  std::lock_guard<std::mutex> lv(s->live_mu);
  for (int k = 0; k < 2; ++k) {
    if (!out[k]) continue;
    for (size_t i = 0; i < n[k] && i < caps[k]; ++i) {
      const me_book_entry& e = side[k][i];
      me_book_order& o = out[k][i];
      memset(&o, 0, sizeof o);
      put(o.order_id, sizeof o.order_id, "OID-" + std::to_string(e.seq));
      auto it = s->live.find(e.seq);
      if (it != s->live.end()) put(o.client_id, sizeof o.client_id, it->second.client);
      o.price = e.price_q4;
      o.scale = 4;
      o.quantity = e.qty;
      o.side = e.side;
    }
  }
  if (n_bids) *n_bids = n[0];
  if (n_asks) *n_asks = n[1];
  return ME_OK;
}

extern "C" int me_service_market_data(me_service* s, const char* symbol, me_market_data* out) {
  memset(out, 0, sizeof(*out));
  out->scale = 4;
  me_level b{}, a{};
  size_t nb = 0, na = 0;
  const int rc = me_service_book(s, symbol, &b, &a, 1, &nb, &na);
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

extern "C" uint64_t me_service_updates_dropped(const me_service* s) {
  me_service* m = const_cast<me_service*>(s);
  std::lock_guard<std::mutex> lk(m->upd_mu);
  return m->updates_dropped;
}

extern "C" int me_service_stats(const me_service* s, uint64_t* reclaimed_books, uint64_t* recovered_orders) {
  if (!s) return ME_E_INVALID;
  me_service* m = const_cast<me_service*>(s);
  std::lock_guard<std::mutex> lk(m->mu);
  {
    std::lock_guard<std::mutex> lr(m->ref_mu);
    if (reclaimed_books) *reclaimed_books = m->reclaimed;
  }
  if (recovered_orders) *recovered_orders = m->recovered;
  return ME_OK;
}

extern "C" int me_service_last_error(const me_service* s, char* buf, size_t cap) {
  std::lock_guard<std::mutex> lk(s->err_mu);
  if (buf && cap) put(buf, cap, s->err);
  return (int)s->err.size();
}

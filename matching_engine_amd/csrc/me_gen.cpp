// me_gen.cpp — deterministic synthetic order streams for the five benchmark configurations
// (SURVEY.md §8(d)). Replaces the reference's one-shot CLI client (src/client/client.cpp) as the
// load generator; emits already-normalized records (symbol ids interned, Q4 prices), i.e. what
// the submit-order path hands to the batcher.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "me_engine.h"

namespace {

inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

struct Rng {  // xoshiro256**
  uint64_t s[4];
  explicit Rng(uint64_t seed) {
    uint64_t x = seed;
    for (int i = 0; i < 4; ++i) s[i] = x = splitmix64(x);
  }
  static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9;
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return r;
  }
  // uniform in [0, n) (Lemire, unbiased)
  uint64_t below(uint64_t n) {
    unsigned __int128 m = (unsigned __int128)next() * n;
    uint64_t l = (uint64_t)m;
    if (l < n) {
      uint64_t t = (0 - n) % n;
      while (l < t) {
        m = (unsigned __int128)next() * n;
        l = (uint64_t)m;
      }
    }
    return (uint64_t)(m >> 64);
  }
  double unit() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
};

}  // namespace

struct me_gen {
  me_gen_params p;
  Rng rng;
  uint64_t next_seq = 1;
  std::vector<int64_t> mid;
  std::vector<int8_t> dir;          // drift direction of each symbol
  std::vector<uint32_t> since;      // records of each symbol since its mid last moved
  std::vector<double> zipf_cdf;
  std::vector<std::vector<uint64_t>> cancel_pool;  // per symbol: LIMIT seqs not yet targeted
  explicit me_gen(const me_gen_params& pp) : p(pp), rng(pp.seed) {}
};

extern "C" me_gen* me_gen_create(const me_gen_params* p) {
  if (!p || p->num_symbols == 0 || p->levels < 64 || p->max_qty <= 0 || p->spread_ticks < 0 ||
      (int64_t)p->spread_ticks * 2 + 1 > (int64_t)p->levels || p->market_pct + p->cancel_pct > 100 ||
      p->far_pct > 100 || p->drift_step < 0 || (p->drift_step > 0 && p->drift_every == 0))
    return nullptr;
  me_gen* g = new me_gen(*p);
  g->next_seq = p->seq_start ? p->seq_start : 1;
  g->mid.resize(p->num_symbols);
  g->dir.resize(p->num_symbols);
  g->since.assign(p->num_symbols, 0);
  for (uint32_t s = 0; s < p->num_symbols; ++s) {
    // per-symbol mid: 100.0000 +- 10.0000 in Q4, fixed by (seed, symbol)
    const uint64_t h = splitmix64(p->seed * 0x100000001B3ull ^ (uint64_t)s);
    g->mid[s] = 1000000 + (int64_t)(h % 200001) - 100000;
    g->dir[s] = (h >> 40) & 1 ? 1 : -1;
  }
  if (p->zipf_s > 0) {
    g->zipf_cdf.resize(p->num_symbols);
    double acc = 0;
    for (uint32_t s = 0; s < p->num_symbols; ++s) {
      acc += 1.0 / pow((double)(s + 1), p->zipf_s);
      g->zipf_cdf[s] = acc;
    }
    for (auto& v : g->zipf_cdf) v /= acc;
  }
  if (p->cancel_pct) g->cancel_pool.resize(p->num_symbols);
  return g;
}

extern "C" void me_gen_destroy(me_gen* g) { delete g; }

extern "C" int me_gen_base_prices(const me_gen* g, int64_t* out) {
  if (!g || !out) return ME_E_INVALID;
  for (uint32_t s = 0; s < g->p.num_symbols; ++s) out[s] = g->mid[s] - (int64_t)(g->p.levels / 2);
  return ME_OK;
}

static inline uint32_t pick_symbol(me_gen* g) {
  if (g->zipf_cdf.empty()) return (uint32_t)g->rng.below(g->p.num_symbols);
  const double u = g->rng.unit();
  auto it = std::lower_bound(g->zipf_cdf.begin(), g->zipf_cdf.end(), u);
  if (it == g->zipf_cdf.end()) --it;
  return (uint32_t)(it - g->zipf_cdf.begin());
}

extern "C" int me_gen_next(me_gen* g, size_t n, uint64_t* seq, int64_t* price_q4, int32_t* qty, uint32_t* symbol,
                           uint8_t* kind) {
  if (!g) return ME_E_INVALID;
  const me_gen_params& p = g->p;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t sq = g->next_seq++;
    const uint32_t s = pick_symbol(g);
    if (p.drift_step > 0 && ++g->since[s] >= p.drift_every) {  // the symbol's market moves
      g->since[s] = 0;
      g->mid[s] += g->dir[s] * (int64_t)p.drift_step;
    }
    const uint32_t r = (uint32_t)g->rng.below(100);
    uint8_t k;
    int64_t px = 0;
    int32_t q = 0;
    bool cancelled = false;
    if (r < p.cancel_pct) {
      auto& pool = g->cancel_pool[s];
      if (!pool.empty()) {
        const size_t j = (size_t)g->rng.below(pool.size());
        px = (int64_t)pool[j];
        pool[j] = pool.back();
        pool.pop_back();
        k = ME_KIND(ME_SIDE_BUY, ME_TYPE_LIMIT, ME_OP_CANCEL);
        cancelled = true;
      }
    }
    if (!cancelled) {
      const uint32_t side = (g->rng.next() >> 63) ? ME_SIDE_SELL : ME_SIDE_BUY;
      const bool market = r >= p.cancel_pct && r < p.cancel_pct + p.market_pct;
      if (market) {
        q = (int32_t)(1 + g->rng.below((uint64_t)p.max_qty));
        if (p.market_qty_mult > 0) q = (int32_t)(1 + g->rng.below((uint64_t)p.market_qty_mult)) * p.max_qty;
        k = ME_KIND(side, ME_TYPE_MARKET, ME_OP_NEW);
      } else {
        int64_t off = (int64_t)g->rng.below(2 * (uint64_t)p.spread_ticks + 1) - p.spread_ticks;
        if (p.far_pct && g->rng.below(100) < p.far_pct) {  // far away from the window, either side
          off = (int64_t)p.levels + (int64_t)g->rng.below(63 * (uint64_t)p.levels + 1);
          if (g->rng.next() >> 63) off = -off;
        }
        px = g->mid[s] + off;
        if (px < 1) px = 1;
        q = (int32_t)(1 + g->rng.below((uint64_t)p.max_qty));
        k = ME_KIND(side, ME_TYPE_LIMIT, ME_OP_NEW);
        if (p.cancel_pct) g->cancel_pool[s].push_back(sq);
      }
    }
    if (seq) seq[i] = sq;
    if (price_q4) price_q4[i] = px;
    if (qty) qty[i] = q;
    if (symbol) symbol[i] = s;
    if (kind) kind[i] = k;
  }
  return ME_OK;
}

extern "C" int me_gen_seed_book(me_gen* g, uint32_t symbol, uint32_t per_side, uint64_t* seq, int64_t* price_q4,
                                int32_t* qty, uint8_t* kind) {
  if (!g || symbol >= g->p.num_symbols) return ME_E_INVALID;
  if ((uint64_t)per_side * 2 + 1 > g->p.levels) return ME_E_INVALID;
  const int64_t m = g->mid[symbol];
  for (uint32_t j = 0; j < 2 * per_side; ++j) {
    const bool bid = j < per_side;
    const uint32_t d = (bid ? j : j - per_side) + 1;
    const uint64_t sq = g->next_seq++;
    if (seq) seq[j] = sq;
    if (price_q4) price_q4[j] = bid ? m - d : m + d;
    if (qty) qty[j] = (int32_t)(1 + g->rng.below((uint64_t)g->p.max_qty));
    if (kind) kind[j] = ME_KIND(bid ? ME_SIDE_BUY : ME_SIDE_SELL, ME_TYPE_LIMIT, ME_OP_NEW);
    if (g->p.cancel_pct) g->cancel_pool[symbol].push_back(sq);
  }
  return ME_OK;
}

extern "C" uint32_t me_shard_of(uint32_t symbol, uint32_t shards) {
  if (shards <= 1) return 0;
  return (uint32_t)(splitmix64((uint64_t)symbol) % shards);
}

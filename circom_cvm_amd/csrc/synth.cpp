// synth.cpp -- seeded synthetic --O0 systems (the benchmark workloads of BASELINE.md).
//
// circomlib / circom-ecdsa sources are not available offline, so the workloads are structural
// stand-ins emitted directly as the rs_input the Rust side would marshal (DESIGN.md "Workloads"):
//
//  kind 0  mixed  (metric circuit): per "template instance" a linear
//          cluster of log-normal size (median 40), the wiring equalities of its interface
//          signals, constant assignments used as selectors, and quadratic rows over the
//          instance's signals; row mix ~30% eq / 5% const-eq / 35% linear / 30% quadratic.
//          A few quadratic rows have a constant selector in A, so they turn linear after the
//          constant frame and feed rounds >= 2.
//  kind 1  linear (config 2): every row x_new = a*x_prev + b*x_other + c; 50% of rows in
//          clusters of 8, 40% in clusters of 2048, 10% in one big cluster; 1/64 of the rows
//          touch a public input.
//  kind 2  chain  (config 4 stand-in): long dependent chains of limb-carry rows with quadratic
//          rows whose A collapses after substitution, i.e. deep rounds >= 2.
//
// Coefficients: 60% from {1, p-1, 2^k}, 40% uniform in [1, p) (splitmix64 stream).
#include <algorithm>
#include <array>
#include <cmath>

#include "host_common.hpp"

namespace rs {

struct SplitMix {
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
  }
  double uni() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  uint64_t below(uint64_t n) { return n ? next() % n : 0; }
};

struct Gen {
  SplitMix rng;
  uint64_t p[4];
  int bits;
  uint32_t next_sig = 1;
  Block ce, eq, lin, na, nb, nc;
  uint64_t n_ce = 0, n_eq = 0, n_lin = 0, n_q = 0;

  void rand_elem(uint64_t v[4]) {
    for (;;) {
      for (int i = 0; i < 4; ++i) v[i] = rng.next();
      int top = (bits - 1) / 64;
      for (int i = top + 1; i < 4; ++i) v[i] = 0;
      int tb = bits - 64 * top;
      if (tb < 64) v[top] &= (1ULL << tb) - 1;
      bool less = false;
      for (int i = 3; i >= 0; --i)
        if (v[i] != p[i]) { less = v[i] < p[i]; break; }
      if (less && (v[0] | v[1] | v[2] | v[3])) return;
    }
  }
  void coef(uint64_t v[4]) {
    double r = rng.uni();
    v[0] = v[1] = v[2] = v[3] = 0;
    if (r < 0.25) { v[0] = 1; return; }
    if (r < 0.45) { neg_one(v); return; }
    if (r < 0.60) {
      int k = 1 + (int)rng.below(bits - 2);
      v[k / 64] = 1ULL << (k % 64);
      return;
    }
    rand_elem(v);
  }
  void neg_one(uint64_t v[4]) {
    memcpy(v, p, 32);
    v[0] -= 1;
  }
  void neg(const uint64_t a[4], uint64_t r[4]) {
    unsigned __int128 borrow = 0;
    for (int i = 0; i < 4; ++i) {
      unsigned __int128 d = (unsigned __int128)p[i] - a[i] - (uint64_t)borrow;
      r[i] = (uint64_t)d;
      borrow = (d >> 64) & 1;
    }
  }
  uint32_t fresh() { return next_sig++; }

  // A generated linear row lands in the block map_tree would classify it into
  // (dag/src/map_to_constraint_list.rs:28-33, algebra.rs:1346-1372).
  void linear_row(std::vector<std::pair<uint32_t, std::array<uint64_t, 4>>> &terms) {
    std::sort(terms.begin(), terms.end(),
              [](const std::pair<uint32_t, std::array<uint64_t, 4>> &x,
                 const std::pair<uint32_t, std::array<uint64_t, 4>> &y) { return x.first < y.first; });
    terms.erase(std::unique(terms.begin(), terms.end(),
                            [](const std::pair<uint32_t, std::array<uint64_t, 4>> &x,
                               const std::pair<uint32_t, std::array<uint64_t, 4>> &y) {
                              return x.first == y.first;
                            }),
                terms.end());
    bool has0 = !terms.empty() && terms[0].first == 0;
    size_t n = terms.size();
    if ((has0 && n == 2) || (!has0 && n == 1)) { row(ce, terms); n_ce++; return; }
    if (!has0 && n == 2) {
      uint64_t m[4];
      neg(terms[1].second.data(), m);
      if (memcmp(m, terms[0].second.data(), 32) == 0) { row(eq, terms); n_eq++; return; }
    }
    row(lin, terms);
    n_lin++;
  }

  // one row of a block from (signal, coef) pairs; merges duplicate signals by skipping them
  template <class V>
  void row(Block &b, V &terms) {
    std::sort(terms.begin(), terms.end(),
              [](const std::pair<uint32_t, std::array<uint64_t, 4>> &x,
                 const std::pair<uint32_t, std::array<uint64_t, 4>> &y) { return x.first < y.first; });
    uint32_t last = 0xffffffffu;
    for (auto &t : terms) {
      if (t.first == last) continue;
      last = t.first;
      b.push(t.first, t.second.data());
    }
    b.end_row();
  }
};

typedef std::vector<std::pair<uint32_t, std::array<uint64_t, 4>>> Terms;

static void add(Gen &g, Terms &t, uint32_t s) {
  std::array<uint64_t, 4> c;
  g.coef(c.data());
  t.push_back({s, c});
}
static void add_v(Terms &t, uint32_t s, const uint64_t v[4]) {
  std::array<uint64_t, 4> c;
  memcpy(c.data(), v, 32);
  t.push_back({s, c});
}

static void gen_mixed(Gen &g, uint64_t R, uint32_t n_pub, uint32_t n_priv, uint32_t first_priv) {
  const double f_eq = 0.30, f_ce = 0.05, f_lin = 0.35, f_q = 0.30;
  const uint64_t lin_target = (uint64_t)(f_lin * R);
  std::vector<uint32_t> nodes, pool, sels;
  uint32_t pub_used = 0;
  Terms t;
  uint64_t one[4] = {1, 0, 0, 0};
  double carry_eq = 0, carry_ce = 0, carry_q = 0;
  while (g.n_lin < lin_target) {
    // log-normal cluster size, median 40
    double z = std::sqrt(-2.0 * std::log(std::max(g.rng.uni(), 1e-300))) *
               std::cos(6.283185307179586 * g.rng.uni());
    uint64_t n = (uint64_t)std::llround(40.0 * std::exp(1.1 * z));
    n = std::max<uint64_t>(1, std::min<uint64_t>(n, 200000));
    n = std::min<uint64_t>(n, lin_target - g.n_lin);
    nodes.clear();
    pool.clear();
    uint32_t root = g.fresh();
    nodes.push_back(root);
    pool.push_back(root);
    std::vector<uint32_t> frees;
    // wiring equalities, constant selectors (emitted before the instance body, like <== wiring)
    double want_eq = carry_eq + n * (f_eq / f_lin);
    double want_ce = carry_ce + n * (f_ce / f_lin);
    double want_q = carry_q + n * (f_q / f_lin);
    uint64_t k_eq = (uint64_t)want_eq, k_ce = (uint64_t)want_ce, k_q = (uint64_t)want_q;
    carry_eq = want_eq - k_eq;
    carry_ce = want_ce - k_ce;
    carry_q = want_q - k_q;
    // linear body: a random recursive tree over fresh signals
    for (uint64_t i = 0; i < n; ++i) {
      t.clear();
      uint32_t x = g.fresh();
      add(g, t, x);
      add(g, t, nodes[g.rng.below(nodes.size())]);
      double r = g.rng.uni();
      if (r < 0.45) {
        uint32_t w;
        if (!frees.empty() && g.rng.uni() < 0.3) w = frees[g.rng.below(frees.size())];
        else { w = g.fresh(); frees.push_back(w); pool.push_back(w); }
        add(g, t, w);
      } else if (r < 0.55 && nodes.size() > 2) {
        add(g, t, nodes[g.rng.below(nodes.size())]);
      }
      if (g.rng.uni() < 0.3) add(g, t, 0);
      if (pub_used < n_pub && g.rng.uni() < 1.0 / 4096) add(g, t, 1 + 1 + (pub_used++));
      g.linear_row(t);
      nodes.push_back(x);
      if (g.rng.uni() < 0.5) pool.push_back(x);
    }
    // equalities: aliases of instance signals (larger fresh id := smaller), some alias chains
    std::vector<uint32_t> aliases;
    for (uint64_t i = 0; i < k_eq; ++i) {
      t.clear();
      uint32_t y = g.fresh();
      uint32_t s = (!aliases.empty() && g.rng.uni() < 0.15) ? aliases[g.rng.below(aliases.size())]
                                                           : pool[g.rng.below(pool.size())];
      uint64_t c[4], nc_[4];
      g.coef(c);
      g.neg(c, nc_);
      add_v(t, y, c);
      add_v(t, s, nc_);
      g.row(g.eq, t);
      g.n_eq++;
      aliases.push_back(y);
    }
    // constant equalities: selectors fixed to a constant
    sels.clear();
    for (uint64_t i = 0; i < k_ce; ++i) {
      t.clear();
      uint32_t s = g.fresh();
      add_v(t, s, one);
      if (g.rng.uni() < 0.8) add(g, t, 0);
      g.row(g.ce, t);
      g.n_ce++;
      sels.push_back(s);
    }
    // quadratic rows over the instance (aliases are how they see the body)
    for (uint64_t i = 0; i < k_q; ++i) {
      Terms a, b, c;
      auto pick = [&]() -> uint32_t {
        double r = g.rng.uni();
        if (r < 0.5 && !aliases.empty()) return aliases[g.rng.below(aliases.size())];
        if (r < 0.55) return first_priv + (uint32_t)g.rng.below(n_priv);
        return pool[g.rng.below(pool.size())];
      };
      if (!sels.empty() && g.rng.uni() < 0.04) {
        add_v(a, sels[g.rng.below(sels.size())], one);
      } else {
        add(g, a, pick());
        if (g.rng.uni() < 0.3) add(g, a, 0);
      }
      add(g, b, pick());
      if (g.rng.uni() < 0.4) add(g, b, pick());
      if (g.rng.uni() < 0.3) add(g, b, 0);
      uint32_t out = g.fresh();
      add_v(c, out, one);
      if (g.rng.uni() < 0.3) add(g, c, pick());
      g.row(g.na, a);
      g.row(g.nb, b);
      g.row(g.nc, c);
      g.n_q++;
    }
  }
}

static void gen_linear(Gen &g, uint64_t R, uint32_t n_pub) {
  Terms t;
  uint64_t made = 0;
  uint32_t pub_used = 0;
  auto cluster = [&](uint64_t n) {
    std::vector<uint32_t> xs;
    xs.push_back(g.fresh());
    for (uint64_t i = 0; i < n && made < R; ++i, ++made) {
      t.clear();
      uint32_t x = g.fresh();
      add(g, t, x);
      add(g, t, xs.back());
      add(g, t, xs.size() > 1 ? xs[g.rng.below(xs.size())] : g.fresh());
      if (g.rng.uni() < 0.5) add(g, t, 0);
      if (made % 64 == 63) add(g, t, 2 + (pub_used++ % n_pub));
      g.linear_row(t);
      xs.push_back(x);
    }
  };
  uint64_t big = R / 10;
  cluster(big);
  while (made < R) {
    // rows: 50% in clusters of 8, 40% in clusters of 2048 -> P(8) : P(2048) = 320 : 1
    if (g.rng.uni() < 320.0 / 321.0) cluster(8);
    else cluster(2048);
  }
}

static void gen_chain(Gen &g, uint64_t R, uint32_t n_pub) {
  // limb decompositions with carries: x_{i+1} = x_i + 2^64 * c_i - l_i, quadratic range rows
  // l_i * (l_i - 1) style, and selector rows A = {x_k} that collapse when x_k becomes constant.
  Terms t, a, b, c;
  uint64_t one[4] = {1, 0, 0, 0};
  uint64_t made = 0;
  while (made < R) {
    uint64_t depth = std::min<uint64_t>(4096, R - made);
    uint32_t x = g.fresh();
    t.clear();
    add_v(t, x, one);
    add(g, t, 0);
    g.row(g.ce, t);
    g.n_ce++;
    made++;
    for (uint64_t i = 0; i + 1 < depth && made < R; ++i) {
      uint32_t l = g.fresh(), cy = g.fresh(), nx = g.fresh();
      t.clear();
      add(g, t, nx);
      add(g, t, x);
      add(g, t, l);
      add(g, t, cy);
      g.linear_row(t);
      made++;
      a.clear(); b.clear(); c.clear();
      add_v(a, l, one);
      add_v(b, l, one);
      add(g, b, 0);
      g.row(g.na, a);
      g.row(g.nb, b);
      g.row(g.nc, c);
      g.n_q++;
      made++;
      if (g.rng.uni() < 0.05) {
        a.clear(); b.clear(); c.clear();
        add_v(a, x, one);
        add_v(b, cy, one);
        add_v(c, g.fresh(), one);
        g.row(g.na, a);
        g.row(g.nb, b);
        g.row(g.nc, c);
        g.n_q++;
        made++;
      }
      x = nx;
    }
  }
  (void)n_pub;
}

}  // namespace rs

using namespace rs;

extern "C" int rs_synth(uint32_t kind, uint64_t rows, uint64_t seed, uint32_t prime_id,
                        rs_input **out) {
  if (prime_id >= 8 || kind > 2) { set_error("rs_synth: bad kind/prime"); return RS_E_INVALID; }
  Gen g;
  g.rng.s = seed;
  memcpy(g.p, kPrimes[prime_id], 32);
  g.bits = bit_length(g.p);
  const uint32_t n_out = 1, n_pub = 32, n_priv = 32;
  g.next_sig = 1 + n_out + n_pub + n_priv;
  if (kind == 0) gen_mixed(g, rows, n_pub, n_priv, 1 + n_out + n_pub);
  else if (kind == 1) gen_linear(g, rows, n_pub);
  else gen_chain(g, rows, n_pub);
  rs_input *in = (rs_input *)calloc(1, sizeof(rs_input));
  in->prime_id = prime_id;
  memcpy(in->prime, g.p, 32);
  in->max_signal = g.next_sig;
  in->n_pub_out = n_out;
  in->n_pub_in = n_pub;
  in->n_priv_in = n_priv;
  in->n_forbidden = 1 + n_out + n_pub;
  in->forbidden = (uint32_t *)malloc(sizeof(uint32_t) * in->n_forbidden);
  for (uint64_t i = 0; i < in->n_forbidden; ++i) in->forbidden[i] = (uint32_t)i;
  to_lc(g.ce, in->cons_eq);
  to_lc(g.eq, in->eq);
  to_lc(g.lin, in->linear);
  to_lc(g.na, in->nl_a);
  to_lc(g.nb, in->nl_b);
  to_lc(g.nc, in->nl_c);
  *out = in;
  return RS_OK;
}

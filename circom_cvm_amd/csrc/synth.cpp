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
//  kind 2  chain  (config 4 stand-in, ECDSAVerify): deep process_4 chains whose composition fills
//          right-hand sides of ~2,000 terms, constant cascades that run 8 rounds, chained
//          4-limb big-integer products (see gen_chain).
//  kind 3  poseidon (config 3 stand-in): Poseidon(16) (t = 17) 16-ary Merkle paths of depth 20.
//  kind 4  sha (config 1 stand-in): sha256 compression gadgets (XOR3, Ch, Maj, BinSum, Num2Bits).
//  kind 5  templated (config 5 as SURVEY 8(d) words it): 64-row template instances replicated with
//          signal offsets, wired into chains of log-normal length (see gen_templated).
//  kind 6  templated with the 2e5 tail: kind 5 whose first chain has 9,000 instances (one ~2e5-row
//          linear cluster), so one workload has both the replication and the tail of config 5.
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

// A quadratic row A * B = C of single-signal operands (circom's `out <== x * y`).
static void quad(Gen &g, uint32_t x, uint32_t y, uint32_t out) {
  const uint64_t one[4] = {1, 0, 0, 0};
  Terms a, b, c;
  add_v(a, x, one);
  add_v(b, y, one);
  add_v(c, out, one);
  g.row(g.na, a);
  g.row(g.nb, b);
  g.row(g.nc, c);
  g.n_q++;
}
// b * (b - 1) = 0 (bit / range check)
static void bit_row(Gen &g, uint32_t x) {
  const uint64_t one[4] = {1, 0, 0, 0};
  uint64_t m1[4];
  g.neg_one(m1);
  Terms a, b, c;
  add_v(a, x, one);
  add_v(b, x, one);
  add_v(b, 0, m1);
  g.row(g.na, a);
  g.row(g.nb, b);
  g.row(g.nc, c);
  g.n_q++;
}

// kind 2 (BASELINE configs[3], circom-ecdsa ECDSAVerify stand-in): three ingredients.
//  (a) deep chains: L-row linear clusters (process_4) x_i = f(x_{i-1}, y_i, y_{i-1}); y_i and
//      x_i / y_i each occur in two rows, so the uniques phase only consumes the two end rows and the
//      ordered loop deletes x_i row by row: create_nonoverlapping_substitutions_4
//      (simplification_utils.rs:465-479) then composes x_i into a right-hand side over y_1..y_i --
//      O(L) entries, O(L^2) fill-in.  Every y_i is range checked (kept); every 64th x_i feeds a
//      quadratic row, which the frames expand to ~i entries;
//  (b) constant cascades t_k = t_{k-1}^2 from a constant t_0: row k turns linear only after round k
//      has eliminated t_{k-1} (apply_substitution_to_map, constraint_simplification.rs:345-396), so a
//      depth-D cascade runs D + 1 rounds;
//  (c) bulk: 4-limb big-integer products (16 limb products, 7 carry columns, carry range checks),
//      chained: the columns' outputs are the next product's limbs.
static void gen_chain(Gen &g, uint64_t R, uint32_t n_pub) {
  const uint64_t one[4] = {1, 0, 0, 0};
  uint64_t m1[4];
  g.neg_one(m1);
  uint64_t made = 0;
  Terms t, a, b, c;
  // (a) deep chains
  const uint64_t L = 2048;
  const uint64_t n_deep = std::max<uint64_t>(1, R / 100000);
  for (uint64_t q = 0; q < n_deep && made < R; ++q) {
    uint32_t yp = g.fresh(), xp = g.fresh();  // y before x: x has the larger id (max-id tie break)
    for (uint64_t i = 1; i <= L; ++i) {
      const uint32_t y = g.fresh(), x = g.fresh();
      t.clear();
      add(g, t, x);
      add(g, t, xp);
      add(g, t, y);
      add(g, t, yp);
      if (g.rng.uni() < 0.3) add(g, t, 0);
      g.linear_row(t);
      bit_row(g, y);
      made += 2;
      if (i % 64 == 0) {
        quad(g, x, x, g.fresh());
        made++;
      }
      yp = y;
      xp = x;
    }
  }
  // (b) constant cascades of depth 2..7 (rounds 3..8)
  for (int d = 2; d <= 7 && made < R; ++d) {
    uint32_t tp = g.fresh();
    t.clear();
    add_v(t, tp, one);
    add(g, t, 0);
    g.row(g.ce, t);
    g.n_ce++;
    made++;
    for (int k = 1; k <= d; ++k) {
      const uint32_t tk = g.fresh();
      quad(g, tp, tp, tk);
      made++;
      tp = tk;
    }
  }
  // (c) chained 4-limb products
  uint32_t A[4], B[4];
  auto fresh_limbs = [&](uint32_t *v) {
    for (int i = 0; i < 4; ++i) v[i] = g.fresh();
  };
  fresh_limbs(A);
  fresh_limbs(B);
  uint64_t two64[4] = {0, 1, 0, 0};
  uint64_t mtwo64[4];
  g.neg(two64, mtwo64);
  uint32_t pub_used = 0;
  while (made < R) {
    uint32_t P[4][4];
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) {
        P[i][j] = g.fresh();
        quad(g, A[i], B[j], P[i][j]);
        made++;
      }
    uint32_t carry = 0, out[7];
    for (int col = 0; col < 7; ++col) {
      const uint32_t cy = g.fresh();
      out[col] = g.fresh();
      t.clear();
      for (int i = 0; i < 4; ++i)
        if (col - i >= 0 && col - i < 4) add_v(t, P[i][col - i], one);
      if (carry) add_v(t, carry, one);
      add_v(t, cy, mtwo64);
      add_v(t, out[col], m1);
      if (pub_used < n_pub && g.rng.uni() < 1.0 / 8192) add(g, t, 2 + (pub_used++));
      g.linear_row(t);
      bit_row(g, cy);
      made += 2;
      carry = cy;
    }
    // the next product multiplies the low limbs of this one by fresh limbs (a chain of products)
    for (int i = 0; i < 4; ++i) A[i] = out[i];
    if (g.rng.uni() < 0.25) fresh_limbs(A);
    fresh_limbs(B);
  }
}

// kind 3 (BASELINE configs[2], Poseidon(16) Merkle tree stand-in; circomlib's constants are not
// available offline): 16-ary Merkle paths, each level = 16 one-hot selector bits (e(e-1) = 0,
// sum e = 1), 16 mux rows in_j = sib_j + e_j (cur - sib_j), then one Poseidon permutation of width
// t = 17 (R_F = 8 full rounds, R_P = 68 partial): per round an Ark row a_i = s_i + c_i per lane, the
// x^5 S-box as three quadratic rows (every lane in full rounds, lane 0 in partial rounds), and the
// MDS mix as linear rows -- dense 17-term rows in full rounds, the sparse S/V form of circomlib's
// PoseidonEx in partial rounds.  The partial rounds' lanes 1..16 pass through linear rows only, so
// each permutation's partial rounds form one ~2,300-row process_4 cluster whose merges of 17-term
// rows with 256-bit random coefficients are what stress treat_constraint_4
// (simplification_utils.rs:312-349); the S-box rows then receive right-hand sides of up to ~85 terms.
static void gen_poseidon(Gen &g, uint64_t R, uint32_t n_pub) {
  constexpr int T = 17, RF = 8, RP = 68, NR = RF + RP;
  typedef std::array<uint64_t, 4> E4;
  std::vector<E4> M(T * T), S(T), V(T), C(NR * T);  // fixed per circuit, like circomlib's tables
  for (auto *vec : {&M, &S, &V, &C})
    for (auto &x : *vec) g.rand_elem(x.data());
  const uint64_t one[4] = {1, 0, 0, 0};
  uint64_t m1[4];
  g.neg_one(m1);
  Terms t, a, b, c;
  uint64_t made = 0;
  uint32_t pub_used = 0;
  uint32_t st[T], y[T];
  while (made < R) {
    uint32_t cur = g.fresh();  // the leaf
    for (int lvl = 0; lvl < 20 && made < R; ++lvl) {
      uint32_t e[16], in[16];
      for (int j = 0; j < 16; ++j) {
        e[j] = g.fresh();
        bit_row(g, e[j]);
      }
      t.clear();
      for (int j = 0; j < 16; ++j) add_v(t, e[j], one);
      add_v(t, 0, m1);
      g.linear_row(t);
      for (int j = 0; j < 16; ++j) {
        const uint32_t sib = g.fresh();
        in[j] = g.fresh();
        a.clear(); b.clear(); c.clear();
        add_v(a, e[j], one);
        add_v(b, cur, one);
        add_v(b, sib, m1);
        add_v(c, in[j], one);
        add_v(c, sib, m1);
        g.row(g.na, a);
        g.row(g.nb, b);
        g.row(g.nc, c);
        g.n_q++;
      }
      made += 33;
      // capacity lane: a constant (initialState = 0)
      st[0] = g.fresh();
      t.clear();
      add_v(t, st[0], one);
      g.row(g.ce, t);
      g.n_ce++;
      made++;
      for (int j = 0; j < 16; ++j) st[j + 1] = in[j];
      for (int r = 0; r < NR; ++r) {
        const bool full = r < RF / 2 || r >= RF / 2 + RP;
        for (int i = 0; i < T; ++i) {  // Ark
          const uint32_t ai = g.fresh();
          uint64_t nc_[4];
          g.neg(C[r * T + i].data(), nc_);
          t.clear();
          add_v(t, ai, one);
          add_v(t, st[i], m1);
          add_v(t, 0, nc_);
          g.linear_row(t);
          made++;
          if (full || i == 0) {  // S-box x^5
            const uint32_t x2 = g.fresh(), x4 = g.fresh(), yo = g.fresh();
            quad(g, ai, ai, x2);
            quad(g, x2, x2, x4);
            quad(g, x4, ai, yo);
            made += 3;
            y[i] = yo;
          } else {
            y[i] = ai;
          }
        }
        uint32_t m[T];
        for (int i = 0; i < T; ++i) {  // Mix
          m[i] = g.fresh();
          t.clear();
          add_v(t, m[i], one);
          uint64_t nv[4];
          if (full) {
            for (int j = 0; j < T; ++j) {
              g.neg(M[i * T + j].data(), nv);
              add_v(t, y[j], nv);
            }
          } else if (i == 0) {
            for (int j = 0; j < T; ++j) {
              g.neg(S[j].data(), nv);
              add_v(t, y[j], nv);
            }
          } else {
            add_v(t, y[i], m1);
            g.neg(V[i].data(), nv);
            add_v(t, y[0], nv);
          }
          g.linear_row(t);
          made++;
        }
        for (int i = 0; i < T; ++i) st[i] = m[i];
      }
      cur = st[1];
    }
    if (pub_used < n_pub) {  // the root is published: an equality with a public input
      t.clear();
      uint64_t cc[4], nc_[4];
      g.coef(cc);
      g.neg(cc, nc_);
      add_v(t, cur, cc);
      add_v(t, 2 + (pub_used++), nc_);
      g.linear_row(t);
      made++;
    }
  }
}

// kind 4 (BASELINE configs[0], circomlib sha256_2 stand-in: circomlib is not available offline): per
// compression round the bit-level gadgets of Sha256compression -- XOR3 (sigma functions, two
// quadratic rows per bit: mid = b c, out = a (1 - 2b - 2c + 4 mid) + b + c - 2 mid), Ch (one
// quadratic row per bit), Maj (two), and BinSum adders: one long linear row sum_k sum_i 2^i in_k[i] =
// sum_i 2^i out[i] (+ carry bits), whose output bits are range checked (b (b - 1) = 0) -- plus the
// message schedule's Num2Bits rows.  ~64 rounds + 48 schedule words per compression (~30k rows).
static void gen_sha(Gen &g, uint64_t R, uint32_t n_pub) {
  const uint64_t one[4] = {1, 0, 0, 0};
  uint64_t m1[4], m2[4], four[4] = {4, 0, 0, 0};
  g.neg_one(m1);
  const uint64_t two[4] = {2, 0, 0, 0};
  g.neg(two, m2);
  Terms t, a, b, c;
  uint64_t made = 0;
  uint32_t pub_used = 0;
  auto word = [&](uint32_t *w) {
    for (int i = 0; i < 32; ++i) w[i] = g.fresh();
  };
  auto pow2 = [](int i, uint64_t v[4]) {
    v[0] = v[1] = v[2] = v[3] = 0;
    v[i / 64] = 1ULL << (i % 64);
  };
  // XOR3 of three bits -> new bit (two quadratic rows)
  auto xor3 = [&](uint32_t x, uint32_t yb, uint32_t z) -> uint32_t {
    const uint32_t mid = g.fresh(), out = g.fresh();
    quad(g, yb, z, mid);
    a.clear(); b.clear(); c.clear();
    add_v(a, x, one);
    add_v(b, 0, one);
    add_v(b, yb, m2);
    add_v(b, z, m2);
    add_v(b, mid, four);
    add_v(c, out, one);
    add_v(c, yb, m1);
    add_v(c, z, m1);
    add_v(c, mid, two);
    g.row(g.na, a);
    g.row(g.nb, b);
    g.row(g.nc, c);
    g.n_q++;
    made += 2;
    return out;
  };
  // BinSum of n 32-bit words: one linear row + 32 + carry output bits with range checks
  auto binsum = [&](const std::vector<const uint32_t *> &ops, uint32_t *out) {
    const int nc = 32 + (ops.size() > 1 ? (int)std::ceil(std::log2((double)ops.size())) : 0);
    t.clear();
    uint64_t v[4], nv[4];
    for (auto *w : ops)
      for (int i = 0; i < 32; ++i) {
        pow2(i, v);
        add_v(t, w[i], v);
      }
    for (int i = 0; i < nc; ++i) {
      const uint32_t ob = g.fresh();
      if (i < 32) out[i] = ob;
      pow2(i, v);
      g.neg(v, nv);
      add_v(t, ob, nv);
      bit_row(g, ob);
    }
    g.linear_row(t);
    made += 1 + nc;
  };
  while (made < R) {
    // message: 16 words from 512 input bits (Num2Bits of 16 words: x = sum 2^i b_i, b range-checked)
    std::vector<std::array<uint32_t, 32>> W(64);
    for (int k = 0; k < 16; ++k) {
      const uint32_t x = g.fresh();
      word(W[k].data());
      t.clear();
      uint64_t v[4];
      for (int i = 0; i < 32; ++i) {
        pow2(i, v);
        add_v(t, W[k][i], v);
        bit_row(g, W[k][i]);
      }
      add_v(t, x, m1);
      if (pub_used < n_pub && k == 0) add_v(t, 2 + (pub_used++), one);
      g.linear_row(t);
      made += 33;
    }
    for (int k = 16; k < 64 && made < R; ++k) {  // schedule: W[k] = s1(W[k-2]) + W[k-7] + s0(W[k-15]) + W[k-16]
      uint32_t s0[32], s1[32];
      for (int i = 0; i < 32; ++i) {
        s0[i] = xor3(W[k - 15][(i + 7) % 32], W[k - 15][(i + 18) % 32], W[k - 15][(i + 3) % 32]);
        s1[i] = xor3(W[k - 2][(i + 17) % 32], W[k - 2][(i + 19) % 32], W[k - 2][(i + 10) % 32]);
      }
      binsum({s1, W[k - 7].data(), s0, W[k - 16].data()}, W[k].data());
    }
    uint32_t H[8][32];
    for (auto &h : H) word(h);
    for (int r = 0; r < 64 && made < R; ++r) {
      uint32_t S1[32], ch[32], S0[32], mj[32], K[32], T1[32], T2[32], na_[32], ne_[32];
      for (int i = 0; i < 32; ++i) {
        S1[i] = xor3(H[4][(i + 6) % 32], H[4][(i + 11) % 32], H[4][(i + 25) % 32]);
        S0[i] = xor3(H[0][(i + 2) % 32], H[0][(i + 13) % 32], H[0][(i + 22) % 32]);
        // Ch = e f + (1 - e) g = e (f - g) + g
        ch[i] = g.fresh();
        a.clear(); b.clear(); c.clear();
        add_v(a, H[4][i], one);
        add_v(b, H[5][i], one);
        add_v(b, H[6][i], m1);
        add_v(c, ch[i], one);
        add_v(c, H[6][i], m1);
        g.row(g.na, a); g.row(g.nb, b); g.row(g.nc, c);
        g.n_q++;
        // Maj = a b + a c + b c - 2 a b c: mid = b c, out = a (b + c - 2 mid) + mid
        const uint32_t mid = g.fresh();
        mj[i] = g.fresh();
        quad(g, H[1][i], H[2][i], mid);
        a.clear(); b.clear(); c.clear();
        add_v(a, H[0][i], one);
        add_v(b, H[1][i], one);
        add_v(b, H[2][i], one);
        add_v(b, mid, m2);
        add_v(c, mj[i], one);
        add_v(c, mid, m1);
        g.row(g.na, a); g.row(g.nb, b); g.row(g.nc, c);
        g.n_q++;
        made += 3;
      }
      word(K);  // the round constant's bits (constants in circomlib; free signals here)
      binsum({H[7], S1, ch, K, W[r].data()}, T1);
      binsum({S0, mj}, T2);
      binsum({T1, T2}, na_);
      binsum({H[3], T1}, ne_);
      for (int w = 7; w > 0; --w) memcpy(H[w], H[w - 1], sizeof(H[w]));
      memcpy(H[0], na_, sizeof(na_));
      memcpy(H[4], ne_, sizeof(ne_));
    }
  }
}

// kind 5 (SURVEY 8(d) config 5 as written: "rows are replicated per template instance of 64 rows,
// to mimic DAG replication"): 16 templates of 64 rows each (19 eq / 3 const-eq / 22 linear / 20
// quadratic), generated once over local signal ids with fixed coefficients; every instance is a
// template with its signals offset (dag/src/lib.rs:73-78 apply_offset), so instances of a template
// share coefficients exactly as a compiled circuit's do.  Instances form wiring chains of
// log-normal length (median 2 instances, up to ~9,000 = 2e5 linear rows): instance k's 4 inputs
// are tied to instance k-1's 4 outputs by equalities (`c.in <== d.out`), so after eq renaming the
// linear rows of a chain form one cluster.  Inside a template the linear rows define internal
// signals from earlier ones (a DAG, 2-4 terms), the quadratic rows multiply defined signals (one in
// 25 with a constant selector in A: those rows turn linear and feed round 2), the equalities
// alias defined signals for the quadratic rows.
// tail (kind 6): the first chain has 9,000 instances -- one cluster of ~2e5 linear rows, the tail
// SURVEY 8(d) config 5 names -- and the rest follow the log-normal lengths above.
static void gen_templated(Gen &g, uint64_t R, uint32_t n_pub, bool tail) {
  // templates, interface, locals per instance (1-4 inputs, 5-46 definitions, 47-61 aliases, 63-65
  // selectors)
  constexpr uint32_t kT = 16, kIn = 4, kOut = 4, kL = 66;
  struct LRow {
    uint8_t blk;  // 0 eq, 1 const-eq, 2 linear, 3 quadratic
    std::vector<std::pair<uint32_t, std::array<uint64_t, 4>>> a, b, c;  // local ids (0 = constant)
  };
  std::vector<std::vector<LRow>> tpl(kT);
  const uint64_t one[4] = {1, 0, 0, 0};
  auto term = [&](uint32_t s) {
    std::array<uint64_t, 4> c;
    g.coef(c.data());
    return std::make_pair(s, c);
  };
  for (uint32_t t = 0; t < kT; ++t) {
    // locals: 1..4 inputs, then 22 linear-defined, 20 quadratic-defined, 3 selectors, 15 aliases
    std::vector<uint32_t> defd = {1, 2, 3, 4};
    uint32_t nx = kIn + 1;
    std::vector<LRow> rows;
    std::vector<uint32_t> sels;
    for (int j = 0; j < 3; ++j) {  // selectors fixed to a constant
      LRow r;
      r.blk = 1;
      const uint32_t s = kL - 1 - j;
      sels.push_back(s);
      std::array<uint64_t, 4> o;
      memcpy(o.data(), one, 32);
      r.c.push_back({s, o});
      if (g.rng.uni() < 0.8) r.c.push_back(term(0));
      rows.push_back(r);
    }
    auto pick = [&]() { return defd[defd.size() - 1 - g.rng.below(std::min<size_t>(defd.size(), 12))]; };
    uint32_t last_lin = 0, n_lin = 0;
    for (int j = 0; j < 22 + 20; ++j) {  // linear (even j and the last two) and quadratic (odd j)
      LRow r;
      const uint32_t x = nx++;
      if ((j & 1) == 0 || j >= 40) {  // linear: x = previous linear definition + 0-2 others (+ c)
        r.blk = 2;
        r.c.push_back(term(x));
        if (last_lin) r.c.push_back(term(last_lin));  // the backbone: inputs -> ... -> outputs
        if (n_lin < kIn) r.c.push_back(term(1 + n_lin));
        const int nt = (int)g.rng.below(3);
        for (int u = 0; u < nt; ++u) r.c.push_back(term(pick()));
        if (g.rng.uni() < 0.3) r.c.push_back(term(0));
        last_lin = x;
        ++n_lin;
      } else {  // quadratic: x = (a) * (b) (+ c)
        r.blk = 3;
        if (g.rng.uni() < 0.04 * 2) {
          std::array<uint64_t, 4> o;
          memcpy(o.data(), one, 32);
          r.a.push_back({sels[g.rng.below(sels.size())], o});
        } else {
          r.a.push_back(term(pick()));
          if (g.rng.uni() < 0.3) r.a.push_back(term(0));
        }
        r.b.push_back(term(pick()));
        if (g.rng.uni() < 0.4) r.b.push_back(term(pick()));
        std::array<uint64_t, 4> o;
        memcpy(o.data(), one, 32);
        r.c.push_back({x, o});
        if (g.rng.uni() < 0.3) r.c.push_back(term(pick()));
      }
      rows.push_back(r);
      defd.push_back(x);
    }
    for (int j = 0; j < 15; ++j) {  // aliases of defined signals
      LRow r;
      r.blk = 0;
      const uint32_t y = nx++;
      const uint32_t s = defd[kIn + g.rng.below(defd.size() - kIn)];
      std::array<uint64_t, 4> c, nc_;
      g.coef(c.data());
      g.neg(c.data(), nc_.data());
      r.c.push_back({y, c});
      r.c.push_back({s, nc_});
      rows.push_back(r);
      defd.push_back(y);
    }
    tpl[t] = std::move(rows);
  }
  // outputs of a template: linear-defined locals (definitions j = 40, 41, 38, 36)
  const uint32_t out_local[kOut] = {kIn + 1 + 40, kIn + 1 + 41, kIn + 1 + 38, kIn + 1 + 36};
  uint64_t made = 0;
  uint32_t pub_used = 0;
  Terms t, a, b, c;
  while (made < R) {
    double z = std::sqrt(-2.0 * std::log(std::max(g.rng.uni(), 1e-300))) * std::cos(6.283185307179586 * g.rng.uni());
    uint64_t len = (uint64_t)std::llround(2.0 * std::exp(1.3 * z));
    len = std::max<uint64_t>(1, std::min<uint64_t>(len, 9000));
    if (tail && made == 0) len = 9000;
    uint32_t prev = 0;  // base of the previous instance of the chain (0: none)
    for (uint64_t k = 0; k < len && made < R; ++k) {
      const std::vector<LRow> &T = tpl[g.rng.below(kT)];
      const uint32_t base = g.next_sig - 1;  // local l -> base + l
      g.next_sig += kL - 1;
      for (uint32_t q = 0; q < kIn; ++q) {  // wiring: in_q <== prev.out_q (or a public input)
        uint32_t src = 0;
        if (prev) src = prev + out_local[q];
        else if (pub_used < n_pub && g.rng.uni() < 1.0 / 512) src = 2 + (pub_used++);
        if (!src) continue;
        t.clear();
        uint64_t cc[4], nn[4];
        g.coef(cc);
        g.neg(cc, nn);
        add_v(t, base + 1 + q, cc);
        add_v(t, src, nn);
        g.row(g.eq, t);
        g.n_eq++;
        ++made;
      }
      for (const LRow &r : T) {
        auto off = [&](const Terms &src, Terms &dst) {
          dst.clear();
          for (auto &e : src) dst.push_back({e.first ? base + e.first : 0u, e.second});
        };
        off(r.c, c);
        if (r.blk == 3) {
          off(r.a, a);
          off(r.b, b);
          g.row(g.na, a);
          g.row(g.nb, b);
          g.row(g.nc, c);
          g.n_q++;
        } else {
          g.linear_row(c);  // classified as map_tree would (eq / const-eq / linear)
        }
        ++made;
      }
      prev = base;
    }
  }
}

}  // namespace rs

using namespace rs;

extern "C" int rs_synth(uint32_t kind, uint64_t rows, uint64_t seed, uint32_t prime_id,
                        rs_input **out) {
  if (prime_id >= 8 || kind > 6) { set_error("rs_synth: bad kind/prime"); return RS_E_INVALID; }
  Gen g;
  g.rng.s = seed;
  memcpy(g.p, kPrimes[prime_id], 32);
  g.bits = bit_length(g.p);
  const uint32_t n_out = 1, n_pub = 32, n_priv = 32;
  g.next_sig = 1 + n_out + n_pub + n_priv;
  if (kind == 0) gen_mixed(g, rows, n_pub, n_priv, 1 + n_out + n_pub);
  else if (kind == 1) gen_linear(g, rows, n_pub);
  else if (kind == 2) gen_chain(g, rows, n_pub);
  else if (kind == 3) gen_poseidon(g, rows, n_pub);
  else if (kind == 4) gen_sha(g, rows, n_pub);
  else gen_templated(g, rows, n_pub, kind == 6);
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

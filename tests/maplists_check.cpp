// maplists_check.cpp -- CPU check of circom_cvm_amd/csrc/maplists.hpp (the lazy row lists of the
// non-linear signal map across rounds) against the plain recursion it memoises
// (apply_substitution_to_map, constraint_simplification.rs:369-377).
//
// One MapLists lives through all rounds, as in the engine: after every batch is added, random
// signals are resolved and compared with the unmemoised recursion -- so a memo entry made in an
// earlier round must never answer for a different (signal, bound) pair later.
// usage: maplists_check <seed> <rounds> <signals>; prints "ok <checks>" or the first mismatch.
#include <cstdio>
#include <cstdlib>
#include <random>

#include "maplists.hpp"

using rs::MapLists;

static std::vector<uint32_t> naive(const MapLists &M, const MapLists::Lists &init, uint32_t x, size_t u) {
  std::vector<uint32_t> out;
  for (size_t b = 0; b < u; ++b) {
    const MapLists::Batch &B = M.batches[b];
    for (size_t j = 0; j < B.from.size(); ++j) {
      bool has = false;
      for (uint64_t t = B.ptr[j]; t < B.ptr[j + 1]; ++t) has |= B.keys[t] == x;
      if (!has) continue;
      auto it = init.find(B.from[j]);
      if (it != init.end()) out.insert(out.end(), it->second.begin(), it->second.end());
      const std::vector<uint32_t> r = naive(M, init, B.from[j], b);
      out.insert(out.end(), r.begin(), r.end());
    }
  }
  return out;
}

int main(int argc, char **argv) {
  const uint64_t seed = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1;
  const int rounds = argc > 2 ? atoi(argv[2]) : 6;
  const uint32_t S = argc > 3 ? (uint32_t)atoi(argv[3]) : 40;
  std::mt19937_64 rng(seed);
  // the "device": every signal's initial list (ascending rows), queried on demand
  MapLists::Lists truth;
  for (uint32_t s = 1; s < S; ++s) {
    std::vector<uint32_t> l;
    for (uint32_t r = 0; r < 30; ++r)
      if (rng() % 7 == 0) l.push_back(r);
    if (!l.empty()) truth[s] = l;
  }
  MapLists M;
  std::vector<bool> queried(S, false);
  auto query = [&](const std::vector<uint32_t> &sigs) {
    for (uint32_t s : sigs) {
      if (queried[s]) continue;
      queried[s] = true;
      auto it = truth.find(s);
      M.minit[s] = it == truth.end() ? std::vector<uint32_t>() : it->second;
    }
  };
  std::vector<bool> deleted(S, false);
  uint64_t checks = 0;
  for (int r = 0; r < rounds; ++r) {
    // a round's substitutions: distinct `from`s (never deleted before), RHS over other live signals
    MapLists::Batch B;
    B.ptr.push_back(0);
    std::vector<uint32_t> froms;
    for (uint32_t s = 1; s < S; ++s)
      if (!deleted[s] && rng() % 4 == 0) froms.push_back(s);
    std::vector<bool> is_from(S, false);
    for (uint32_t f : froms) is_from[f] = true;
    for (uint32_t f : froms) {
      std::vector<uint32_t> keys;
      for (uint32_t s = 1; s < S; ++s)
        if (!is_from[s] && !deleted[s] && rng() % 3 == 0) keys.push_back(s);
      B.from.push_back(f);
      B.keys.insert(B.keys.end(), keys.begin(), keys.end());
      B.ptr.push_back(B.keys.size());
    }
    for (uint32_t f : froms) deleted[f] = true;
    M.add_batch(std::move(B));
    // resolve a random handful, as a round asks for its turning substitutions' signals
    for (int q = 0; q < 4; ++q) {
      std::vector<uint32_t> X;
      for (uint32_t s = 1; s < S; ++s)
        if (rng() % 5 == 0) X.push_back(s);
      const MapLists::Lists got = M.resolve(X, query);
      for (uint32_t x : X) {
        const std::vector<uint32_t> want = naive(M, truth, x, M.batches.size());
        auto it = got.find(x);
        const std::vector<uint32_t> &g = it == got.end() ? std::vector<uint32_t>() : it->second;
        ++checks;
        if (g != want) {
          printf("mismatch: seed %llu round %d signal %u: got %zu entries, want %zu\n", (unsigned long long)seed, r, x, g.size(),
                 want.size());
          return 1;
        }
      }
    }
  }
  printf("ok %llu\n", (unsigned long long)checks);
  return 0;
}

// maplists.hpp -- the row lists of the non-linear signal map across rounds (host side).
//
// build_non_linear_signal_map (constraint_simplification.rs:327-343) gives every signal of a storage
// row the ascending list of those rows; apply_substitution_to_map (:345-396) then appends, for every
// substitution of a round whose `from` has a list, that list to the list of every key of its
// right-hand side (:369-377).  A later round orders the rows it turns linear by their first position
// in the list of the turning substitution's `from`, so the lists must be exact -- but most appended
// lists are never read, and building them all costs sum |RHS| x |rows| appends per round.
//
// So they are kept lazily: the initial lists of the signals asked for (`minit`, filled by a query
// callback that reads the round-1 storage rows on the device), and per round that another round
// follows its substitutions' `from` and RHS keys (a Batch).  The appended list of x over batches
// [0, u):
//     list(x, u) = concat over b < u, over the substitutions j of batch b whose RHS holds x (in order):
//                  minit[from_j] ++ list(from_j, b)
// (a substitution's `from` is in no RHS of its own round, so a batch's appends never depend on each
// other), memoised per (signal, batch bound).  Header-only and free of HIP so the CPU tests can
// check it against the plain recursion (tests/maplists_check.cpp).
#pragma once

#include <algorithm>
#include <cstdint>
#include <functional>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace rs {

struct MapLists {
  struct Batch {
    std::vector<uint32_t> from, keys;  // the round's ordered `from` list; RHS keys of substitution j
    std::vector<uint64_t> ptr;         // are keys[ptr[j], ptr[j + 1])
    // keys / ptr may be fetched on first use (the engine keeps a device copy and most rounds' lists
    // are never read); `load` fills them, once
    std::function<void(Batch &)> load;
  };
  using Lists = std::unordered_map<uint32_t, std::vector<uint32_t>>;
  Lists minit;                  // initial lists (ascending storage rows), for the queried signals only
  std::vector<Batch> batches;   // one per round that another round followed
  std::vector<Lists> bidx;      // per batch: key -> the substitutions j whose RHS holds it
  // list(x, u), keyed by (u, x): u is at most the number of rounds, x a signal id (< 2^31), so the
  // key does not depend on how many batches exist (it did once, and a key from an earlier round's
  // lookups collided with a different (x, u) after a batch was added)
  std::unordered_map<uint64_t, std::vector<uint32_t>> memo;
  static uint64_t memo_key(uint32_t x, size_t u) { return ((uint64_t)u << 32) | x; }

  void add_batch(Batch &&B) { batches.push_back(std::move(B)); }

  const Lists &index(size_t bi) {
    if (bidx.size() < batches.size()) bidx.resize(batches.size());
    Lists &ix = bidx[bi];
    if (batches[bi].load) {  // a lazily fetched batch: its keys now
      auto ld = std::move(batches[bi].load);
      batches[bi].load = nullptr;
      ld(batches[bi]);
    }
    if (ix.empty() && !batches[bi].keys.empty()) {
      const Batch &B = batches[bi];
      for (uint64_t j = 0; j < B.from.size(); ++j)
        for (uint64_t t = B.ptr[j]; t < B.ptr[j + 1]; ++t) ix[B.keys[t]].push_back((uint32_t)j);
    }
    return ix;
  }

  // list(x, u); the initial lists of every `from` it reaches must be in minit (see `reach`)
  const std::vector<uint32_t> &list(uint32_t x, size_t u) {
    const uint64_t key = memo_key(x, u);
    auto it = memo.find(key);
    if (it != memo.end()) return it->second;
    std::vector<uint32_t> out;
    for (size_t bi = 0; bi < u; ++bi) {
      const Lists &ix = index(bi);
      auto h = ix.find(x);
      if (h == ix.end()) continue;
      for (uint32_t j : h->second) {
        const uint32_t f = batches[bi].from[j];
        const std::vector<uint32_t> &L0 = minit[f];
        out.insert(out.end(), L0.begin(), L0.end());
        const std::vector<uint32_t> &pr = list(f, bi);
        out.insert(out.end(), pr.begin(), pr.end());
      }
    }
    return memo.emplace(key, std::move(out)).first->second;
  }

  // every `from` the lists of X over batches [0, upto) reach and are not memoised yet, ascending
  std::vector<uint32_t> reach(const std::vector<uint32_t> &X, size_t upto) {
    std::vector<uint32_t> froms;
    std::unordered_set<uint64_t> seen;
    std::vector<std::pair<uint32_t, size_t>> work;
    for (uint32_t x : X) work.push_back({x, upto});
    while (!work.empty()) {
      auto [x, u] = work.back();
      work.pop_back();
      const uint64_t k = memo_key(x, u);
      if (!seen.insert(k).second || memo.count(k)) continue;
      for (size_t bi = 0; bi < u; ++bi) {
        const Lists &ix = index(bi);
        auto h = ix.find(x);
        if (h == ix.end()) continue;
        for (uint32_t j : h->second) {
          froms.push_back(batches[bi].from[j]);
          work.push_back({batches[bi].from[j], bi});
        }
      }
    }
    std::sort(froms.begin(), froms.end());
    froms.erase(std::unique(froms.begin(), froms.end()), froms.end());
    return froms;
  }

  // the appended lists of the signals X over every batch so far (non-empty ones only); `query`
  // fills minit for the signals it is given (those not asked for before)
  Lists resolve(const std::vector<uint32_t> &X, const std::function<void(const std::vector<uint32_t> &)> &query) {
    Lists res;
    const size_t upto = batches.size();
    if (X.empty() || upto == 0) return res;
    query(reach(X, upto));
    for (uint32_t x : X) {
      const std::vector<uint32_t> &L = list(x, upto);
      if (!L.empty()) res[x] = L;
    }
    return res;
  }
};

}  // namespace rs

// host_common.hpp -- shared host-side helpers of librs_simplify (error state, prime table,
// owned rs_lc blocks).
#pragma once
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rs_simplify.h"

namespace rs {

void set_error(const std::string &msg);

// program_structure/src/utils/constants.rs:3-13, little-endian limbs.
extern const uint64_t kPrimes[8][4];

inline bool prime_of(const rs_input *in, uint64_t p[4]) {
  if (in->prime_id == RS_PRIME_CUSTOM) {
    memcpy(p, in->prime, 32);
    return (p[0] & 1) && (p[0] | p[1] | p[2] | p[3]) > 1;
  }
  if (in->prime_id >= 8) return false;
  memcpy(p, kPrimes[in->prime_id], 32);
  return true;
}

inline int bit_length(const uint64_t p[4]) {
  for (int i = 3; i >= 0; --i)
    if (p[i]) return 64 * i + 64 - __builtin_clzll(p[i]);
  return 0;
}

// r1cs_porting.rs:6-10
inline int field_size_bytes(const uint64_t p[4]) {
  int bits = bit_length(p);
  return bits % 64 == 0 ? bits / 8 : (bits / 64 + 1) * 8;
}

// Host-owned CSR block builder.
struct Block {
  std::vector<uint64_t> ptr{0};
  std::vector<uint32_t> col;
  std::vector<uint64_t> val;  // 4 limbs per entry
  void push(uint32_t k, const uint64_t v[4]) {
    col.push_back(k);
    val.insert(val.end(), v, v + 4);
  }
  void end_row() { ptr.push_back(col.size()); }
  uint64_t rows() const { return ptr.size() - 1; }
};

// Moves a Block into malloc'ed rs_lc arrays (freed by free_lc).
inline void to_lc(Block &b, rs_lc &lc) {
  lc.n_rows = b.rows();
  lc.nnz = b.col.size();
  lc.ptr = (uint64_t *)malloc(sizeof(uint64_t) * b.ptr.size());
  memcpy(lc.ptr, b.ptr.data(), sizeof(uint64_t) * b.ptr.size());
  lc.col = (uint32_t *)malloc(sizeof(uint32_t) * (b.col.size() ? b.col.size() : 1));
  if (!b.col.empty()) memcpy(lc.col, b.col.data(), sizeof(uint32_t) * b.col.size());
  lc.val = (uint64_t *)malloc(sizeof(uint64_t) * (b.val.size() ? b.val.size() : 4));
  if (!b.val.empty()) memcpy(lc.val, b.val.data(), sizeof(uint64_t) * b.val.size());
  b = Block();
}

// r1cs_io.cpp: the output's custom-gate sections (4 and 5) from an --O0 file, label_to_wire applied
bool r1cs_gate_sections(const char *o0_r1cs, const int32_t *l2w, uint64_t n_labels, std::vector<uint8_t> &out,
                        bool &present);

inline void free_lc(rs_lc &lc) {
  free(lc.ptr);
  free(lc.col);
  free(lc.val);
  lc.ptr = nullptr;
  lc.col = nullptr;
  lc.val = nullptr;
}

}  // namespace rs

// writer.hpp -- the .r1cs constraint section built on the device.
//
// constraint_list/src/r1cs_porting.rs:20-35 writes, per constraint in storage order, A, B and C, each
// as a u32 entry count followed by (u32 wire, field_size bytes of the coefficient) entries in the
// order constraint_writers/src/r1cs_writer.rs:49-72 sorts them: by the little-endian byte string of
// the wire (BigInt::to_bytes_le), the shorter string first on a common prefix.  Serially that is a
// HashMap walk + sort per row; here it is one radix sort of (row, byte-string key) over all entries
// and two scatter kernels into the final byte image, which the host streams to the file.
#pragma once
#include "kernels.hpp"

namespace rs {

// the LE-byte-string order of a wire id as an integer key (the host writer's le_order_key): 4 x 9 bits,
// byte + 1 per byte of the minimal LE string, 0 past its end
__device__ __forceinline__ uint64_t d_le_order_key(uint32_t k) {
  const int len = k == 0 ? 1 : (32 - __clz(k) + 7) / 8;
  uint64_t key = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint64_t b = i < len ? ((k >> (8 * i)) & 0xffu) + 1 : 0;
    key = (key << 9) | b;
  }
  return key;
}
constexpr int kLeKeyBits = 36;

// per entry of one part: sort key (row << 36 | LE key of its wire), value = the entry index
__global__ void k_w_keys(const uint64_t *ptr, uint64_t n_rows, const uint32_t *col, const int32_t *l2w, uint64_t *key,
                         uint32_t *idx, int *err) {
  for (uint64_t r = gtid(); r < n_rows; r += gstride()) {
    for (uint64_t e = ptr[r]; e < ptr[r + 1]; ++e) {
      const uint32_t c = col[e];
      const int32_t w = c == 0 ? 0 : l2w[c];
      // apply_raw_correspondence would panic: flagged, and the entry keeps a key inside its own row
      // (the largest one) so the sort and k_w_entries stay in bounds until the host reads `err`
      if (w < 0) atomicOr(err, 1);
      key[e] = (r << kLeKeyBits) | (w < 0 ? (1ull << kLeKeyBits) - 1 : d_le_order_key((uint32_t)w));
      idx[e] = (uint32_t)e;
    }
  }
}
// bytes of each constraint record: three counts + (4 + fs) per entry
__global__ void k_w_rowbytes(const uint64_t *pa, const uint64_t *pb, const uint64_t *pc, uint64_t n, uint32_t fs, uint64_t *sz) {
  for (uint64_t r = gtid(); r < n; r += gstride())
    sz[r] = 12 + (uint64_t)(4 + fs) * ((pa[r + 1] - pa[r]) + (pb[r + 1] - pb[r]) + (pc[r + 1] - pc[r]));
}
// the three counts of every record (out: 32-bit words; every offset is a multiple of 4)
__global__ void k_w_counts(const uint64_t *pa, const uint64_t *pb, const uint64_t *pc, const uint64_t *roff, uint64_t n,
                           uint32_t fs, uint32_t *out) {
  for (uint64_t r = gtid(); r < n; r += gstride()) {
    const uint64_t na = pa[r + 1] - pa[r], nb = pb[r + 1] - pb[r], nc = pc[r + 1] - pc[r];
    const uint64_t w = roff[r] / 4, es = (4 + fs) / 4;
    out[w] = (uint32_t)na;
    out[w + 1 + na * es] = (uint32_t)nb;
    out[w + 2 + (na + nb) * es] = (uint32_t)nc;
  }
}
// the entries of part q in their sorted order: wire, then the first fs bytes of the canonical value
__global__ void k_w_entries(const uint64_t *skey, const uint32_t *sidx, uint64_t nnz, int q, const uint64_t *pa,
                            const uint64_t *pb, const uint64_t *pc, const uint64_t *roff, const uint32_t *col,
                            const uint64_t *val, const int32_t *l2w, uint32_t fs, uint32_t *out) {
  const uint64_t *pq = q == 0 ? pa : (q == 1 ? pb : pc);
  const uint64_t es = (4 + fs) / 4;
  for (uint64_t j = gtid(); j < nnz; j += gstride()) {
    const uint64_t r = skey[j] >> kLeKeyBits;
    const uint32_t e = sidx[j];
    const uint64_t t = j - pq[r];
    uint64_t base = roff[r] / 4 + 1;  // after A's count
    if (q >= 1) base += (pa[r + 1] - pa[r]) * es + 1;
    if (q >= 2) base += (pb[r + 1] - pb[r]) * es + 1;
    uint32_t *o = out + base + t * es;
    const uint32_t c = col[e];
    o[0] = c == 0 ? 0u : (uint32_t)l2w[c];  // a removed signal (-1) only reaches here when err is set
    const uint32_t *v = (const uint32_t *)(val + 4 * (uint64_t)e);
    for (uint32_t i = 0; i < fs / 4; ++i) o[1 + i] = v[i];
  }
}
// wire -> label (r1cs_porting.rs:48-53): the kept signals in rank order
__global__ void k_w_w2l(const int32_t *l2w, uint64_t S, uint64_t *w2l) {
  for (uint64_t s = gtid(); s < S; s += gstride())
    if (l2w[s] >= 0) w2l[l2w[s]] = s;
}

}  // namespace rs

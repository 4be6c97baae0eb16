// r1cs_io.cpp -- the file formats around the path (host side of the drop-in boundary).
//
//   rs_read_r1cs_o0 : an --O0 .r1cs (dag/src/r1cs_porting.rs:5-135, which writes the rows in the
//                     DFS order map_tree classifies them) -> rs_input, classified exactly like
//                     dag/src/map_to_constraint_list.rs:12-44 with algebra.rs:1346-1372.
//   rs_write_r1cs   : constraint_list/src/r1cs_porting.rs:4-124 + constraint_writers/src/
//                     r1cs_writer.rs:16-353 (constraints section first, header, wire->label;
//                     keys written in lexicographic order of their minimal little-endian bytes).
//   rs_write_sym    : constraint_list/src/sym_porting.rs:5-37 -- the --O0 .sym lines with the
//                     witness column remapped (-1 when the label is not a wire).
//   rs_write_constraints_json / rs_write_substitution_json : the --json and
//                     --simplification_substitution outputs (constraint_list/src/json_porting.rs,
//                     constraint_writers/src/json_writer.rs).
#include <algorithm>
#include <cstdio>
#include <fstream>
#include <sstream>

#include "host_common.hpp"

namespace rs {

static bool read_file(const char *path, std::vector<uint8_t> &buf) {
  FILE *f = fopen(path, "rb");
  if (!f) return false;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  buf.resize(n > 0 ? n : 0);
  bool ok = n <= 0 || fread(buf.data(), 1, n, f) == (size_t)n;
  fclose(f);
  return ok;
}

template <class T>
static T rd(const uint8_t *p) {
  T v;
  memcpy(&v, p, sizeof(T));
  return v;
}

// p - a == b  for canonical nonzero a, b  (signal_equals_signal: c1 * -1 == c0)
static bool neg_equal(const uint64_t p[4], const uint64_t *a, const uint64_t *b) {
  unsigned __int128 borrow = 0;
  for (int i = 0; i < 4; ++i) {
    unsigned __int128 d = (unsigned __int128)p[i] - a[i] - (uint64_t)borrow;
    if ((uint64_t)d != b[i]) return false;
    borrow = (d >> 64) & 1;
  }
  return true;
}

// LE-byte-string order key of a signal id (r1cs_writer.rs:49-72, sort of Vec<u8> keys).
static inline uint64_t le_order_key(uint32_t k) {
  int len = k == 0 ? 1 : (32 - __builtin_clz(k) + 7) / 8;
  uint64_t key = 0;
  for (int i = 0; i < 4; ++i) {
    uint64_t b = i < len ? ((k >> (8 * i)) & 0xff) + 1 : 0;
    key = (key << 9) | b;
  }
  return key;
}

// Bounds-checked reader over one section [off, off + size) of an .r1cs buffer: every read fails
// (with the error set) instead of running past the section or the file.
struct Cursor {
  const std::vector<uint8_t> &b;
  uint64_t pos, end;
  Cursor(const std::vector<uint8_t> &buf, uint64_t off, uint64_t size) : b(buf), pos(off), end(off + size) {}
  uint64_t left() const { return end - pos; }
  bool bytes(void *dst, uint64_t n) {
    if (n > left()) { set_error("truncated r1cs section"); return false; }
    memcpy(dst, &b[pos], n);
    pos += n;
    return true;
  }
  bool skip(uint64_t n) {
    if (n > left()) { set_error("truncated r1cs section"); return false; }
    pos += n;
    return true;
  }
  bool u32(uint32_t &v) { return bytes(&v, 4); }
  bool u64(uint64_t &v) { return bytes(&v, 8); }
};

// Section table of an .r1cs file (r1cs_writer.rs:147-204): the first section of each type 1-5.
struct R1csSections {
  bool have[6] = {};
  uint64_t off[6] = {}, size[6] = {};
};
static bool scan_sections(const std::vector<uint8_t> &buf, R1csSections &S) {
  uint32_t nsec = rd<uint32_t>(&buf[8]);
  uint64_t off = 12;
  for (uint32_t s = 0; s < nsec; ++s) {
    if (off + 12 > buf.size()) { set_error("truncated r1cs section table"); return false; }
    const uint32_t t = rd<uint32_t>(&buf[off]);
    const uint64_t sz = rd<uint64_t>(&buf[off + 4]);
    off += 12;
    if (sz > buf.size() - off) { set_error("r1cs section runs past the end of the file"); return false; }
    if (t >= 1 && t <= 5 && !S.have[t]) { S.have[t] = true; S.off[t] = off; S.size[t] = sz; }
    off += sz;
  }
  return true;
}
// Custom gates applied (section 5, r1cs_writer.rs:408-450): u32 count, then per application a u32
// gate index, a u32 signal count and u64 signals.  Collects the signals (sorted, distinct) and/or
// the raw applications.
static bool read_gate_applications(const std::vector<uint8_t> &buf, const R1csSections &S, uint64_t n_labels,
                                   std::vector<uint32_t> *sigs, std::vector<std::pair<uint32_t, std::vector<uint64_t>>> *apps) {
  Cursor c(buf, S.off[5], S.size[5]);
  uint32_t na = 0;
  if (!c.u32(na)) return false;
  for (uint32_t a = 0; a < na; ++a) {
    uint32_t gi = 0, ns = 0;
    if (!c.u32(gi) || !c.u32(ns)) return false;
    if ((uint64_t)ns * 8 > c.left()) { set_error("truncated custom-gate application"); return false; }
    std::vector<uint64_t> v(ns);
    for (uint32_t i = 0; i < ns; ++i) {
      c.u64(v[i]);
      if (v[i] >= n_labels) { set_error("custom-gate signal >= n_labels"); return false; }
      if (sigs) sigs->push_back((uint32_t)v[i]);
    }
    if (apps) apps->push_back({gi, std::move(v)});
  }
  if (sigs) {
    std::sort(sigs->begin(), sigs->end());
    sigs->erase(std::unique(sigs->begin(), sigs->end()), sigs->end());
  }
  return true;
}

// Sections 4 and 5 of the output as r1cs_porting.rs:54-121 writes them, from an --O0 file's:
// section 4 unchanged, section 5 with its signals mapped label -> wire.  `out` gets the two sections
// with their headers (empty, present = false, when the --O0 file has neither).
bool r1cs_gate_sections(const char *o0_r1cs, const int32_t *l2w, uint64_t n_labels, std::vector<uint8_t> &out,
                        bool &present) {
  out.clear();
  present = false;
  std::vector<uint8_t> buf;
  if (!read_file(o0_r1cs, buf) || buf.size() < 12 || memcmp(buf.data(), "r1cs", 4) != 0) {
    set_error(std::string("cannot read r1cs file ") + o0_r1cs);
    return false;
  }
  R1csSections S;
  if (!scan_sections(buf, S)) return false;
  if (!S.have[4] && !S.have[5]) return true;
  present = true;
  auto put32 = [&](uint32_t v) { out.insert(out.end(), (uint8_t *)&v, (uint8_t *)&v + 4); };
  auto put64 = [&](uint64_t v) { out.insert(out.end(), (uint8_t *)&v, (uint8_t *)&v + 8); };
  put32(4);
  if (S.have[4]) {
    put64(S.size[4]);
    out.insert(out.end(), buf.begin() + S.off[4], buf.begin() + S.off[4] + S.size[4]);
  } else {
    put64(4);
    put32(0);
  }
  std::vector<std::pair<uint32_t, std::vector<uint64_t>>> apps;
  if (S.have[5] && !read_gate_applications(buf, S, n_labels, nullptr, &apps)) return false;
  std::vector<uint8_t> s5;
  auto p32 = [&](uint32_t v) { s5.insert(s5.end(), (uint8_t *)&v, (uint8_t *)&v + 4); };
  auto p64 = [&](uint64_t v) { s5.insert(s5.end(), (uint8_t *)&v, (uint8_t *)&v + 8); };
  p32((uint32_t)apps.size());
  for (auto &a : apps) {
    p32(a.first);
    p32((uint32_t)a.second.size());
    for (uint64_t sg : a.second) {
      if (l2w[sg] < 0) {
        set_error("custom-gate signal without a wire (SignalMap::get(..).unwrap() panics)");
        return false;
      }
      p64((uint64_t)l2w[sg]);
    }
  }
  put32(5);
  put64(s5.size());
  out.insert(out.end(), s5.begin(), s5.end());
  return true;
}

}  // namespace rs

using namespace rs;

// BigInt::to_str_radix(10) of a canonical 4-limb value
static std::string dec_string(const uint64_t *v) {
  uint64_t x[4] = {v[0], v[1], v[2], v[3]};
  char buf[96];
  int n = 0;
  do {
    unsigned __int128 rem = 0;  // x /= 10^19, digits of the remainder
    for (int i = 3; i >= 0; --i) {
      unsigned __int128 cur = (rem << 64) | x[i];
      x[i] = (uint64_t)(cur / 10000000000000000000ull);
      rem = cur % 10000000000000000000ull;
    }
    uint64_t r = (uint64_t)rem;
    const bool last = (x[0] | x[1] | x[2] | x[3]) == 0;
    for (int d = 0; d < 19 && (!last || r || d == 0); ++d) { buf[n++] = (char)('0' + r % 10); r /= 10; }
  } while (x[0] | x[1] | x[2] | x[3]);
  std::string s(buf, buf + n);
  std::reverse(s.begin(), s.end());
  return s;
}

// hashmap_as_json (json_porting.rs:16-26) + JsonValue::to_string: {"k":"v",...}, keys ascending
// (as numbers), `ids` mapped through `l2w` when given (apply_correspondence).
static bool map_json(std::string &o, const rs_lc &L, uint64_t beg, uint64_t len, const int32_t *l2w, uint64_t n_labels) {
  std::vector<std::pair<uint64_t, uint64_t>> ord;  // (key, entry)
  for (uint64_t e = beg; e < beg + len; ++e) {
    uint64_t k = L.col[e];
    if (l2w) {
      int64_t w = k < n_labels ? l2w[k] : -1;
      if (w < 0) return false;
      k = (uint64_t)w;
    }
    ord.push_back({k, e});
  }
  std::sort(ord.begin(), ord.end());
  o += '{';
  for (size_t i = 0; i < ord.size(); ++i) {
    if (i) o += ',';
    o += '"';
    o += std::to_string(ord[i].first);
    o += "\":\"";
    o += dec_string(L.val + 4 * ord[i].second);
    o += '"';
  }
  o += '}';
  return true;
}

extern "C" {

int rs_read_r1cs_o0(const char *path, rs_input **out) {
  std::vector<uint8_t> buf;
  if (!read_file(path, buf) || buf.size() < 12 || memcmp(buf.data(), "r1cs", 4) != 0) {
    set_error(std::string("cannot read r1cs file ") + path);
    return RS_E_INVALID;
  }
  R1csSections S;
  if (!scan_sections(buf, S)) return RS_E_INVALID;
  if (!S.have[1] || !S.have[2]) { set_error("r1cs without header/constraints"); return RS_E_INVALID; }
  Cursor hc(buf, S.off[1], S.size[1]);
  uint32_t fs = 0;
  if (!hc.u32(fs)) return RS_E_INVALID;
  if (fs == 0 || fs > 32 || fs % 8) { set_error("unsupported field size"); return RS_E_INVALID; }
  uint64_t p[4] = {0, 0, 0, 0};
  uint32_t n_wires = 0, n_out = 0, n_pub = 0, n_prv = 0, n_cons = 0;
  uint64_t n_labels = 0;
  if (!hc.bytes(p, fs) || !hc.u32(n_wires) || !hc.u32(n_out) || !hc.u32(n_pub) || !hc.u32(n_prv) ||
      !hc.u64(n_labels) || !hc.u32(n_cons))
    return RS_E_INVALID;
  if (n_labels == 0 || n_labels > 0x7fffffffull || 1 + (uint64_t)n_out + n_pub > n_labels) {
    set_error("r1cs header: bad label count");
    return RS_E_INVALID;
  }
  // custom-gate signals (section 5, written by dag/src/r1cs_porting.rs:74-107) are forbidden:
  // map_tree inserts every signal of a custom-gate node (dag/src/map_to_constraint_list.rs:22-24)
  std::vector<uint32_t> gate_sigs;
  if (S.have[5] && !read_gate_applications(buf, S, n_labels, &gate_sigs, nullptr)) return RS_E_INVALID;
  if (S.have[4]) {  // custom gates used (r1cs_writer.rs:358-405): checked for shape only
    Cursor gc(buf, S.off[4], S.size[4]);
    uint32_t ng = 0;
    if (!gc.u32(ng)) return RS_E_INVALID;
    for (uint32_t g = 0; g < ng; ++g) {
      uint8_t ch = 1;
      while (ch != 0)
        if (!gc.bytes(&ch, 1)) return RS_E_INVALID;
      uint32_t np = 0;
      if (!gc.u32(np) || !gc.skip((uint64_t)np * fs)) return RS_E_INVALID;
    }
  }

  // forbidden_if_main = {0} u outputs u public inputs (dag/src/lib.rs:174, 179-204) u custom-gate
  // signals, sorted and distinct
  std::vector<uint32_t> forb;
  forb.reserve(1 + (uint64_t)n_out + n_pub + gate_sigs.size());
  for (uint64_t i = 0; i < 1 + (uint64_t)n_out + n_pub; ++i) forb.push_back((uint32_t)i);
  forb.insert(forb.end(), gate_sigs.begin(), gate_sigs.end());
  std::sort(forb.begin(), forb.end());
  forb.erase(std::unique(forb.begin(), forb.end()), forb.end());

  Block ce, eq, lin, na, nb, nc;
  Cursor cc(buf, S.off[2], S.size[2]);
  std::vector<uint32_t> ks[3];
  std::vector<uint64_t> vs[3];
  for (uint32_t r = 0; r < n_cons; ++r) {
    for (int part = 0; part < 3; ++part) {
      ks[part].clear();
      vs[part].clear();
      uint32_t n = 0;
      if (!cc.u32(n)) return RS_E_INVALID;
      if ((uint64_t)n * (4 + fs) > cc.left()) { set_error("truncated r1cs constraint"); return RS_E_INVALID; }
      for (uint32_t e = 0; e < n; ++e) {
        uint32_t k = 0;
        uint64_t v[4] = {0, 0, 0, 0};
        cc.u32(k);
        cc.bytes(v, fs);
        if (k >= n_labels) { set_error("r1cs constraint: signal >= n_labels"); return RS_E_INVALID; }
        ks[part].push_back(k);
        vs[part].insert(vs[part].end(), v, v + 4);
      }
    }
    bool lin_row = ks[0].empty() && ks[1].empty();
    auto push = [&](Block &b, int part) {
      for (size_t e = 0; e < ks[part].size(); ++e) b.push(ks[part][e], &vs[part][4 * e]);
      b.end_row();
    };
    if (lin_row) {
      const auto &k = ks[2];
      bool has0 = std::find(k.begin(), k.end(), 0u) != k.end();
      if ((has0 && k.size() == 2) || (!has0 && k.size() == 1)) {
        push(ce, 2);  // signal_equals_constant
      } else if (!has0 && k.size() == 2 && neg_equal(p, &vs[2][4], &vs[2][0])) {
        push(eq, 2);  // signal_equals_signal
      } else {
        push(lin, 2);
      }
    } else {
      push(na, 0);
      push(nb, 1);
      push(nc, 2);
    }
  }
  rs_input *in = (rs_input *)calloc(1, sizeof(rs_input));
  in->prime_id = RS_PRIME_CUSTOM;
  for (int i = 0; i < 8; ++i)
    if (memcmp(kPrimes[i], p, 32) == 0) in->prime_id = i;
  memcpy(in->prime, p, 32);
  in->max_signal = n_labels;
  in->n_pub_out = n_out;
  in->n_pub_in = n_pub;
  in->n_priv_in = n_prv;
  in->n_forbidden = forb.size();
  in->forbidden = (uint32_t *)malloc(sizeof(uint32_t) * forb.size());
  memcpy(in->forbidden, forb.data(), sizeof(uint32_t) * forb.size());
  to_lc(ce, in->cons_eq);
  to_lc(eq, in->eq);
  to_lc(lin, in->linear);
  to_lc(na, in->nl_a);
  to_lc(nb, in->nl_b);
  to_lc(nc, in->nl_c);
  *out = in;
  return RS_OK;
}

void rs_input_free(rs_input *in) {
  if (!in) return;
  for (rs_lc *b : {&in->cons_eq, &in->eq, &in->linear, &in->nl_a, &in->nl_b, &in->nl_c}) free_lc(*b);
  free(in->forbidden);
  free(in);
}

}  // extern "C"

// r1cs_porting.rs:4-124.  `gates` (optional): the --O0 file's custom-gate sections, re-emitted as
// the O2 writer does (:54-121): section 4 unchanged, section 5 with every signal mapped label -> wire.
static int write_r1cs(const char *path, const rs_input *in, const rs_output *out, const char *o0_path,
                      const R1csSections *gates) {
  uint64_t p[4];
  if (!prime_of(in, p)) { set_error("unknown prime"); return RS_E_INVALID; }
  int fs = field_size_bytes(p);
  FILE *f = fopen(path, "wb");
  if (!f) { set_error(std::string("cannot write ") + path); return RS_E_INVALID; }
  std::vector<uint8_t> body;
  body.reserve(1 << 20);
  auto put32 = [&](std::vector<uint8_t> &b, uint32_t v) {
    uint8_t t[4];
    memcpy(t, &v, 4);
    b.insert(b.end(), t, t + 4);
  };
  auto put64 = [&](std::vector<uint8_t> &b, uint64_t v) {
    uint8_t t[8];
    memcpy(t, &v, 8);
    b.insert(b.end(), t, t + 8);
  };
  std::vector<std::pair<uint64_t, uint64_t>> ord;  // (order key, entry)
  const rs_lc *parts[3] = {&out->a, &out->b, &out->c};
  rs_rows it[3];
  for (int q = 0; q < 3; ++q) rs_rows_begin(out, q, &it[q]);
  const bool with_gates = gates && (gates->have[4] || gates->have[5]);
  fwrite(with_gates ? "r1cs\x01\x00\x00\x00\x05\x00\x00\x00" : "r1cs\x01\x00\x00\x00\x03\x00\x00\x00", 1, 12, f);
  // constraints section (r1cs_porting.rs:20-35) -- written first, size back-patched
  std::vector<uint8_t> hdr;
  put32(hdr, 2);
  put64(hdr, 0);
  long sec_pos = 12;
  fwrite(hdr.data(), 1, hdr.size(), f);
  uint64_t sec_size = 0;
  for (uint64_t r = 0; r < out->n_constraints; ++r) {
    body.clear();
    for (int q = 0; q < 3; ++q) {
      const rs_lc &b = *parts[q];
      ord.clear();
      uint64_t rb, rl;
      rs_rows_next(&it[q], r, &rb, &rl);
      for (uint64_t e = rb; e < rb + rl; ++e) {
        uint32_t k = b.col[e];
        uint32_t w;
        if (k == 0) w = 0;
        else {
          int64_t ww = k < out->n_labels ? out->label_to_wire[k] : -1;
          if (ww < 0) {
            fclose(f);
            set_error("constraint mentions a removed signal (apply_raw_correspondence panics)");
            return RS_E_INTERNAL;
          }
          w = (uint32_t)ww;
        }
        ord.push_back({le_order_key(w), ((uint64_t)w << 32) | (e - rb)});
      }
      std::sort(ord.begin(), ord.end());
      put32(body, (uint32_t)ord.size());
      for (auto &x : ord) {
        put32(body, (uint32_t)(x.second >> 32));
        uint64_t e = rb + (x.second & 0xffffffffu);
        const uint8_t *v = (const uint8_t *)(b.val + 4 * e);
        body.insert(body.end(), v, v + fs);
      }
    }
    fwrite(body.data(), 1, body.size(), f);
    sec_size += body.size();
  }
  long end_pos = ftell(f);
  fseek(f, sec_pos + 4, SEEK_SET);
  fwrite(&sec_size, 8, 1, f);
  fseek(f, end_pos, SEEK_SET);
  // header section (r1cs_writer.rs:246-269)
  hdr.clear();
  put32(hdr, 1);
  put64(hdr, 4 + fs + 4 * 4 + 8 + 4);
  put32(hdr, (uint32_t)fs);
  hdr.insert(hdr.end(), (const uint8_t *)p, (const uint8_t *)p + fs);
  put32(hdr, (uint32_t)out->n_wires);
  put32(hdr, (uint32_t)in->n_pub_out);
  put32(hdr, (uint32_t)in->n_pub_in);
  put32(hdr, (uint32_t)in->n_priv_in);
  put64(hdr, out->n_labels);
  put32(hdr, (uint32_t)out->n_constraints);
  fwrite(hdr.data(), 1, hdr.size(), f);
  // wire -> label section (r1cs_porting.rs:48-53, get_witness_as_vec lib.rs:187-193)
  std::vector<uint64_t> w2l(out->n_wires, 0);
  for (uint64_t s = 0; s < out->n_labels; ++s)
    if (out->label_to_wire[s] >= 0) w2l[out->label_to_wire[s]] = s;
  hdr.clear();
  put32(hdr, 3);
  put64(hdr, 8 * out->n_wires);
  fwrite(hdr.data(), 1, hdr.size(), f);
  fwrite(w2l.data(), 8, w2l.size(), f);
  if (with_gates) {
    std::vector<uint8_t> gs;
    bool present = false;
    if (!r1cs_gate_sections(o0_path, out->label_to_wire, out->n_labels, gs, present)) {
      fclose(f);
      return RS_E_INVALID;
    }
    fwrite(gs.data(), 1, gs.size(), f);
  }
  bool ok = !ferror(f);
  fclose(f);
  if (!ok) { set_error("write error"); return RS_E_INVALID; }
  return RS_OK;
}

extern "C" {

int rs_write_r1cs(const char *path, const rs_input *in, const rs_output *out) {
  return write_r1cs(path, in, out, nullptr, nullptr);
}

int rs_write_r1cs_gates(const char *path, const rs_input *in, const rs_output *out, const char *o0_r1cs) {
  std::vector<uint8_t> buf;
  if (!read_file(o0_r1cs, buf) || buf.size() < 12 || memcmp(buf.data(), "r1cs", 4) != 0) {
    set_error(std::string("cannot read r1cs file ") + o0_r1cs);
    return RS_E_INVALID;
  }
  R1csSections S;
  if (!scan_sections(buf, S)) return RS_E_INVALID;
  return write_r1cs(path, in, out, o0_r1cs, &S);
}

int rs_write_constraints_json(const char *path, const rs_output *out) {
  FILE *f = fopen(path, "wb");
  if (!f) { set_error(std::string("cannot write ") + path); return RS_E_INVALID; }
  // ConstraintJSON::new / write_constraint / end (json_writer.rs:10-45)
  fputs("{\n\"constraints\": [", f);
  std::string line;
  const rs_lc *parts[3] = {&out->a, &out->b, &out->c};
  rs_rows it[3];
  for (int q = 0; q < 3; ++q) rs_rows_begin(out, q, &it[q]);
  for (uint64_t r = 0; r < out->n_constraints; ++r) {
    line.assign(r ? ",\n[" : "\n[");
    for (int q = 0; q < 3; ++q) {
      if (q) line += ',';
      uint64_t rb, rl;
      rs_rows_next(&it[q], r, &rb, &rl);
      if (!map_json(line, *parts[q], rb, rl, out->label_to_wire, out->n_labels)) {
        fclose(f);
        set_error("constraint mentions a removed signal (apply_correspondence panics)");
        return RS_E_INTERNAL;
      }
    }
    line += ']';
    fwrite(line.data(), 1, line.size(), f);
  }
  fputs("\n]\n}", f);
  bool ok = !ferror(f);
  fclose(f);
  if (!ok) { set_error("write error"); return RS_E_INVALID; }
  return RS_OK;
}

int rs_write_substitution_json(const char *path, const rs_output *out) {
  FILE *f = fopen(path, "wb");
  if (!f) { set_error(std::string("cannot write ") + path); return RS_E_INVALID; }
  // SubstitutionJSON::new / write_substitution / end (json_writer.rs:99-131)
  fputs("{", f);
  std::string line;
  for (uint64_t i = 0; i < out->n_log; ++i) {
    line.assign(i ? ",\n\"" : "\n\"");
    line += std::to_string(out->log_from[i]);
    line += "\" : ";
    map_json(line, out->log_to, out->log_to.ptr[i], out->log_to.ptr[i + 1] - out->log_to.ptr[i], nullptr, 0);
    fwrite(line.data(), 1, line.size(), f);
  }
  fputs("\n}", f);
  bool ok = !ferror(f);
  fclose(f);
  if (!ok) { set_error("write error"); return RS_E_INVALID; }
  return RS_OK;
}

int rs_write_sym(const char *o0_sym, const char *path, const rs_output *out) {
  std::ifstream src(o0_sym);
  if (!src) { set_error(std::string("cannot read ") + o0_sym); return RS_E_INVALID; }
  FILE *f = fopen(path, "wb");
  if (!f) { set_error(std::string("cannot write ") + path); return RS_E_INVALID; }
  std::string line;
  while (std::getline(src, line)) {
    if (line.empty()) continue;
    size_t c1 = line.find(','), c2 = line.find(',', c1 + 1);
    if (c1 == std::string::npos || c2 == std::string::npos) { fclose(f); set_error("bad sym line"); return RS_E_INVALID; }
    uint64_t orig = strtoull(line.c_str(), nullptr, 10);
    int64_t w = orig < out->n_labels ? out->label_to_wire[orig] : -1;
    fprintf(f, "%llu,%lld%s\n", (unsigned long long)orig, (long long)w, line.c_str() + c2);
  }
  fclose(f);
  return RS_OK;
}

}  // extern "C"

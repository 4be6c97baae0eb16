// Host build of the device field arithmetic (circom_cvm_amd/csrc/field.hpp: the same
// __host__ __device__ functions the kernels inline), driven by tests/test_oracle.py.
// stdin, one case per line, hex: p a b  ->  stdout: a+b a-b a*b a^-1 a^2 a*b (the last by fmul256;
// canonical; a^-1 = 0 for a = 0).
// Products and the inverse go through the Montgomery form (fto_mont / fmul / finv / ffrom_mont),
// so both the 256-bit radix-2^29 path and the one-word path (p < 2^64) are exercised.
#include <cstdio>
#include <cstring>
#include <string>

#include "field.hpp"

using namespace rs;

static Fe parse(const char *s) {
  Fe x = fe_zero();
  const size_t n = strlen(s);
  for (size_t i = 0; i < n; ++i) {
    const char c = s[n - 1 - i];
    const uint64_t d = c <= '9' ? c - '0' : (c | 32) - 'a' + 10;
    x.l[i / 16] |= d << (4 * (i % 16));
  }
  return x;
}
static void put(const Fe &x) { printf("%016llx%016llx%016llx%016llx", (unsigned long long)x.l[3], (unsigned long long)x.l[2], (unsigned long long)x.l[1], (unsigned long long)x.l[0]); }

int main() {
  char ps[80], as[80], bs[80];
  while (scanf("%79s %79s %79s", ps, as, bs) == 3) {
    const Fe pf = parse(ps), a = parse(as), b = parse(bs);
    const FieldP F = make_field(pf.l);
    const Fe am = fto_mont(F, a), bm = fto_mont(F, b);
    put(fadd(F, a, b));
    printf(" ");
    put(fsub(F, a, b));
    printf(" ");
    put(ffrom_mont(F, fmul(F, am, bm)));
    printf(" ");
    put(ffrom_mont(F, finv(F, am)));
    printf(" ");
    put(ffrom_mont(F, fsqr(F, am)));
    printf(" ");
    put(ffrom_mont(F, fmul256(F, am, bm)));  // the 256-bit path on the same residues
    printf("\n");
  }
  return 0;
}

// host_common.cpp -- host-side state shared by every part of librs_simplify: the prime table and
// the per-thread error message behind rs_last_error().  Plain C++ (no HIP), so the host pieces
// (reader, writers, generator) also build alone, e.g. for the sanitizer check (oracle/Makefile asan).
#include "host_common.hpp"

namespace rs {

const uint64_t kPrimes[8][4] = {
    {0x43e1f593f0000001ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL, 0x30644e72e131a029ULL},
    {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL, 0x73eda753299d7d48ULL},
    {0xffffffff00000001ULL, 0, 0, 0},
    {0x3c208c16d87cfd47ULL, 0x97816a916871ca8dULL, 0xb85045b68181585dULL, 0x30644e72e131a029ULL},
    {0x992d30ed00000001ULL, 0x224698fc094cf91bULL, 0x0000000000000000ULL, 0x4000000000000000ULL},
    {0x8c46eb2100000001ULL, 0x224698fc0994a8ddULL, 0x0000000000000000ULL, 0x4000000000000000ULL},
    {0xffffffffffffffffULL, 0x00000000ffffffffULL, 0x0000000000000000ULL, 0xffffffff00000001ULL},
    {0x0a11800000000001ULL, 0x59aa76fed0000001ULL, 0x60b44d1e5c37b001ULL, 0x12ab655e9a2ca556ULL}};

static thread_local std::string g_err;
void set_error(const std::string &m) { g_err = m; }

}  // namespace rs

extern "C" const char *rs_last_error(void) { return rs::g_err.c_str(); }

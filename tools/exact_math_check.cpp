// Validates qkd_ldpc_v_amd/csrc/exact_math.h against the live C library.
// Usage: exact_math_check <samples_per_function_per_thread> [seed]
// Prints mismatch counts per function; exit 0 iff every result is bit-identical
// (NaN results compare equal regardless of sign/payload).
#include <initializer_list>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <cstdlib>
#include <thread>
#include <vector>
#include <atomic>
#include "../qkd_ldpc_v_amd/csrc/exact_math.h"

static inline uint64_t sm64(uint64_t &s) {
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
static inline double u01(uint64_t &s) { return (sm64(s) >> 11) * 0x1.0p-53; }
static inline bool same(double a, double b) {
    if (a != a && b != b) return true;
    uint64_t x, y; memcpy(&x, &a, 8); memcpy(&y, &b, 8); return x == y;
}
// input generators: mode selects a distribution
static double gen(uint64_t &s, int mode) {
    switch (mode) {
    case 0: { uint64_t b = sm64(s); double d; memcpy(&d, &b, 8); return d; }   // any bit pattern
    case 1: return (u01(s) * 2 - 1) * 60.0;                                     // decoder range for tanh(x/2)
    case 2: return (u01(s) * 2 - 1) * 2.0;
    case 3: { double v = 1.0 - std::ldexp(u01(s), -(int)(sm64(s) % 60)); return (sm64(s) & 1) ? v : -v; } // near +-1
    case 4: return (u01(s) * 2 - 1) * std::ldexp(1.0, (int)(sm64(s) % 80) - 70);   // tiny..moderate
    default: return (u01(s) * 2 - 1) * 1.0;
    }
}
int main(int argc, char **argv) {
    long per = argc > 1 ? atol(argv[1]) : 1000000;
    uint64_t seed0 = argc > 2 ? strtoull(argv[2], 0, 10) : 12345;
    unsigned nt = std::thread::hardware_concurrency(); if (!nt) nt = 4;
    const char *names[10] = {"tanh", "atanh", "expm1", "log1p", "tanh_bf", "atanh_bf", "expm1_bf", "log1p_bf", "tanh_dec", "atanh_dec"};
    std::atomic<long> bad[10]; for (auto &b : bad) b = 0;
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t) th.emplace_back([&, t] {
        uint64_t s = seed0 * 1000003 + t;
        for (long i = 0; i < per; ++i) {
            int mode = (int)(i % 6);
            double x = gen(s, mode);
            if (!same(ql_exact::tanh_exact(x), std::tanh(x))) { if (bad[0]++ < 5) printf("tanh  x=%a got=%a ref=%a\n", x, ql_exact::tanh_exact(x), std::tanh(x)); }
            double y = (mode == 1) ? x / 60.0 : x;
            if (!same(ql_exact::atanh_exact(y), std::atanh(y))) { if (bad[1]++ < 5) printf("atanh x=%a got=%a ref=%a\n", y, ql_exact::atanh_exact(y), std::atanh(y)); }
            double z = (mode == 1) ? x * 1.5 : x;
            if (!same(ql_exact::expm1_exact(z), std::expm1(z))) { if (bad[2]++ < 5) printf("expm1 x=%a got=%a ref=%a\n", z, ql_exact::expm1_exact(z), std::expm1(z)); }
            if (!same(ql_exact::log1p_exact(x), std::log1p(x))) { if (bad[3]++ < 5) printf("log1p x=%a got=%a ref=%a\n", x, ql_exact::log1p_exact(x), std::log1p(x)); }
            if (!same(ql_exact::tanh_bf(x), std::tanh(x))) { if (bad[4]++ < 5) printf("tanh_bf  x=%a got=%a ref=%a\n", x, ql_exact::tanh_bf(x), std::tanh(x)); }
            if (!same(ql_exact::atanh_bf(y), std::atanh(y))) { if (bad[5]++ < 5) printf("atanh_bf x=%a got=%a ref=%a\n", y, ql_exact::atanh_bf(y), std::atanh(y)); }
            if (!same(ql_exact::expm1_bf(z), std::expm1(z))) { if (bad[6]++ < 5) printf("expm1_bf x=%a got=%a ref=%a\n", z, ql_exact::expm1_bf(z), std::expm1(z)); }
            if (!same(ql_exact::tanh_dec(x), std::tanh(x))) { if (bad[8]++ < 5) printf("tanh_dec  x=%a got=%a ref=%a\n", x, ql_exact::tanh_dec(x), std::tanh(x)); }
            if (!same(ql_exact::atanh_dec(y), std::atanh(y))) { if (bad[9]++ < 5) printf("atanh_dec x=%a got=%a ref=%a\n", y, ql_exact::atanh_dec(y), std::atanh(y)); }
            if (!same(ql_exact::log1p_bf(x), std::log1p(x))) { if (bad[7]++ < 5) printf("log1p_bf x=%a got=%a ref=%a\n", x, ql_exact::log1p_bf(x), std::log1p(x)); }
        }
    });
    for (auto &x : th) x.join();
    long tot = 0;
    for (int f = 0; f < 10; ++f) { printf("%s mismatches: %ld / %ld\n", names[f], bad[f].load(), per * (long)nt); tot += bad[f]; }
    // Sweep the high words around every branch boundary of the four functions.
    const uint32_t bounds[] = {0x3FDA827A, 0xbfd2bec3, 0xbfd2bec4, 0x3e200000, 0x3c900000, 0x43400000, 0x3ff00000,
                               0x3fd62e42, 0x3FF0A2B2, 0x4043687A, 0x40862E42, 0x40360000, 0x3c800000, 0x3fe00000,
                               0x3ff6a09e, 0x3fe6a09e, 0x3e300000, 0x7ff00000};
    long bb = 0, nb = 0;
    for (uint32_t base : bounds)
        for (int d = -300; d <= 300; ++d)
            for (uint32_t lo : {0u, 1u, 0x80000000u, 0xffffffffu, 0x12345678u})
                for (int sg = 0; sg < 2; ++sg) {
                    const uint32_t hi = (base + d) ^ (sg ? 0x80000000u : 0u);
                    const uint64_t b = ((uint64_t)hi << 32) | lo;
                    double x; memcpy(&x, &b, 8);
                    const double r[10] = {std::tanh(x), std::atanh(x), std::expm1(x), std::log1p(x),
                                         std::tanh(x), std::atanh(x), std::expm1(x), std::log1p(x),
                                         std::tanh(x), std::atanh(x)};
                    const double g[10] = {ql_exact::tanh_exact(x), ql_exact::atanh_exact(x), ql_exact::expm1_exact(x),
                                         ql_exact::log1p_exact(x), ql_exact::tanh_bf(x), ql_exact::atanh_bf(x),
                                         ql_exact::expm1_bf(x), ql_exact::log1p_bf(x), ql_exact::tanh_dec(x),
                                         ql_exact::atanh_dec(x)};
                    for (int f = 0; f < 10; ++f) {
                        ++nb;
                        if (!same(r[f], g[f]) && bb++ < 5) printf("boundary %s x=%a ref=%a got=%a\n", names[f], x, r[f], g[f]);
                    }
                }
    printf("boundary mismatches: %ld / %ld\n", bb, nb);
    return (tot || bb) ? 1 : 0;
}

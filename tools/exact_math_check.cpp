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
static thread_local int dummy_flag = 0;
// the decoder's expm1 class table (exact_math.h: tanh_half_common_t)
static ql_exact::Expm1A g_ctab_a[ql_exact::EXPM1_CLASSES];
static ql_exact::Expm1B g_ctab_b[ql_exact::EXPM1_CLASSES];
static ql_exact::Expm1B g_ctab_bw[ql_exact::EXPM1_CLASSES];  // the word form (expm1_class<true>)
static inline bool same(double a, double b) {
    if (a != a && b != b) return true;
    uint64_t x, y; memcpy(&x, &a, 8); memcpy(&y, &b, 8); return x == y;
}
// both table forms; a disagreement between them is reported as a mismatch
static double tanh_t(double b, double lim, double tl) {
    const double z0 = ql_exact::tanh_half_clip_t(b, lim, tl, &dummy_flag, ql_exact::Expm1Tab{g_ctab_a, g_ctab_b, 1});
    const double z1 = ql_exact::tanh_half_clip_t<true>(b, lim, tl, &dummy_flag, ql_exact::Expm1Tab{g_ctab_a, g_ctab_bw, 1});
    return same(z0, z1) ? z0 : -999.0;
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
    for (int i = 0; i < ql_exact::EXPM1_CLASSES; ++i)
    {
        ql_exact::expm1_class(i + ql_exact::EXPM1_K_MIN, &g_ctab_a[i], &g_ctab_b[i]);
        ql_exact::expm1_class<true>(i + ql_exact::EXPM1_K_MIN, &g_ctab_a[i], &g_ctab_bw[i]);
    }
    const char *names[15] = {"tanh", "atanh", "expm1", "log1p", "tanh_bf", "atanh_bf", "expm1_bf", "log1p_bf", "tanh_dec", "atanh_dec", "tanh_half_dec", "atanh2_dec", "tanh_half_clip", "atanh2_clip", "tanh_half_clip_t"};
    std::atomic<long> bad[15]; for (auto &b : bad) b = 0;
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
            // edge forms: tanh(b / 2.) and 2. * atanh(p), on b in the decoder's +-100 and on p near +-1
            const double b = (mode == 1) ? x * (100.0 / 60.0) : x;
            if (!same(ql_exact::tanh_half_dec(b), std::tanh(b / 2.))) { if (bad[10]++ < 5) printf("tanh_half_dec b=%a got=%a ref=%a\n", b, ql_exact::tanh_half_dec(b), std::tanh(b / 2.)); }
            if (!same(ql_exact::atanh2_dec(y), 2. * std::atanh(y))) { if (bad[11]++ < 5) printf("atanh2_dec p=%a got=%a ref=%a\n", y, ql_exact::atanh2_dec(y), 2. * std::atanh(y)); }
            // clipped forms at the shipped threshold (100), a small one (10) and off (inf)
            {
                const double T = (i % 3 == 0) ? 100.0 : (i % 3 == 1) ? 10.0 : HUGE_VAL;
                const double lim = T < 44.0 ? T : 44.0;
                const double rt = std::tanh(ql_exact::clip_thr(b, T) / 2.);
                if (!same(ql_exact::tanh_half_clip(b, lim, std::tanh(lim / 2.), &dummy_flag), rt)) { if (bad[12]++ < 5) printf("tanh_half_clip b=%a T=%g got=%a ref=%a\n", b, T, ql_exact::tanh_half_clip(b, lim, std::tanh(lim / 2.), &dummy_flag), rt); }
                if (!same(tanh_t(b, lim, std::tanh(lim / 2.)), rt)) { if (bad[14]++ < 5) printf("tanh_half_clip_t b=%a T=%g got=%a ref=%a\n", b, T, tanh_t(b, lim, std::tanh(lim / 2.)), rt); }
                const double Ta = (i % 3 == 0) ? 100.0 : (i % 3 == 1) ? 3.0 : HUGE_VAL;
                const double ra = ql_exact::clip_thr(2. * std::atanh(y), Ta);
                if (!same(ql_exact::atanh2_clip(y, Ta, 2. * std::atanh(0x1.fffffffffffffp-1)), ra)) { if (bad[13]++ < 5) printf("atanh2_clip p=%a T=%g got=%a ref=%a\n", y, Ta, ql_exact::atanh2_clip(y, Ta, 2. * std::atanh(0x1.fffffffffffffp-1)), ra); }
            }
        }
    });
    for (auto &x : th) x.join();
    long tot = 0;
    for (int f = 0; f < 15; ++f) { printf("%s mismatches: %ld / %ld\n", names[f], bad[f].load(), per * (long)nt); tot += bad[f]; }
    // Sweep the high words around every branch boundary of the four functions.
    const uint32_t bounds[] = {0x3FDA827A, 0xbfd2bec3, 0xbfd2bec4, 0x3e200000, 0x3c900000, 0x43400000, 0x3ff00000,
                               0x3fd62e42, 0x3FF0A2B2, 0x4043687A, 0x40862E42, 0x40360000, 0x3c800000, 0x3fe00000,
                               0x3ff6a09e, 0x3fe6a09e, 0x3e300000, 0x7ff00000,
                               // edge forms (thresholds on b = 2x and on p)
                               0x40000000, 0x40460000, 0x3fefffff, 0x3fe00000, 0x3FE62E42, 0x4000A2B2, 0x40590000};
    long bb = 0, nb = 0;
    for (uint32_t base : bounds)
        for (int d = -300; d <= 300; ++d)
            for (uint32_t lo : {0u, 1u, 0x80000000u, 0xffffffffu, 0x12345678u})
                for (int sg = 0; sg < 2; ++sg) {
                    const uint32_t hi = (base + d) ^ (sg ? 0x80000000u : 0u);
                    const uint64_t b = ((uint64_t)hi << 32) | lo;
                    double x; memcpy(&x, &b, 8);
                    const double r[15] = {std::tanh(x), std::atanh(x), std::expm1(x), std::log1p(x),
                                         std::tanh(x), std::atanh(x), std::expm1(x), std::log1p(x),
                                         std::tanh(x), std::atanh(x), std::tanh(x / 2.), 2. * std::atanh(x),
                                         std::tanh(ql_exact::clip_thr(x, 100.0) / 2.),
                                         ql_exact::clip_thr(2. * std::atanh(x), 100.0),
                                         std::tanh(ql_exact::clip_thr(x, 100.0) / 2.)};
                    const double g[15] = {ql_exact::tanh_exact(x), ql_exact::atanh_exact(x), ql_exact::expm1_exact(x),
                                         ql_exact::log1p_exact(x), ql_exact::tanh_bf(x), ql_exact::atanh_bf(x),
                                         ql_exact::expm1_bf(x), ql_exact::log1p_bf(x), ql_exact::tanh_dec(x),
                                         ql_exact::atanh_dec(x), ql_exact::tanh_half_dec(x), ql_exact::atanh2_dec(x),
                                         ql_exact::tanh_half_clip(x, 44.0, std::tanh(22.0), &dummy_flag), ql_exact::atanh2_clip(x, 100.0, 2. * std::atanh(0x1.fffffffffffffp-1)),
                                         tanh_t(x, 44.0, std::tanh(22.0))};
                    for (int f = 0; f < 15; ++f) {
                        ++nb;
                        if (!same(r[f], g[f]) && bb++ < 5) printf("boundary %s x=%a ref=%a got=%a\n", names[f], x, r[f], g[f]);
                    }
                }
    // explicit edge values of the clipped edge forms (x and -x, three thresholds)
    {
        const double C_TOP = 2. * std::atanh(0x1.fffffffffffffp-1);
        const double vals[] = {0.0, 0x1p-1074, 0x1p-1022, 0x1p-60, 0x1p-55, 0x1p-54, 0x1.fffffffffffffp-55, 0x1p-29,
                               0x1p-28, 0x1.fffffffffffffp-29, 0.5, 0x1.fffffffffffffp-2, 1.0, 0x1.fffffffffffffp-1,
                               0x1.ffffffffffffep-1, 0x1.ffffffffffffdp-1, 1.0 - 0x1p-21, 1.0 - 0x1p-22, 0x1.0000000000001p+0,
                               2.0, 3.0, 10.0, 43.999999999999993, 44.0, 44.000000000000007, 99.99999999999999, 100.0,
                               100.00000000000001, 1e300, 1.7976931348623157e308, HUGE_VAL, NAN};
        for (double v0 : vals)
            for (int sg = 0; sg < 2; ++sg)
                for (double T : {100.0, 10.0, 3.0, (double)HUGE_VAL}) {
                    const double v = sg ? -v0 : v0;
                    const double lim = T < 44.0 ? T : 44.0;
                    const double rt = std::tanh(ql_exact::clip_thr(v, T) / 2.);
                    const double gt = ql_exact::tanh_half_clip(v, lim, std::tanh(lim / 2.), &dummy_flag);
                    const double gt2 = tanh_t(v, lim, std::tanh(lim / 2.));
                    nb += 1;
                    if (!same(rt, gt2) && bb++ < 20) printf("edge tanh_half_clip_t v=%a T=%g ref=%a got=%a\n", v, T, rt, gt2);
                    const double ra = ql_exact::clip_thr(2. * std::atanh(v), T);
                    const double ga = ql_exact::atanh2_clip(v, T, C_TOP);
                    nb += 2;
                    if (!same(rt, gt) && bb++ < 20) printf("edge tanh_half_clip v=%a T=%g ref=%a got=%a\n", v, T, rt, gt);
                    if (!same(ra, ga) && bb++ < 20) printf("edge atanh2_clip v=%a T=%g ref=%a got=%a\n", v, T, ra, ga);
                }
    }
    // atanh's log1p argument a = 2|p| / (1 - |p|) (or the small form) next to
    // every power of two: u0 = 1 + a with its high mantissa word near 0 or
    // 0xfffff (s_log1p.c's |f| < 2^-20 case and the up/down normalisation)
    {
        const double C_TOP = 2. * std::atanh(0x1.fffffffffffffp-1);
        long pb = 0;
        for (int j = -30; j <= 54; ++j)
            for (int side = -1; side <= 1; side += 2)
                for (int d = 0; d < 400; ++d) {
                    const double u0 = std::ldexp(1.0, j > 0 ? j : 0) * (side < 0 ? (1.0 - std::ldexp((double)d, -53)) : (1.0 + std::ldexp((double)d, -52)));
                    const double a = (j > 0) ? u0 - 1.0 : std::ldexp(1.0 + std::ldexp((double)d * side, -52), j);
                    for (int e = -2; e <= 2; ++e) {
                        double pv = a / (a + 2.0);
                        for (int t = 0; t < (e < 0 ? -e : e); ++t) pv = std::nextafter(pv, e < 0 ? 0.0 : 2.0);
                        for (double v : {pv, -pv}) {
                            nb += 2;
                            if (!same(ql_exact::atanh2_clip(v, HUGE_VAL, C_TOP), 2. * std::atanh(v)) && pb++ < 5)
                                printf("pow2 atanh2_clip p=%a ref=%a got=%a\n", v, 2. * std::atanh(v), ql_exact::atanh2_clip(v, HUGE_VAL, C_TOP));
                            if (!same(ql_exact::atanh2_dec(v), 2. * std::atanh(v)) && pb++ < 5)
                                printf("pow2 atanh2_dec p=%a ref=%a got=%a\n", v, 2. * std::atanh(v), ql_exact::atanh2_dec(v));
                        }
                    }
                }
        printf("power-of-two atanh mismatches: %ld\n", pb);
        bb += pb;
    }
    // log1p arguments a around s_log1p.c's k = 0 cut (hi word 0x3FDA827A) and
    // the sqrt(2) normalisation cut of u0 = 1 + a (hi word 0x3FF6A09E): for a
    // just below the k = 0 cut, 1 + a already normalises upwards
    {
        const double C_TOP = 2. * std::atanh(0x1.fffffffffffffp-1);
        long kb = 0;
        uint64_t s = 99;
        for (long i = 0; i < 4000000; ++i) {
            const uint64_t hi = 0x3FDA8270ull + (sm64(s) % 0x14);  // 0x3FDA8270 .. 0x3FDA8283
            const uint64_t bits = (hi << 32) | (sm64(s) & 0xffffffffull);
            double a; memcpy(&a, &bits, 8);
            double pv = a / (a + 2.0);
            const int e = (int)(sm64(s) % 5) - 2;
            for (int t = 0; t < (e < 0 ? -e : e); ++t) pv = std::nextafter(pv, e < 0 ? 0.0 : 2.0);
            const double v = (i & 1) ? -pv : pv;
            nb += 1;
            if (!same(ql_exact::atanh2_clip(v, HUGE_VAL, C_TOP), 2. * std::atanh(v)) && kb++ < 5)
                printf("k0-cut atanh2_clip p=%a ref=%a got=%a\n", v, 2. * std::atanh(v), ql_exact::atanh2_clip(v, HUGE_VAL, C_TOP));
        }
        printf("k0-cut atanh mismatches: %ld\n", kb);
        bb += kb;
    }
    printf("boundary mismatches: %ld / %ld\n", bb, nb);
    return (tot || bb) ? 1 : 0;
}

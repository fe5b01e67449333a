// exact_math.h — bit-exact restatement of the double-precision tanh / atanh the
// reference decoder obtains from the C library (glibc 2.35 on the reference's
// Ubuntu 22.04 image, the same image the GPU box runs).
//
// Why: the SPA decoder (reference src/qkd_ldpc_algorithm.cpp:60,68) calls
// `tanh(b2c / 2.)` and `2. * atanh(prod)` once per edge per iteration.  A GPU
// libm (ocml) differs from glibc by an ulp here and there, which makes posterior
// LLRs drift and — in non-converging frames — hard decisions diverge.  Restating
// glibc's published fdlibm-derived algorithms (expm1/log1p based; Sun fdlibm 5.3
// as carried in glibc sysdeps/ieee754/dbl-64) with the identical sequence of IEEE
// operations makes the HIP decoder bit-exact with the CPU reference, soft values
// included.  Validated against the live glibc by tests/test_exact_math.py
// (tools/exact_math_check.cpp), hundreds of millions of inputs per function.
//
// Rules for this file: every operation is a plain IEEE-754 binary64 op (no FMA
// contraction: compile with -ffp-contract=off), divisions are true divisions
// (or div_rn_safe where the operands provably need no scaling: same bits),
// and the evaluation order below is load-bearing.  Branches are written as
// branches; the compiler turns short ones into selects.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define QL_HD __host__ __device__ __forceinline__
#else
#define QL_HD static inline
#endif

namespace ql_exact {

QL_HD uint32_t hi_word(double x) {
    return (uint32_t)(__builtin_bit_cast(uint64_t, x) >> 32);
}
QL_HD uint32_t lo_word(double x) {
    return (uint32_t)__builtin_bit_cast(uint64_t, x);
}
QL_HD double with_hi_word(double x, uint32_t hi) {
    uint64_t b = __builtin_bit_cast(uint64_t, x);
    b = (b & 0xffffffffull) | ((uint64_t)hi << 32);
    return __builtin_bit_cast(double, b);
}
// a / b for operands the caller has proven to lie in the range where gfx950's
// IEEE division sequence applies no scaling (both |a|, |b| in [2^-900, 2^900]
// or a == 0, quotient normal, b finite non-zero).  There v_div_scale_f64
// returns its operands unchanged, v_div_fmas_f64 is a plain fma and
// v_div_fixup_f64 passes the quotient through, so dropping those three leaves
// the identical Newton-Raphson + correction sequence: the same correctly
// rounded quotient in 8 instructions instead of 11.  The host divides.
QL_HD double div_rn_safe(double a, double b) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(b);
    double e = __builtin_fma(-b, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-b, r, 1.0);
    r = __builtin_fma(r, e, r);
    const double q = a * r;
    const double rem = __builtin_fma(-b, q, a);
    return __builtin_fma(rem, r, q);
#else
    return a / b;
#endif
}

QL_HD double from_words(uint32_t hi, uint32_t lo) {
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | (uint64_t)lo);
}

// expm1(x) — fdlibm s_expm1.c as in glibc dbl-64 (Estrin form of the rational
// correction polynomial).  Callers here only pass finite x with |x| < 56 ln2 or
// large negative x; the overflow / NaN / inf filters are still restated.
QL_HD double expm1_exact(double x) {
    const double ln2_hi = 6.93147180369123816490e-01;  // 0x3fe62e42 fee00000
    const double ln2_lo = 1.90821492927058770002e-10;  // 0x3dea39ef 35793c76
    const double invln2 = 1.44269504088896338700e+00;  // 0x3ff71547 652b82fe
    const double Q1 = -3.33333333333331316428e-02;     // BFA11111 111110F4
    const double Q2 = 1.58730158725481460165e-03;      // 3F5A01A0 19FE5585
    const double Q3 = -7.93650757867487942473e-05;     // BF14CE19 9EAADBB7
    const double Q4 = 4.00821782732936239552e-06;      // 3ED0CFCA 86E65239
    const double Q5 = -2.01099218183624371326e-07;     // BE8AFDB7 6E09C32D
    const double o_threshold = 7.09782712893383973096e+02;

    uint32_t hx = hi_word(x);
    const uint32_t xsb = hx & 0x80000000u;
    hx &= 0x7fffffffu;

    if (hx >= 0x4043687Au) {                 // |x| >= 56 ln2
        if (hx >= 0x40862E42u) {             // |x| >= 709.78
            if (hx >= 0x7ff00000u) {
                if (((hx & 0xfffffu) | lo_word(x)) != 0) return x + x;  // NaN
                return (xsb == 0) ? x : -1.0;
            }
            if (x > o_threshold) return __builtin_inf();
        }
        if (xsb != 0) return 1.0e-300 - 1.0;  // -1 (inexact)
    }

    double hi, lo, c = 0.0, t;
    int32_t k;
    if (hx > 0x3fd62e42u) {                  // |x| > 0.5 ln2
        if (hx < 0x3FF0A2B2u) {              // and |x| < 1.5 ln2
            if (xsb == 0) { hi = x - ln2_hi; lo = ln2_lo; k = 1; }
            else          { hi = x + ln2_hi; lo = -ln2_lo; k = -1; }
        } else {
            k = (int32_t)(invln2 * x + ((xsb == 0) ? 0.5 : -0.5));
            t = (double)k;
            hi = x - t * ln2_hi;
            lo = t * ln2_lo;
        }
        x = hi - lo;
        c = (hi - x) - lo;
    } else if (hx < 0x3c900000u) {           // |x| < 2^-54
        return x;
    } else {
        k = 0;
    }

    const double hfx = 0.5 * x;
    const double hxs = x * hfx;
    const double R1 = 1.0 + hxs * Q1;
    const double h2 = hxs * hxs;
    const double R2 = Q2 + hxs * Q3;
    const double h4 = h2 * h2;
    const double R3 = Q4 + hxs * Q5;
    const double r1 = R1 + h2 * R2 + h4 * R3;
    t = 3.0 - r1 * hfx;
    double e = hxs * ((r1 - t) / (6.0 - x * t));
    if (k == 0) return x - (x * e - hxs);
    e = (x * (e - c) - c);
    e -= hxs;
    if (k == -1) return 0.5 * (x - e) - 0.5;
    if (k == 1) {
        if (x < -0.25) return -2.0 * (e - (x + 0.5));
        return 1.0 + 2.0 * (x - e);
    }
    double y;
    if (k <= -2 || k > 56) {
        y = 1.0 - (e - x);
        if (k == 1024) y = y * 2.0 * 0x1p1023;
        else y = with_hi_word(y, hi_word(y) + ((uint32_t)k << 20));
        return y - 1.0;
    }
    if (k < 20) {
        t = from_words(0x3ff00000u - (0x200000u >> k), 0u);   // 1 - 2^-k
        y = t - (e - x);
        y = with_hi_word(y, hi_word(y) + ((uint32_t)k << 20));
    } else {
        t = from_words((uint32_t)(0x3ff - k) << 20, 0u);       // 2^-k
        y = x - (e + t);
        y += 1.0;
        y = with_hi_word(y, hi_word(y) + ((uint32_t)k << 20));
    }
    return y;
}

// log1p(x) — fdlibm s_log1p.c as in glibc dbl-64 (Estrin form of the series).
QL_HD double log1p_exact(double x) {
    const double ln2_hi = 6.93147180369123816490e-01;  // 3fe62e42 fee00000
    const double ln2_lo = 1.90821492927058770002e-10;  // 3dea39ef 35793c76
        const double Lp1 = 6.666666666666735130e-01;       // 3FE55555 55555593
    const double Lp2 = 3.999999999940941908e-01;       // 3FD99999 9997FA04
    const double Lp3 = 2.857142874366239149e-01;       // 3FD24924 94229359
    const double Lp4 = 2.222219843214978396e-01;       // 3FCC71C5 1D8E78AF
    const double Lp5 = 1.818357216161805012e-01;       // 3FC74664 96CB03DE
    const double Lp6 = 1.531383769920937332e-01;       // 3FC39A09 D078C69F
    const double Lp7 = 1.479819860511658591e-01;       // 3FC2F112 DF3E5244

    const int32_t hx = (int32_t)hi_word(x);
    const int32_t ax = hx & 0x7fffffff;
    double f = 0.0, c = 0.0, u;
    int32_t k = 1, hu = 0;

    if (hx < 0x3FDA827A) {                   // x < 0.41422
        if (ax >= 0x3ff00000) {              // x <= -1.0
            if (x == -1.0) return -__builtin_inf();  // -two54/0.0
            return __builtin_nan("");                 // (x-x)/(x-x)
        }
        if (ax < 0x3e200000) {               // |x| < 2^-29
            if (ax < 0x3c900000) return x;   // |x| < 2^-54
            return x - x * x * 0.5;
        }
        if (hx > 0 || hx <= (int32_t)0xbfd2bec3) {  // -0.2929 < x < 0.41422
            k = 0; f = x; hu = 1;
        }
    } else if (hx >= 0x7ff00000) {
        return x + x;
    }
    if (k != 0) {
        if (hx < 0x43400000) {
            u = 1.0 + x;
            hu = (int32_t)hi_word(u);
            k = (hu >> 20) - 1023;
            c = (k > 0) ? 1.0 - (u - x) : x - (u - 1.0);
            c /= u;
        } else {
            u = x;
            hu = (int32_t)hi_word(u);
            k = (hu >> 20) - 1023;
            c = 0;
        }
        hu &= 0x000fffff;
        if (hu < 0x6a09e) {
            u = with_hi_word(u, (uint32_t)(hu | 0x3ff00000));
        } else {
            k += 1;
            u = with_hi_word(u, (uint32_t)(hu | 0x3fe00000));
            hu = (0x00100000 - hu) >> 2;
        }
        f = u - 1.0;
    }
    const double hfsq = 0.5 * f * f;
    if (hu == 0) {                           // |f| < 2^-20
        if (f == 0.0) {
            if (k == 0) return 0.0;
            c += k * ln2_lo;
            return k * ln2_hi + c;
        }
        const double R = hfsq * (1.0 - 0.66666666666666666 * f);
        if (k == 0) return f - R;
        return k * ln2_hi - ((R - (k * ln2_lo + c)) - f);
    }
    const double s = f / (2.0 + f);
    const double z = s * s;
    const double R1 = z * Lp1;
    const double z2 = z * z;
    const double R2 = Lp2 + z * Lp3;
    const double z4 = z2 * z2;
    const double R3 = Lp4 + z * Lp5;
    const double z6 = z4 * z2;
    const double R4 = Lp6 + z * Lp7;
    const double R = R1 + z2 * R2 + z4 * R3 + z6 * R4;
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return k * ln2_hi - ((hfsq - (s * (hfsq + R) + (k * ln2_lo + c))) - f);
}

// tanh(x) — fdlibm s_tanh.c as in glibc dbl-64.  Its two branches call
// expm1(+2|x|) or expm1(-2|x|) and then divide by (t + 2); here the argument
// and the numerator are selected first, so expm1 and the division each run
// once (bitwise the same operations: -2*|x| == -(2*|x|), -t/(t+2) == (-t)/(t+2)).
QL_HD double tanh_exact(double x) {
    const uint32_t jx = hi_word(x);
    const uint32_t ix = jx & 0x7fffffffu;
    const double ax = __builtin_fabs(x);
    const bool big = ix >= 0x3ff00000u;      // |x| >= 1
    const double two_ax = 2.0 * ax;
    const double t = expm1_exact(big ? two_ax : -two_ax);
    const double q = (big ? 2.0 : -t) / (t + 2.0);
    double z = big ? 1.0 - q : q;
    if (ix >= 0x40360000u) z = 1.0 - 1.0e-300;  // |x| >= 22 (incl. inf): 1 (inexact)
    z = ((int32_t)jx >= 0) ? z : -z;
    if (ix < 0x3c800000u) z = x * (1.0 + x);     // |x| < 2^-55 (x*(1+x) == x also at +-0)
    if (x != x) z = x + x;                       // NaN
    return z;
}

// atanh(x) — glibc dbl-64 e_atanh.c (log1p based).  Both finite branches
// call log1p once; the argument is selected first.
QL_HD double atanh_exact(double x) {
    const double xa = __builtin_fabs(x);
    const bool small = xa < 0.5;
    const double twoxa = xa + xa;
    const double den = 1.0 - xa;
    // small: t + t*xa/(1-xa) with t = 2xa; else (xa+xa)/(1-xa)
    const double num = small ? twoxa * xa : twoxa;
    const double qd = num / den;
    const double arg = small ? twoxa + qd : qd;
    double t = 0.5 * log1p_exact(arg);
    t = __builtin_copysign(t, x);
    if (xa < 0x1.0p-28) t = x;
    if (!(xa < 1.0)) {                           // |x| >= 1 or NaN
        t = (xa > 1.0) ? __builtin_nan("") : __builtin_copysign(__builtin_inf(), x);  // x/0.0
        if (x != x) t = x + x;
    }
    return t;
}

// ---------------------------------------------------------------------------
// Branch-free forms (what the GPU kernels call).  Identical IEEE operation
// sequences to the functions above, but every case's cheap tail is computed and
// the right one selected, while the expensive shared part (argument reduction,
// polynomial, the division) runs once.  A wave whose lanes fall in different
// cases then runs one path instead of several.  Exact for every input
// (tools/exact_math_check.cpp tests both forms against the C library).

QL_HD double add_exponent(double y, int32_t k) {  // y * 2^k by exponent add (glibc SET_HIGH_WORD)
    return with_hi_word(y, hi_word(y) + ((uint32_t)k << 20));
}

QL_HD double expm1_bf(double x) {
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double invln2 = 1.44269504088896338700e+00;
    const double Q1 = -3.33333333333331316428e-02, Q2 = 1.58730158725481460165e-03;
    const double Q3 = -7.93650757867487942473e-05, Q4 = 4.00821782732936239552e-06;
    const double Q5 = -2.01099218183624371326e-07;
    const double o_threshold = 7.09782712893383973096e+02;

    const uint32_t hw = hi_word(x);
    const bool neg = (hw & 0x80000000u) != 0;
    const uint32_t hx = hw & 0x7fffffffu;
    // argument reduction: k = 0 (|x| <= ln2/2), +-1 (|x| < 1.5 ln2), else rounded
    const int32_t kgen = (int32_t)(invln2 * x + (neg ? -0.5 : 0.5));
    int32_t k = (hx < 0x3FF0A2B2u) ? (neg ? -1 : 1) : kgen;
    k = (hx > 0x3fd62e42u) ? k : 0;
    const double t = (double)k;
    const double hi = x - t * ln2_hi;   // == x - ln2_hi / x + ln2_hi at k = +-1, == x at k = 0
    const double lo = t * ln2_lo;
    const double xr = hi - lo;
    const double c = (hi - xr) - lo;
    // shared rational correction
    const double hfx = 0.5 * xr;
    const double hxs = xr * hfx;
    const double R1 = 1.0 + hxs * Q1;
    const double h2 = hxs * hxs;
    const double R2 = Q2 + hxs * Q3;
    const double h4 = h2 * h2;
    const double R3 = Q4 + hxs * Q5;
    const double r1 = R1 + h2 * R2 + h4 * R3;
    const double t3 = 3.0 - r1 * hfx;
    const double e = hxs * ((r1 - t3) / (6.0 - xr * t3));
    // reconstructions
    const double y0 = xr - (xr * e - hxs);                       // k == 0
    const double e2 = (xr * (e - c) - c) - hxs;
    const double ym1 = 0.5 * (xr - e2) - 0.5;                    // k == -1
    const double yp1 = (xr < -0.25) ? -2.0 * (e2 - (xr + 0.5)) : 1.0 + 2.0 * (xr - e2);  // k == 1
    const bool far = (k <= -2 || k > 56);
    const int32_t kb = (k < 2) ? 2 : ((k > 19) ? 19 : k);        // keep the shift defined
    const double tb = from_words(0x3ff00000u - (0x200000u >> kb), 0u);   // 1 - 2^-k
    const double tc = from_words((uint32_t)(0x3ff - k) << 20, 0u);       // 2^-k
    const double ya = (far ? 1.0 : tb) - (e2 - xr);              // far, or 2 <= k < 20
    const double yc = (xr - (e2 + tc)) + 1.0;                    // 20 <= k <= 56
    const double ypre = (far || k < 20) ? ya : yc;
    const double ysc = (k == 1024) ? ypre * 2.0 * 0x1p1023 : add_exponent(ypre, k);
    double y = far ? ysc - 1.0 : ysc;
    y = (k == 1) ? yp1 : y;
    y = (k == -1) ? ym1 : y;
    y = (k == 0) ? y0 : y;
    // filters
    if (hx < 0x3c900000u) y = x;                                 // |x| < 2^-54
    if (hx >= 0x4043687Au && neg) y = 1.0e-300 - 1.0;            // x < -56 ln2: -1
    if (hx >= 0x40862E42u) {
        if (x > o_threshold) y = __builtin_inf();
        if (hx >= 0x7ff00000u) y = (((hx & 0xfffffu) | lo_word(x)) != 0) ? x + x : (neg ? -1.0 : x);
    }
    return y;
}

QL_HD double log1p_bf(double x) {
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01;
    const double Lp3 = 2.857142874366239149e-01, Lp4 = 2.222219843214978396e-01;
    const double Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01;
    const double Lp7 = 1.479819860511658591e-01;

    const int32_t hx = (int32_t)hi_word(x);
    const int32_t ax = hx & 0x7fffffff;
    const bool small = hx < 0x3FDA827A;
    const bool k0 = small && (hx > 0 || hx <= (int32_t)0xbfd2bec3);  // -0.2929 < x < 0.41422
    // k != 0 path: u = 1 + x (or x when x >= 2^53), normalised into [sqrt(2)/2, sqrt(2))
    const bool huge = hx >= 0x43400000;
    const double u0 = huge ? x : 1.0 + x;
    int32_t hu = (int32_t)hi_word(u0);
    int32_t k = (hu >> 20) - 1023;
    double c = (k > 0) ? 1.0 - (u0 - x) : x - (u0 - 1.0);
    c = huge ? 0.0 : c / u0;
    hu &= 0x000fffff;
    const bool up = hu >= 0x6a09e;
    const double u = with_hi_word(u0, (uint32_t)(hu | (up ? 0x3fe00000 : 0x3ff00000)));
    k = up ? k + 1 : k;
    hu = up ? (0x00100000 - hu) >> 2 : hu;
    double f = u - 1.0;
    // k == 0 path takes x itself
    f = k0 ? x : f;
    k = k0 ? 0 : k;
    hu = k0 ? 1 : hu;
    c = k0 ? 0.0 : c;
    const double hfsq = 0.5 * f * f;
    const double dk = (double)k;
    // main series
    const double s = f / (2.0 + f);
    const double z = s * s;
    const double R1 = z * Lp1;
    const double z2 = z * z;
    const double R2 = Lp2 + z * Lp3;
    const double z4 = z2 * z2;
    const double R3 = Lp4 + z * Lp5;
    const double z6 = z4 * z2;
    const double R4 = Lp6 + z * Lp7;
    const double R = R1 + z2 * R2 + z4 * R3 + z6 * R4;
    double y = (k == 0) ? f - (hfsq - s * (hfsq + R))
                        : dk * ln2_hi - ((hfsq - (s * (hfsq + R) + (dk * ln2_lo + c))) - f);
    // |f| < 2^-20 path
    const double Rs = hfsq * (1.0 - 0.66666666666666666 * f);
    const double ysmall = (k == 0) ? f - Rs : dk * ln2_hi - ((Rs - (dk * ln2_lo + c)) - f);
    const double yzero = (k == 0) ? 0.0 : dk * ln2_hi + (c + dk * ln2_lo);
    y = (hu == 0) ? ((f == 0.0) ? yzero : ysmall) : y;
    // specials
    if (small && ax < 0x3e200000) y = (ax < 0x3c900000) ? x : x - x * x * 0.5;  // |x| < 2^-29
    if (small && ax >= 0x3ff00000) y = (x == -1.0) ? -__builtin_inf() : __builtin_nan("");  // x <= -1
    if (!small && hx >= 0x7ff00000) y = x + x;                                   // +inf / NaN
    return y;
}

QL_HD double tanh_bf(double x) {
    const uint32_t jx = hi_word(x);
    const uint32_t ix = jx & 0x7fffffffu;
    const double ax = __builtin_fabs(x);
    const bool big = ix >= 0x3ff00000u;
    const double two_ax = 2.0 * ax;
    const double t = expm1_bf(big ? two_ax : -two_ax);
    const double q = (big ? 2.0 : -t) / (t + 2.0);
    double z = big ? 1.0 - q : q;
    z = (ix >= 0x40360000u) ? 1.0 - 1.0e-300 : z;
    z = ((int32_t)jx >= 0) ? z : -z;
    z = (ix < 0x3c800000u) ? x * (1.0 + x) : z;
    z = (x != x) ? x + x : z;
    return z;
}

QL_HD double atanh_bf(double x) {
    const double xa = __builtin_fabs(x);
    const bool small = xa < 0.5;
    const double twoxa = xa + xa;
    const double qd = (small ? twoxa * xa : twoxa) / (1.0 - xa);
    double t = 0.5 * log1p_bf(small ? twoxa + qd : qd);
    t = __builtin_copysign(t, x);
    t = (xa < 0x1.0p-28) ? x : t;
    t = (xa > 1.0) ? __builtin_nan("") : t;
    t = (xa == 1.0) ? __builtin_copysign(__builtin_inf(), x) : t;
    t = (x != x) ? x + x : t;
    return t;
}

// ---------------------------------------------------------------------------
// Decoder forms: tanh / atanh with their expm1 / log1p cores specialised to the
// arguments tanh and atanh can hand them when their own result is used.
//   tanh:  the expm1 result matters only for |x| < 22, i.e. for arguments
//          u in (-2, 0] u [2, 44): k is never 1 or 1024, u is never tiny
//          (|x| < 2^-55 is tanh's own tiny case), never < -56 ln2, never
//          overflows.  Those expm1 cases are dropped.
//   atanh: the log1p result matters only for 2^-28 <= |x| < 1, i.e. for
//          arguments in [2^-27, 2^54]: finite, >= 0, never tiny.
// Outside those ranges the final selects of tanh/atanh take over, so both
// functions remain bit-exact for EVERY input (tools/exact_math_check.cpp).

QL_HD double tanh_dec(double x) {
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double invln2 = 1.44269504088896338700e+00;
    const double Q1 = -3.33333333333331316428e-02, Q2 = 1.58730158725481460165e-03;
    const double Q3 = -7.93650757867487942473e-05, Q4 = 4.00821782732936239552e-06;
    const double Q5 = -2.01099218183624371326e-07;

    const uint32_t jx = hi_word(x);
    const uint32_t ix = jx & 0x7fffffffu;
    const double ax = __builtin_fabs(x);
    const bool big = ix >= 0x3ff00000u;          // |x| >= 1: expm1(2|x|), else expm1(-2|x|)
    const double two_ax = 2.0 * ax;
    const double u = big ? two_ax : -two_ax;
    // --- expm1(u) core (s_expm1.c) ---
    const uint32_t uh = hi_word(two_ax);
    const int32_t kgen = (int32_t)(invln2 * u + (big ? 0.5 : -0.5));
    int32_t k = (uh < 0x3FF0A2B2u) ? -1 : kgen;  // only u < 0 reaches |u| < 1.5 ln2
    k = (uh > 0x3fd62e42u) ? k : 0;
    const double t = (double)k;
    const double hi = u - t * ln2_hi;
    const double lo = t * ln2_lo;
    const double xr = hi - lo;
    const double c = (hi - xr) - lo;
    const double hfx = 0.5 * xr;
    const double hxs = xr * hfx;
    const double R1 = 1.0 + hxs * Q1;
    const double h2 = hxs * hxs;
    const double R2 = Q2 + hxs * Q3;
    const double h4 = h2 * h2;
    const double R3 = Q4 + hxs * Q5;
    const double r1 = R1 + h2 * R2 + h4 * R3;
    const double t3 = 3.0 - r1 * hfx;
    // |xr| <= 0.35: denominator ~6, numerator ~-2 (div_rn_safe range)
    const double e = hxs * div_rn_safe(r1 - t3, 6.0 - xr * t3);
    const double y0 = xr - (xr * e - hxs);                       // k == 0
    const double e2 = (xr * (e - c) - c) - hxs;
    const double ym1 = 0.5 * (xr - e2) - 0.5;                    // k == -1
    const bool far = (k <= -2 || k > 56);
    const int32_t kb = (k < 2) ? 2 : ((k > 19) ? 19 : k);
    const double tb = from_words(0x3ff00000u - (0x200000u >> kb), 0u);
    const double tc = from_words((uint32_t)(0x3ff - k) << 20, 0u);
    const double ya = (far ? 1.0 : tb) - (e2 - xr);
    const double yc = (xr - (e2 + tc)) + 1.0;
    const double ysc = add_exponent((far || k < 20) ? ya : yc, k);
    double y = far ? ysc - 1.0 : ysc;
    y = (k == -1) ? ym1 : y;
    y = (k == 0) ? y0 : y;
    // --- tanh from t = expm1(u) (s_tanh.c) ---
    // used only for 2^-55 <= |x| < 22: y + 2 in [1.13, 1.3e19], q in [1.5e-19, 0.87]
    const double q = div_rn_safe(big ? 2.0 : -y, y + 2.0);
    double z = big ? 1.0 - q : q;
    z = (ix >= 0x40360000u) ? 1.0 - 1.0e-300 : z;
    z = ((int32_t)jx >= 0) ? z : -z;
    z = (ix < 0x3c800000u) ? x * (1.0 + x) : z;
    z = (x != x) ? x + x : z;
    return z;
}

QL_HD double atanh_dec(double x) {
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01;
    const double Lp3 = 2.857142874366239149e-01, Lp4 = 2.222219843214978396e-01;
    const double Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01;
    const double Lp7 = 1.479819860511658591e-01;

    const double xa = __builtin_fabs(x);
    const bool smallx = xa < 0.5;
    const double twoxa = xa + xa;
    // result used only for 2^-28 <= |x| < 1: numerator in [2^-55, 2), 1 - |x| in [2^-53, 1]
    const double qd = div_rn_safe(smallx ? twoxa * xa : twoxa, 1.0 - xa);
    const double a = smallx ? twoxa + qd : qd;   // log1p argument, in [2^-27, 2^54]
    // --- log1p(a) core (s_log1p.c) ---
    const int32_t hx = (int32_t)hi_word(a);
    const bool k0 = hx < 0x3FDA827A;             // a < 0.41422: f = a, k = 0
    const bool huge = hx >= 0x43400000;
    const double u0 = huge ? a : 1.0 + a;
    int32_t hu = (int32_t)hi_word(u0);
    int32_t k = (hu >> 20) - 1023;
    double c = (k > 0) ? 1.0 - (u0 - a) : a - (u0 - 1.0);
    // matters only for a in [0.414, 2^54): c = 0 or |c| in [2^-54, 2], u0 in [1.4, 2^54]
    c = huge ? 0.0 : div_rn_safe(c, u0);
    hu &= 0x000fffff;
    const bool up = hu >= 0x6a09e;
    const double u = with_hi_word(u0, (uint32_t)(hu | (up ? 0x3fe00000 : 0x3ff00000)));
    k = up ? k + 1 : k;
    hu = up ? (0x00100000 - hu) >> 2 : hu;
    double f = u - 1.0;
    f = k0 ? a : f;
    k = k0 ? 0 : k;
    hu = k0 ? 1 : hu;
    c = k0 ? 0.0 : c;
    const double hfsq = 0.5 * f * f;
    const double dk = (double)k;
    const double s = div_rn_safe(f, 2.0 + f);       // f = 0 or |f| in [2^-54, 0.42]
    const double z = s * s;
    const double R1 = z * Lp1;
    const double z2 = z * z;
    const double R2 = Lp2 + z * Lp3;
    const double z4 = z2 * z2;
    const double R3 = Lp4 + z * Lp5;
    const double z6 = z4 * z2;
    const double R4 = Lp6 + z * Lp7;
    const double R = R1 + z2 * R2 + z4 * R3 + z6 * R4;
    // k == 0 uses the k != 0 formula with dk = c = 0: 0*ln2_hi - ((hfsq - (P + 0)) - f)
    // == f - (hfsq - P) bitwise, since a - b == -(b - a) exactly and no zero
    // result occurs on this path (f = a > 0).
    double y = dk * ln2_hi - ((hfsq - (s * (hfsq + R) + (dk * ln2_lo + c))) - f);
    if (__builtin_expect(hu == 0, 0)) {          // |f| < 2^-20: rare
        const double Rs = hfsq * (1.0 - 0.66666666666666666 * f);
        const double ysmall = (k == 0) ? f - Rs : dk * ln2_hi - ((Rs - (dk * ln2_lo + c)) - f);
        const double yzero = (k == 0) ? 0.0 : dk * ln2_hi + (c + dk * ln2_lo);
        y = (f == 0.0) ? yzero : ysmall;
    }
    // --- atanh (e_atanh.c) ---
    double t = __builtin_copysign(0.5 * y, x);
    t = (xa < 0x1.0p-28) ? x : t;
    t = (xa > 1.0) ? __builtin_nan("") : t;
    t = (xa == 1.0) ? __builtin_copysign(__builtin_inf(), x) : t;
    t = (x != x) ? x + x : t;
    return t;
}


// ---------------------------------------------------------------------------
// Edge forms (what the SPA kernel calls): the reference's two per-edge calls
// with their scalings folded in, `tanh(b / 2.)` (src/qkd_ldpc_algorithm.cpp:60)
// and `2. * atanh(p)` (:68).  Same IEEE operations as tanh_dec / atanh_dec on
// every input; what changes is how the cases are combined:
//   * the expm1 reconstructions of every k class tanh can reach are one
//     expression, y = add_exponent((xr - (e2 + X3)) + X4, k) + B, with the
//     per-class constants X3, X4, B selected by integer ops (derivation below);
//   * the rare inputs (tiny, |x| >= 22, inf, NaN; atanh's |p| >= 1 - 2^-21,
//     |p| < 2^-28) are recomputed by the full restatement in a branch the
//     wave only enters when one of its lanes needs it (QL_RARE);
//   * b / 2 is never formed on the common path: |b| = 2|x| is the expm1
//     argument magnitude itself; 2 * copysign(0.5 * y, p) == copysign(y, p).
// A divergent `if` on a rare lane condition: the wave skips the body (exec
// empty) unless one of its lanes needs it.  QL_COUNT_COMMON drops the rare
// bodies — for instruction counting only, never in a product build.
#if defined(QL_COUNT_COMMON)
#define QL_RARE(c) if (false)
#else
#define QL_RARE(c) if (__builtin_expect((c), 0))
#endif

// tanh(b / 2.) bit-identical to glibc.  Common path: 2^-54 <= |b| < 44 (that
// is 2^-55 <= |x| < 22 for x = b/2, computed exactly as |b|/2).
//
// expm1(u), u = +-|b|, reconstructions of s_expm1.c with D = xr - e2:
//   k = 0        xr - (xr*e - hxs)             == D              (c = +0 here)
//   k = -1       0.5*(xr - e2) - 0.5           == add_exp(D + -1, -1)
//                 (0.5*D exact, and RN commutes with scaling by 2^-1)
//   k <= -2, k > 56   add_exp(1 - (e2 - xr), k) - 1 == add_exp(D + 1, k) + -1
//   2 <= k < 20  add_exp((1 - 2^-k) - (e2 - xr), k) == add_exp(D + tb, k)
//   20 <= k <= 56  add_exp((xr - (e2 + 2^-k)) + 1, k)
// (a - (e2 - xr) == a + (xr - e2) bitwise for a != 0; e2 + -0 == e2; y + -0 == y).
// k = 1 and k = 1024 are unreachable (u in (-2, 0] or [2, 44)).
// tanh tail: z = C + num / (y + 2) with (x > 0 shown; x < 0 negates C, num)
//   |x| < 1:  C = -0, num = -y        (z = -y/(y+2))
//   |x| >= 1: C = 1,  num = -2        (z = 1 - 2/(y+2))
QL_HD double tanh_half_full(double b) { return tanh_dec(b / 2.); }

// Common path of tanh(b / 2.); *ib = hi word of |b|.  Exact for
// 2^-54 <= |b| < 44; other lanes get a don't-care value.
QL_HD double tanh_half_common(double b, uint32_t *ib_out) {
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double invln2 = 1.44269504088896338700e+00;
    const double Q1 = -3.33333333333331316428e-02, Q2 = 1.58730158725481460165e-03;
    const double Q3 = -7.93650757867487942473e-05, Q4 = 4.00821782732936239552e-06;
    const double Q5 = -2.01099218183624371326e-07;

    const uint32_t jb = hi_word(b);
    const uint32_t ib = jb & 0x7fffffffu;         // hi word of |b| = 2|x|
    const uint32_t sx = jb & 0x80000000u;
    const bool big = ib >= 0x40000000u;            // |x| >= 1
    const double ab = __builtin_fabs(b);
    const double u = big ? ab : -ab;
    double kf = invln2 * u + (big ? 0.5 : -0.5);
#if !defined(__HIP_DEVICE_COMPILE__)
    kf = (kf > 1e6 || kf < -1e6 || kf != kf) ? 0.0 : kf;  // host: keep the cast defined on special lanes
#endif
    int32_t k = (ib < 0x3FF0A2B2u) ? -1 : (int32_t)kf;   // only u < 0 reaches |u| < 1.5 ln2
    k = (ib > 0x3fd62e42u) ? k : 0;
    const double t = (double)k;
    const double hi = u - t * ln2_hi;
    const double lo = t * ln2_lo;
    const double xr = hi - lo;
    const double c = (hi - xr) - lo;
    const double hfx = 0.5 * xr;
    const double hxs = xr * hfx;
    const double R1 = 1.0 + hxs * Q1;
    const double h2 = hxs * hxs;
    const double R2 = Q2 + hxs * Q3;
    const double h4 = h2 * h2;
    const double R3 = Q4 + hxs * Q5;
    const double r1 = R1 + h2 * R2 + h4 * R3;
    const double t3 = 3.0 - r1 * hfx;
    const double e = hxs * div_rn_safe(r1 - t3, 6.0 - xr * t3);
    const double e2 = (xr * (e - c) - c) - hxs;
    // per-class constants (all with a zero low word)
    const uint32_t ku = (uint32_t)k;
    const bool fcls = (ku - 20u) <= 36u;           // 20 <= k <= 56
    const bool far = (ku + 1u) > 57u;              // k <= -2 or k > 56
    uint32_t a_hi = 0x3ff00000u - (0x200000u >> (ku & 31u));   // 1 - 2^-k; 1 when far
    a_hi = (k == 0) ? 0x80000000u : a_hi;          // -0
    a_hi = (k == -1) ? 0xbff00000u : a_hi;         // -1
    const double X3 = from_words(fcls ? (0x3ff00000u - (ku << 20)) : 0x80000000u, 0u);  // 2^-k or -0
    const double X4 = from_words(fcls ? 0x3ff00000u : a_hi, 0u);
    const double B = from_words(far ? 0xbff00000u : 0x80000000u, 0u);                 // -1 or -0
    const double y = add_exponent((xr - (e2 + X3)) + X4, k) + B;
    const double num = big ? from_words(0xc0000000u ^ sx, 0u) : from_words(hi_word(y) ^ 0x80000000u ^ sx, lo_word(y));
    const double C = from_words(big ? (0x3ff00000u ^ sx) : 0x80000000u, 0u);
    *ib_out = ib;
    return C + div_rn_safe(num, y + 2.0);
}

// Table form of the per-class constants above.  They depend on k alone, and
// the common path only reaches k in [-3, 63] (u in (-2, 0] or [2, 44)), so a
// 67-entry table indexed by k + 3 holds X3, X4 and B, and also s_tanh.c's
// tail constant C: |x| >= 1 exactly when k > 0 (u >= 2 gives k >= 3, u in
// (-2, 0] gives k in [-3, 0]).  All four are whole doubles (16-byte LDS reads
// land them in register pairs: no assembly of hi words over a zero low word);
// the exponent addend k << 20 is one shift-add on the hi word.  Same
// constants, same IEEE operations as tanh_half_common.
// An entry is a 16-byte A part (X3, X4) and a 16-byte B part (B, C);
// Expm1Tab::step is the entry stride in 16-byte units (2: A and B interleaved,
// 32-byte entries — the decoder's layout; 1: two separate arrays).
struct alignas(16) Expm1A {
    double x3, x4;
};
struct alignas(16) Expm1B {
    double b, c;
};
// The word form of the B part (W = true below): B and C as high words and the
// exponent addend k << 20 stored, not shifted — the form the split-frame SPA
// instantiation runs faster with (fewer live registers there).
struct alignas(16) Expm1Bw {
    uint32_t b_hi, c_hi, k20, pad;
};
struct Expm1Tab {
    const Expm1A *a;
    const Expm1B *b;
    int step;  // entry stride in 16-byte units (1: two arrays)
};
constexpr int EXPM1_K_MIN = -3, EXPM1_K_MAX = 63, EXPM1_CLASSES = EXPM1_K_MAX - EXPM1_K_MIN + 1;
template <bool W = false>
QL_HD void expm1_class(int32_t k, Expm1A *ea, Expm1B *eb) {
    const uint32_t ku = (uint32_t)k;
    const bool fcls = (ku - 20u) <= 36u;
    const bool far = (ku + 1u) > 57u;
    const bool big = k > 0;
    uint32_t a_hi = 0x3ff00000u - (0x200000u >> (ku & 31u));
    a_hi = (k == 0) ? 0x80000000u : a_hi;
    a_hi = (k == -1) ? 0xbff00000u : a_hi;
    ea->x3 = from_words(fcls ? (0x3ff00000u - (ku << 20)) : 0x80000000u, 0u);
    ea->x4 = from_words(fcls ? 0x3ff00000u : a_hi, 0u);
    if constexpr (W) {
        Expm1Bw *ew = reinterpret_cast<Expm1Bw *>(eb);
        ew->b_hi = far ? 0xbff00000u : 0x80000000u;
        ew->c_hi = big ? 0x3ff00000u : 0x80000000u;
        ew->k20 = ku << 20;
        ew->pad = 0;
    } else {
        eb->b = from_words(far ? 0xbff00000u : 0x80000000u, 0u);
        eb->c = from_words(big ? 0x3ff00000u : 0x80000000u, 0u);
    }
}

// tanh_half_common with the class constants from `tab` (EXPM1_CLASSES
// entries, entry i = expm1_class(i + EXPM1_K_MIN)).  Lanes outside the common
// path (the callers' rare branch recomputes them) read a clamped entry.
// k: s_expm1.c's explicit k = -1 for 0.5 ln2 < |u| < 1.5 ln2 (hi-word tests)
// is what the rounded formula gives there anyway — only u < 0 reaches that
// range, where invln2 * u - 0.5 lies in [-1.99999997, -1.00000001] — so only
// the k = 0 test (|u| <= 0.5 ln2 by hi word) remains.  The result's sign:
// the magnitude C + num / (y + 2) is > 0 on this path, so copysign by b.
// W: the table's B parts are in the word form (expm1_class<true>), and u is
// the select of +-|b| — the same IEEE operations either way.
template <bool W = false>
QL_HD double tanh_half_common_t(double b, uint32_t *ib_out, Expm1Tab tab) {
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double invln2 = 1.44269504088896338700e+00;
    const double Q1 = -3.33333333333331316428e-02, Q2 = 1.58730158725481460165e-03;
    const double Q3 = -7.93650757867487942473e-05, Q4 = 4.00821782732936239552e-06;
    const double Q5 = -2.01099218183624371326e-07;

    const uint32_t jb = hi_word(b);
    const uint32_t ib = jb & 0x7fffffffu;
    const bool big = ib >= 0x40000000u;
    // u = +-|b| as |b| * (+-1): exact, one select and one multiply (the
    // sign-word form the compiler would make of it needs an or, a select and
    // a copy of the low word; |b| is the multiply's abs source modifier)
#if defined(__HIP_DEVICE_COMPILE__)
    double u;
    if constexpr (W) u = big ? __builtin_fabs(b) : -__builtin_fabs(b);
    else asm("v_mul_f64 %0, |%1|, %2" : "=v"(u) : "v"(b), "v"(big ? 1.0 : -1.0));
#else
    const double u = big ? __builtin_fabs(b) : -__builtin_fabs(b);
#endif
    double kf = invln2 * u + (big ? 0.5 : -0.5);
#if !defined(__HIP_DEVICE_COMPILE__)
    kf = (kf > 1e6 || kf < -1e6 || kf != kf) ? 0.0 : kf;
#endif
    int32_t k = (int32_t)kf;
    k = (ib > 0x3fd62e42u) ? k : 0;
    const int32_t kc = k < EXPM1_K_MIN ? EXPM1_K_MIN : (k > EXPM1_K_MAX ? EXPM1_K_MAX : k);
    const Expm1A ca = tab.a[(kc - EXPM1_K_MIN) * tab.step];  // issued early, used after the division
    const Expm1B cb = tab.b[(kc - EXPM1_K_MIN) * tab.step];
    const Expm1Bw cw = reinterpret_cast<const Expm1Bw *>(tab.b)[(kc - EXPM1_K_MIN) * tab.step];
    const double t = (double)k;
    const double hi = __builtin_fma(-t, ln2_hi, u);  // == u - t * ln2_hi: t * ln2_hi is exact (ln2_hi has 32 bits, |k| < 2^11)
    const double lo = t * ln2_lo;
    const double xr = hi - lo;
    const double c = (hi - xr) - lo;
    const double hfx = 0.5 * xr;
    const double hxs = xr * hfx;
    const double R1 = 1.0 + hxs * Q1;
    const double h2 = hxs * hxs;
    const double R2 = Q2 + hxs * Q3;
    const double h4 = h2 * h2;
    const double R3 = Q4 + hxs * Q5;
    const double r1 = R1 + h2 * R2 + h4 * R3;
    const double t3 = 3.0 - r1 * hfx;
    const double e = hxs * div_rn_safe(r1 - t3, 6.0 - xr * t3);
    const double e2 = (xr * (e - c) - c) - hxs;
    const double ypre = (xr - (e2 + ca.x3)) + ca.x4;
    // s_tanh.c evaluates |x| and negates last: z = +-(C + num / (y + 2)) with
    // C = 1, num = -2 (|x| >= 1) or C = -0, num = -y; the sign goes on at the
    // end (round-to-nearest is symmetric; the sum is never 0 on this path).
    const double y = W ? with_hi_word(ypre, hi_word(ypre) + cw.k20) + from_words(cw.b_hi, 0u)
                       : with_hi_word(ypre, hi_word(ypre) + ((uint32_t)kc << 20)) + cb.b;
    const double num = big ? from_words(0xc0000000u, 0u) : from_words(hi_word(y) ^ 0x80000000u, lo_word(y));
    const double zp = (W ? from_words(cw.c_hi, 0u) : cb.c) + div_rn_safe(num, y + 2.0);
    *ib_out = ib;
    return __builtin_copysign(zp, b);
}

QL_HD double tanh_half_dec(double b) {
    uint32_t ib;
    double z = tanh_half_common(b, &ib);
    const bool special = (ib - 0x3c900000u) >= (0x40460000u - 0x3c900000u);  // tiny, |x| >= 22, inf, NaN
    QL_RARE(special) z = tanh_half_full(b);
    return z;
}

// The reference's threshold_matrix on one value (src/array_and_matrix_operations.cpp:962-969):
// |v| > thr -> +-thr, NaN passes; thr = +inf disables it.
QL_HD double clip_thr(double v, double thr) { return (__builtin_fabs(v) > thr) ? __builtin_copysign(thr, v) : v; }

// tanh(clip_thr(b, thr) / 2.) with lim = min(thr, 44) and t_lim = glibc
// tanh(lim / 2.) (host-computed; 1 for lim = 44).  For |b| >= lim the result is
// +-t_lim clipped or not (|b| > thr clips to +-thr, and tanh(+-x) = +-1 for
// |x| >= 22), so the clip only matters on lanes the rare branch takes; its body
// is the three cases glibc's s_tanh.c returns early on, inline:
//   |x| < 2^-55: x*(1+x);  NaN: x+x;  else +-t_lim.   (x = b / 2.)
// *tiny_or_nan is set (never cleared) when the result is NaN or below 2^-55
// in magnitude: the only results outside [2^-55, 1] (see div_rn_safe's range).
QL_HD double tanh_half_clip(double b, double lim, double t_lim, int *tiny_or_nan) {
    uint32_t ib;
    double z = tanh_half_common(b, &ib);
    const bool special = (ib < 0x3c900000u) || !(__builtin_fabs(b) < lim);  // tiny, |b| >= lim, NaN
    QL_RARE(special) {
        const double x = b / 2.;
        z = (ib < 0x3c900000u) ? x * (1.0 + x) : __builtin_copysign(t_lim, b);
        z = (b != b) ? x + x : z;
        if (ib < 0x3c900000u || b != b) *tiny_or_nan = 1;
    }
    return z;
}

// tanh_half_clip on tanh_half_common_t (the table form).
template <bool W = false>
QL_HD double tanh_half_clip_t(double b, double lim, double t_lim, int *tiny_or_nan, Expm1Tab tab) {
    uint32_t ib;
    double z = tanh_half_common_t<W>(b, &ib, tab);
    const bool special = (ib < 0x3c900000u) || !(__builtin_fabs(b) < lim);
    QL_RARE(special) {
        const double x = b / 2.;
        z = (ib < 0x3c900000u) ? x * (1.0 + x) : __builtin_copysign(t_lim, b);
        z = (b != b) ? x + x : z;
        if (ib < 0x3c900000u || b != b) *tiny_or_nan = 1;
    }
    return z;
}

// 2 * atanh(p) bit-identical to 2. * glibc atanh.  Common path:
// 2^-28 <= |p| < 1 - 2^-21 (log1p argument a in [2^-27, 2^22): finite, u0 = 1 + a).
QL_HD double atanh2_full(double p) { return 2. * atanh_dec(p); }

// Common path of 2. * atanh(p); *ia = hi word of |p|.  Exact for
// 2^-28 <= |p| < 1 - 2^-21; other lanes get a don't-care value.
QL_HD double atanh2_common(double p, uint32_t *ia_out) {
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01;
    const double Lp3 = 2.857142874366239149e-01, Lp4 = 2.222219843214978396e-01;
    const double Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01;
    const double Lp7 = 1.479819860511658591e-01;

    const double xa = __builtin_fabs(p);
    const uint32_t ia = hi_word(xa);
    const bool smallx = xa < 0.5;                  // (e_atanh.c: hi word < 0x3fe00000)
    const double twoxa = xa + xa;
    const double qd = div_rn_safe(smallx ? twoxa * xa : twoxa, 1.0 - xa);
    const double a = smallx ? twoxa + qd : qd;
    // --- log1p(a) core, a in [2^-27, 2^22) ---
    const bool k0 = hi_word(a) < 0x3FDA827Au;      // a < 0.41422: f = a, k = 0, c = 0
    const double u0 = 1.0 + a;
    const int32_t hu = (int32_t)hi_word(u0);
    // c = the rounding error of 1 + a, divided by u0.  s_log1p.c forms it as
    // 1 - (u0 - a) when u0 >= 2 and a - (u0 - 1) otherwise; on a in [2^-27,
    // 2^22) both differences of each form are exact (Sterbenz; u0 - 1 is a
    // multiple of ulp(u0) below 2^53), so both forms are the same exact
    // value and one of them serves every lane.
    double c = div_rn_safe(a - (u0 - 1.0), u0);
    const uint32_t hm = (uint32_t)hu & 0x000fffffu;
    // k0 lanes keep k = 0: u0 = 1 + a is in [1, 2) there, so (hu >> 20) - 1023
    // is 0 and only `up` (possible for a just below 0.41422) must be masked off
    const bool up = !k0 && hm >= 0x6a09eu;
    const int32_t nk = 1023 - (hu >> 20) - (int32_t)up;  // -k
    // u = u0 with its exponent replaced (SET_HIGH_WORD) = u0 * 2^-k exactly
    double f = __builtin_ldexp(u0, nk) - 1.0;
    f = k0 ? a : f;
    c = k0 ? 0.0 : c;
    const double hfsq = 0.5 * f * f;
    const double ndk = (double)nk;  // -k: the k products below by negation (RN is symmetric)
    const double s = div_rn_safe(f, 2.0 + f);
    const double z = s * s;
    const double R1 = z * Lp1;
    const double z2 = z * z;
    const double R2 = Lp2 + z * Lp3;
    const double z4 = z2 * z2;
    const double R3 = Lp4 + z * Lp5;
    const double z6 = z4 * z2;
    const double R4 = Lp6 + z * Lp7;
    const double R = R1 + z2 * R2 + z4 * R3 + z6 * R4;
    // k == 0 through the k != 0 formula (dk = c = 0): see atanh_dec.
    // dk * ln2_hi == -(ndk * ln2_hi) and dk * ln2_lo + c == c - ndk * ln2_lo
    // bitwise; k == 0 only on k0 lanes, where the sum is never 0, so the
    // -0 of -(0 * ln2_hi) cannot surface.
    double y = __builtin_fma(-ndk, ln2_hi, -((hfsq - (s * (hfsq + R) + (c - ndk * ln2_lo))) - f));  // ndk * ln2_hi is exact
    // s_log1p.c's |f| < 2^-20 case is hu == 0 with hu = k0 ? 1 : (up ? (0x100000 -
    // hm) >> 2 : hm), i.e. !k0 && (hm == 0 || hm >= 0xffffd): one test on hm
    // admits exactly those four values (k0 lanes included), the exact
    // condition is applied inside.
    QL_RARE((((uint32_t)hu + 3u) << 12) < 0x4000u) {  // ((hm + 3) mod 2^20) < 4
        const uint32_t hu2 = k0 ? 1u : (up ? (0x00100000u - hm) >> 2 : hm);
        const int32_t k = -nk;
        const double dk = (double)k;
        if (hu2 == 0) {                            // |f| < 2^-20
            const double Rs = hfsq * (1.0 - 0.66666666666666666 * f);
            const double ysmall = (k == 0) ? f - Rs : dk * ln2_hi - ((Rs - (dk * ln2_lo + c)) - f);
            const double yzero = (k == 0) ? 0.0 : dk * ln2_hi + (c + dk * ln2_lo);
            y = (f == 0.0) ? yzero : ysmall;
        }
    }
    *ia_out = ia;
    return __builtin_copysign(y, p);               // 2 * copysign(0.5 * y, p)
}

QL_HD double atanh2_dec(double p) {
    uint32_t ia;
    double r = atanh2_common(p, &ia);
    const bool special = (ia - 0x3e300000u) >= (0x3fefffffu - 0x3e300000u);  // tiny, >= 1 - 2^-21, NaN
    QL_RARE(special) r = atanh2_full(p);
    return r;
}

// clip_thr(2. * atanh(p), thr).  atanh2_common is exact for 2^-28 <= |p| <
// 1 - 2^-53 (the log1p argument stays below 2^53); its result is below 37.5 in
// magnitude and never NaN, so its clip is one compare.  The rare branch holds
// e_atanh.c's early returns and the one value left, |p| = 1 - 2^-53, whose
// 2*atanh is the constant c_top (host-computed by glibc):
//   |p| < 2^-28: 2*p;  |p| = 1: +-inf;  |p| > 1 or NaN: NaN.
QL_HD double atanh2_clip(double p, double thr, double c_top) {
    uint32_t ia;
    double r = atanh2_common(p, &ia);
    const double xa = __builtin_fabs(p);
    // (tests on |p| itself: the hi-word test ia < 0x3e300000 is |p| < 2^-28)
    const bool tiny = xa < 0x1p-28;
    const bool special = tiny || !(xa < 0x1.fffffffffffffp-1);  // tiny, >= 1 - 2^-53, NaN
    QL_RARE(special || __builtin_fabs(r) > thr) {
        double v = (xa == 1.0) ? __builtin_copysign(__builtin_inf(), p) : __builtin_copysign(c_top, p);
        v = tiny ? 2. * p : v;
        v = (xa > 1.0 || p != p) ? 2. * ((p - p) / (p - p)) : v;
        r = clip_thr(special ? v : r, thr);
    }
    return r;
}

}  // namespace ql_exact

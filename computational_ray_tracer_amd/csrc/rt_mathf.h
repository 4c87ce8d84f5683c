// Float-result transcendentals of the wavelength warps (Sampling.h:63-71), evaluated in double and rounded to float
// exactly as the oracle does ((float)std::atanh((double)x), (float)std::cosh((double)x); oracle/rtcore.hpp:68-69),
// but ~4x cheaper than the full-precision double library calls.
//
// The fast path is an fdlibm-style double evaluation (error a few double ulps, ~1e-16 relative).  Its float rounding
// is the correctly rounded float of the true value unless the double result lies within 2^-46 (relative) of a float
// rounding midpoint; that case is detected (the result is perturbed by +-2^-46 and must round to the same float both
// ways) and takes the full-precision library call instead.  So the returned float equals the float rounding of any
// double evaluation accurate to better than 2^-46 -- glibc's on the oracle side, ocml's on the device.
// tools/verify_warps.cpp checks every float input of the warps' domains against glibc exhaustively.
//
// Plain C++ (host) or HIP (device): no HIP types, explicit fma, no contraction (-ffp-contract=off on both sides).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define RTM_FN __host__ __device__ inline
#else
#define RTM_FN inline
#endif

namespace rtm {

RTM_FN uint64_t d2u(double d) { return __builtin_bit_cast(uint64_t, d); }
RTM_FN double u2d(uint64_t u) { return __builtin_bit_cast(double, u); }

// log(u) for u > 0 finite normal (fdlibm e_log.c kernel: u = 2^k m, m in [sqrt(2)/2, sqrt(2)), s = f / (2 + f),
// log(m) = f - (f^2/2 - s (f^2/2 + R(s^2))); error < 1 ulp)
RTM_FN double log_pos(double u) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                 Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    uint64_t b = d2u(u);
    int32_t hx = (int32_t)(b >> 32);
    int32_t k = (hx >> 20) - 1023;
    hx &= 0x000fffff;
    int32_t i = (hx + 0x95f64) & 0x100000;
    double m = u2d(((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (b & 0xffffffffull));
    k += (i >> 20);
    double f = m - 1.0;
    double s = f / (2.0 + f);
    double z = s * s;
    double w = z * z;
    double t1 = w * __builtin_fma(w, __builtin_fma(w, Lg6, Lg4), Lg2);
    double t2 = z * __builtin_fma(w, __builtin_fma(w, __builtin_fma(w, Lg7, Lg5), Lg3), Lg1);
    double R = t2 + t1;
    double hfsq = 0.5 * f * f;
    double dk = (double)k;
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

// exp(r) for |r| <= ~2.3 (k = rint(r / ln2) in [-4, 4]; Cody-Waite reduction, degree-13 Taylor on |t| <= ln2/2)
RTM_FN double exp_small(double r) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const double inv_ln2 = 1.44269504088896338700e+00;
    double kd = __builtin_rint(r * inv_ln2);
    double t = __builtin_fma(-kd, ln2_lo, __builtin_fma(-kd, ln2_hi, r));  // k ln2_hi is exact (32-bit ln2_hi)
    double p = 1.0 / 6227020800.0;                                          // 1/13!
    p = __builtin_fma(p, t, 1.0 / 479001600.0);
    p = __builtin_fma(p, t, 1.0 / 39916800.0);
    p = __builtin_fma(p, t, 1.0 / 3628800.0);
    p = __builtin_fma(p, t, 1.0 / 362880.0);
    p = __builtin_fma(p, t, 1.0 / 40320.0);
    p = __builtin_fma(p, t, 1.0 / 5040.0);
    p = __builtin_fma(p, t, 1.0 / 720.0);
    p = __builtin_fma(p, t, 1.0 / 120.0);
    p = __builtin_fma(p, t, 1.0 / 24.0);
    p = __builtin_fma(p, t, 1.0 / 6.0);
    p = __builtin_fma(p, t, 0.5);
    p = __builtin_fma(p, t, 1.0);
    p = __builtin_fma(p, t, 1.0);
    int32_t k = (int32_t)kd;
    return p * u2d((uint64_t)(int64_t)(1023 + k) << 52);  // exact scaling by 2^k
}

// true when a midpoint between two floats lies within 2^-46 |r| of r (the float rounding is then not certain)
RTM_FN bool near_midpoint(double r, float f) {
    const double e = 1.4210854715202004e-14;  // 2^-46
    return (float)(r * (1.0 + e)) != f || (float)(r * (1.0 - e)) != f;
}

// x in (-1, 1): atanh(x) = (log(1 + x) - log(1 - x)) / 2, where 1 +- x is exact in double for a float |x| >= 2^-29;
// below 2^-20 the series x + x^3/3 (next term x^5/5: relative 2^-40 of x^3/3, far below double rounding)
RTM_FN double atanh_fast(float x) {
    double xd = (double)x;
    double a = 1.0 + xd, b = 1.0 - xd;
    double r = 0.5 * (log_pos(a) - log_pos(b));
    double ax = xd < 0 ? -xd : xd;
    return ax < 9.5367431640625e-07 ? xd + xd * xd * xd * 0.33333333333333331 : r;  // 2^-20
}
// |z| <= ~2.3: cosh(z) = (e^|z| + 1 / e^|z|) / 2
RTM_FN double cosh_fast(float z) {
    double az = z < 0 ? -(double)z : (double)z;
    double E = exp_small(az);
    return 0.5 * (E + 1.0 / E);
}

}  // namespace rtm

/*
 * portable_math.h -- TEST INFRASTRUCTURE (oracle side).
 *
 * Portable powf / expf evaluated in double with only IEEE + - * / and exact bit manipulation, no FMA, so the
 * CPU oracle and the device kernels (romis_amd/csrc/device_math.h carries the same algorithm in HIP) produce
 * identical bits.  They replace glibc's powf (shading.cpp:26 std::pow, tone_mapping.cpp:10 glm::pow) and expf
 * (tone_mapping.cpp:9 glm::exp).  Accuracy: about 1e-14 relative before the final rounding to float, i.e.
 * correctly rounded except within ~1e-14 of a rounding boundary; tests/test_oracle_pinning.py checks them
 * against the glibc results the reference's own tone_mapping.cpp produced.
 */
#ifndef ROMIS_ORACLE_PORTABLE_MATH_H
#define ROMIS_ORACLE_PORTABLE_MATH_H

#include <math.h>
#include <stdint.h>
#include <string.h>

static inline uint64_t pm_bits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
static inline double   pm_from(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
static inline uint32_t pm_fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* 2^n for integer n in [-1022, 1023] */
static inline double pm_ldexp1(int n) { return pm_from((uint64_t)(n + 1023) << 52); }

/* natural log of a positive finite normal double */
static inline double pm_log_d(double a) {
    uint64_t b = pm_bits(a);
    int e = (int)((b >> 52) & 0x7FF) - 1023;
    double m = pm_from((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull); /* [1, 2) */
    if (m > 1.4142135623730951) { m = m * 0.5; e = e + 1; }
    double s = (m - 1.0) / (m + 1.0);
    double s2 = s * s;
    /* atanh series: ln m = 2 s (1 + s2/3 + s2^2/5 + ... ) */
    double p = 1.0 / 23.0;
    p = 1.0 / 21.0 + s2 * p;
    p = 1.0 / 19.0 + s2 * p;
    p = 1.0 / 17.0 + s2 * p;
    p = 1.0 / 15.0 + s2 * p;
    p = 1.0 / 13.0 + s2 * p;
    p = 1.0 / 11.0 + s2 * p;
    p = 1.0 / 9.0 + s2 * p;
    p = 1.0 / 7.0 + s2 * p;
    p = 1.0 / 5.0 + s2 * p;
    p = 1.0 / 3.0 + s2 * p;
    double lnm = (2.0 * s) + (2.0 * s) * (s2 * p);
    return (double)e * 0.69314718055994530942 + lnm;
}

/* e^z for z in about [-745, 709]; callers clamp */
static inline double pm_exp_d(double z) {
    double kf = floor(z * 1.4426950408889634074 + 0.5);
    int k = (int)kf;
    /* r = z - k ln2 with ln2 split so k*LN2_HI is exact for |k| < 2^11 */
    double r = (z - kf * 0.693147180369123816490) - kf * 1.90821492927058770002e-10;
    double p = 1.0 / 6227020800.0;              /* 1/13! */
    p = 1.0 / 479001600.0 + r * p;              /* 1/12! */
    p = 1.0 / 39916800.0 + r * p;
    p = 1.0 / 3628800.0 + r * p;
    p = 1.0 / 362880.0 + r * p;
    p = 1.0 / 40320.0 + r * p;
    p = 1.0 / 5040.0 + r * p;
    p = 1.0 / 720.0 + r * p;
    p = 1.0 / 120.0 + r * p;
    p = 1.0 / 24.0 + r * p;
    p = 1.0 / 6.0 + r * p;
    p = 0.5 + r * p;
    p = 1.0 + r * p;
    p = 1.0 + r * p;
    /* scale by 2^k in two steps so subnormal float results stay representable */
    int k1 = k / 2, k2 = k - k / 2;
    return (p * pm_ldexp1(k1)) * pm_ldexp1(k2);
}

static inline int pm_is_int(float y) { return y == truncf(y); }
static inline int pm_is_odd_int(float y) {
    if (!pm_is_int(y) || fabsf(y) >= 16777216.0f) return 0;
    long long i = (long long)y;
    return (int)(i & 1);
}

/* powf with C99 Annex F special cases. */
static inline float pm_powf(float x, float y) {
    if (y == 0.0f) return 1.0f;
    if (x == 1.0f) return 1.0f;
    if (isnan(x) || isnan(y)) return x + y;
    int yint = pm_is_int(y), yodd = pm_is_odd_int(y);
    if (x == 0.0f) {
        if (y < 0.0f) return yodd ? copysignf(INFINITY, x) : INFINITY;
        return yodd ? x : 0.0f;
    }
    if (isinf(y)) {
        float ax = fabsf(x);
        if (ax == 1.0f) return 1.0f;
        return ((ax < 1.0f) == (y < 0.0f)) ? INFINITY : 0.0f;
    }
    if (isinf(x)) {
        if (x > 0.0f) return y < 0.0f ? 0.0f : INFINITY;
        if (yodd) return y < 0.0f ? -0.0f : -INFINITY;
        return y < 0.0f ? 0.0f : INFINITY;
    }
    if (x < 0.0f && !yint) return NAN;
    double sign = (x < 0.0f && yodd) ? -1.0 : 1.0;
    double ax = fabs((double)x);
    double r;
    if (yint && fabsf(y) <= 1048576.0f) {
        /* integer exponent: binary powering in double */
        uint32_t n = (uint32_t)fabsf(y);
        double base = ax, acc = 1.0;
        while (n) {
            if (n & 1u) acc = acc * base;
            n >>= 1;
            if (n) base = base * base;
        }
        r = (y < 0.0f) ? 1.0 / acc : acc;
    } else {
        double z = (double)y * pm_log_d(ax);
        if (z > 89.0) r = INFINITY;
        else if (z < -104.0) r = 0.0;
        else r = pm_exp_d(z);
    }
    return (float)(sign * r);
}

static inline float pm_expf(float x) {
    if (isnan(x)) return x;
    if (x > 89.0f) return INFINITY;
    if (x < -104.0f) return 0.0f;
    return (float)pm_exp_d((double)x);
}

#endif

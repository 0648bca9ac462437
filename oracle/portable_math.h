/*
 * portable_math.h -- TEST INFRASTRUCTURE (oracle side).
 *
 * powf / expf restated bit for bit from glibc 2.35's flt-32 implementations, the ones the reference's
 * std::pow(float, float) (shading.cpp:26, glm::pow at tone_mapping.cpp:10) and glm::exp (tone_mapping.cpp:9)
 * resolve to on x86-64 Linux.  glibc selects its FMA variants (sysdeps/x86_64/fpu/multiarch/e_powf.c,
 * e_expf.c: __powf_fma / __expf_fma, chosen by the ifunc whenever the CPU has FMA + AVX2) -- the same C code
 * (sysdeps/ieee754/flt-32/e_powf.c, e_expf.c) compiled with contraction, so every a*b+c of the source is one
 * fused multiply-add.  The restatement below spells those fma() calls out where the FMA objects have them
 * (read off this image's libm.so.6: llvm-objdump of the ifunc targets), so the result does not depend on the
 * compiler's contraction choices.  Tables and coefficients are glibc's published constants
 * (__powf_log2_data: POWF_LOG2_TABLE_BITS = 4, POWF_LOG2_POLY_ORDER = 5; __exp2f_data: EXP2F_TABLE_BITS = 5).
 *
 * romis_amd/csrc/device_math.h evaluates the same operation sequence on the GPU (v_fma_f64 is the same fused
 * operation as vfmadd*sd); oracle/check_libm.c compares this header with the image's libm over every
 * non-negative float base for the exponents the scenes use and over every float for expf.
 */
#ifndef ROMIS_ORACLE_PORTABLE_MATH_H
#define ROMIS_ORACLE_PORTABLE_MATH_H

#include <math.h>
#include <stdint.h>
#include <string.h>

static inline uint64_t pm_bits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
static inline double   pm_from(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
static inline uint32_t pm_fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float    pm_ffrom(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* __powf_log2_data.tab: {invc, logc} */
static const double PM_LOG2_TAB[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.efec65b963019p-2}, {0x1.571ed4aaf883dp+0, -0x1.b0b6832d4fca4p-2},
    {0x1.49539f0f010bp+0, -0x1.7418b0a1fb77bp-2},  {0x1.3c995b0b80385p+0, -0x1.39de91a6dcf7bp-2},
    {0x1.30d190c8864a5p+0, -0x1.01d9bf3f2b631p-2}, {0x1.25e227b0b8eap+0, -0x1.97c1d1b3b7afp-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.2f9e393af3c9fp-3}, {0x1.12358f08ae5bap+0, -0x1.960cbbf788d5cp-4},
    {0x1.0953f419900a7p+0, -0x1.a6f9db6475fcep-5}, {0x1p+0, 0x0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.338ca9f24f53dp-4},  {0x1.ca4b31f026aap-1, 0x1.476a9543891bap-3},
    {0x1.b2036576afce6p-1, 0x1.e840b4ac4e4d2p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.40645f0c6651cp-2},
    {0x1.886e6037841edp-1, 0x1.88e9c2c1b9ff8p-2},  {0x1.767dcf5534862p-1, 0x1.ce0a44eb17bccp-2},
};
/* __powf_log2_data.poly */
#define PM_LA0 0x1.27616c9496e0bp-2
#define PM_LA1 (-0x1.71969a075c67ap-2)
#define PM_LA2 0x1.ec70a6ca7baddp-2
#define PM_LA3 (-0x1.7154748bef6c8p-1)
#define PM_LA4 0x1.71547652ab82bp+0

/* __exp2f_data.tab: asuint64(2^(i/32)) - (i << 47) */
static const uint64_t PM_EXP2_TAB[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull,
};
/* __exp2f_data: poly (exp2 of r in [-1/64, 1/64]), shift_scaled, and expf's scaled forms */
#define PM_E2C0 0x1.c6af84b912394p-5
#define PM_E2C1 0x1.ebfce50fac4f3p-3
#define PM_E2C2 0x1.62e42ff0c52d6p-1
#define PM_E2SHIFT 0x1.8p+47
#define PM_EXC0 0x1.c6af84b912394p-20
#define PM_EXC1 0x1.ebfce50fac4f3p-13
#define PM_EXC2 0x1.62e42ff0c52d6p-6
#define PM_EXSHIFT 0x1.8p+52
#define PM_INVLN2N 0x1.71547652b82fep+5

#define PM_SIGN_BIAS 0x10000u   /* 1 << (EXP2F_TABLE_BITS + 11) */

/* math_err.c: xflowf(sign, y) = (sign ? -y : y) * y */
static inline float pm_xflowf(uint32_t sign, float y) { volatile float a = sign ? -y : y; return a * y; }

/* e_powf.c checkint: 0 not an integer, 1 odd, 2 even */
static inline int pm_checkint(uint32_t iy) {
    int e = (int)(iy >> 23 & 0xff);
    if (e < 0x7f) return 0;
    if (e > 0x7f + 23) return 2;
    if (iy & ((1u << (0x7f + 23 - e)) - 1)) return 0;
    if (iy & (1u << (0x7f + 23 - e))) return 1;
    return 2;
}
static inline int pm_zeroinfnan(uint32_t i) { return 2 * i - 1 >= 2u * 0x7f800000 - 1; }
/* issignalingf_inline: 2 * (ix ^ 0x00400000) > 2 * 0x7fc00000 */
static inline int pm_issignaling(uint32_t i) { return 2 * (i ^ 0x00400000u) > 2u * 0x7fc00000u; }

/* the quiet NaN x86 SSE arithmetic returns for x + y: the first NaN operand, quieted */
static inline float pm_nan_add(float x, float y) {
    uint32_t ix = pm_fbits(x), iy = pm_fbits(y);
    if ((ix & 0x7fffffffu) > 0x7f800000u) return pm_ffrom(ix | 0x00400000u);
    if ((iy & 0x7fffffffu) > 0x7f800000u) return pm_ffrom(iy | 0x00400000u);
    return x + y;
}

/* log2_inline (e_powf.c), FMA object: r = fma(z, invc, -1); y = fma(r, A0, A1); p = fma(r, A2, A3);
 * q = fma(r, A4, k + logc); q = fma(r2, p, q); y = fma(y, r4, q) */
static inline double pm_log2_inline(uint32_t ix) {
    uint32_t tmp = ix - 0x3f330000u;
    int i = (int)((tmp >> 19) % 16);
    uint32_t top = tmp & 0xff800000u;
    uint32_t iz = ix - top;
    int k = (int32_t)top >> 23;
    double invc = PM_LOG2_TAB[i][0], logc = PM_LOG2_TAB[i][1];
    double z = (double)pm_ffrom(iz);
    double r = fma(z, invc, -1.0);
    double y0 = logc + (double)k;
    double r2 = r * r;
    double y = fma(r, PM_LA0, PM_LA1);
    double p = fma(r, PM_LA2, PM_LA3);
    double r4 = r2 * r2;
    double q = fma(r, PM_LA4, y0);
    q = fma(r2, p, q);
    return fma(y, r4, q);
}

/* exp2_inline (e_powf.c), FMA object */
static inline double pm_exp2_inline(double xd, uint32_t sign_bias) {
    double kd = xd + PM_E2SHIFT;
    uint64_t ki = pm_bits(kd);
    kd -= PM_E2SHIFT;
    double r = xd - kd;
    uint64_t t = PM_EXP2_TAB[ki % 32];
    uint64_t ski = ki + sign_bias;
    t += ski << 47;
    double s = pm_from(t);
    double z = fma(r, PM_E2C0, PM_E2C1);
    double r2 = r * r;
    double y = fma(r, PM_E2C2, 1.0);
    y = fma(z, r2, y);
    return y * s;
}

/* __powf (sysdeps/ieee754/flt-32/e_powf.c, glibc 2.35) */
static inline float pm_powf(float x, float y) {
    uint32_t sign_bias = 0;
    uint32_t ix = pm_fbits(x), iy = pm_fbits(y);
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u || pm_zeroinfnan(iy)) {
        if (pm_zeroinfnan(iy)) {
            if (2 * iy == 0) return pm_issignaling(ix) ? pm_nan_add(x, y) : 1.0f;
            if (ix == 0x3f800000u) return pm_issignaling(iy) ? pm_nan_add(x, y) : 1.0f;
            if (2 * ix > 2u * 0x7f800000u || 2 * iy > 2u * 0x7f800000u) return pm_nan_add(x, y);
            if (2 * ix == 2u * 0x3f800000u) return 1.0f;
            if ((2 * ix < 2u * 0x3f800000u) == !(iy & 0x80000000u)) return 0.0f;
            return y * y;
        }
        if (pm_zeroinfnan(ix)) {
            float x2 = x * x;
            if ((ix & 0x80000000u) && pm_checkint(iy) == 1) x2 = -x2;
            return (iy & 0x80000000u) ? 1.0f / x2 : x2;
        }
        if (ix & 0x80000000u) {
            int yint = pm_checkint(iy);
            if (yint == 0) return pm_ffrom(0xffc00000u);     /* __math_invalidf: (x - x) / (x - x) on x86 */
            if (yint == 1) sign_bias = PM_SIGN_BIAS;
            ix &= 0x7fffffffu;
        }
        if (ix < 0x00800000u) {
            ix = pm_fbits(pm_ffrom(ix) * 0x1p23f);
            ix &= 0x7fffffffu;
            ix -= 23u << 23;
        }
    }
    double logx = pm_log2_inline(ix);
    double ylogx = (double)y * logx;
    if (((pm_bits(ylogx) >> 47) & 0xffff) >= (pm_bits(126.0) >> 47)) {
        if (ylogx > 0x1.fffffffd1d571p+6) return pm_xflowf(sign_bias, 0x1p97f);     /* __math_oflowf */
        /* (0x1.fffffffa3aae2p+6, ...]: overflow only when rounding away from zero; round-to-nearest here */
        if (ylogx <= -150.0) return pm_xflowf(sign_bias, 0x1p-95f);                 /* __math_uflowf */
        if (ylogx < -149.0) return pm_xflowf(sign_bias, 0x1.4p-75f);                /* __math_may_uflowf */
    }
    return (float)pm_exp2_inline(ylogx, sign_bias);
}

/* __expf (sysdeps/ieee754/flt-32/e_expf.c, glibc 2.35), FMA object: kd = fma(InvLn2N, x, SHIFT);
 * r = fma(InvLn2N, x, -kd) */
static inline float pm_expf(float x) {
    uint32_t ux = pm_fbits(x);
    double xd = (double)x;
    uint32_t abstop = (ux >> 20) & 0x7ff;
    if (abstop >= 0x42a) {                                    /* top12(88.0f) */
        if (ux == 0xff800000u) return 0.0f;
        if (abstop >= 0x7f8) return pm_nan_add(x, x);
        if (x > 0x1.62e42ep6f) return pm_xflowf(0, 0x1p97f);
        if (x < -0x1.9fe368p6f) return pm_xflowf(0, 0x1p-95f);
        if (x < -0x1.9d1d9ep6f) return pm_xflowf(0, 0x1.4p-75f);
    }
    double kd = fma(PM_INVLN2N, xd, PM_EXSHIFT);
    uint64_t ki = pm_bits(kd);
    kd -= PM_EXSHIFT;
    double r = fma(PM_INVLN2N, xd, -kd);
    uint64_t t = PM_EXP2_TAB[ki % 32];
    t += ki << 47;
    double s = pm_from(t);
    double z = fma(r, PM_EXC0, PM_EXC1);
    double r2 = r * r;
    double y = fma(r, PM_EXC2, 1.0);
    y = fma(z, r2, y);
    return (float)(y * s);
}

#endif

// device_math.h -- gfx950 device arithmetic of the ReSTIR path.
//
// Every function reproduces the reference's float operation order exactly (glm 0.9.9.9 as instantiated by
// the reference, see DESIGN.md "Floating point"), compiled with -ffp-contract=off and correctly rounded
// f32 division / sqrt, so results are bit-identical to the CPU restatement in oracle/.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace romis {

struct v3 { float x, y, z; };

// ---- exact fast forms of the correctly rounded f32 sqrt / reciprocal / division ---------------------------
// Each returns bit for bit what the IEEE operation returns, on the input range its guard states; callers take
// the library expansion for lanes outside it.  tests/hip/fastmath_check.hip checks them exhaustively (sqrt,
// reciprocal: every float) and on 2^32 random + edge operand pairs (division); DESIGN.md §4 has the proofs.
//
// sqrt: the compiler's own correctly rounded expansion for -fhip-fp32-correctly-rounded-divide-sqrt
// (v_sqrt_f32, then pick s-1ulp / s / s+1ulp by the sign of the fma residuals) without its denormal rescaling
// and +-0 / inf fix-ups, which are identities for q in [2^-96, FLT_MAX].
__device__ __forceinline__ bool sqrt_fast_ok(float q) { return q >= 0x1p-96f && q <= 3.402823466e+38F; }
__device__ __forceinline__ float sqrt_rn_core(float q) {
    const float s = __builtin_amdgcn_sqrtf(q);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u), sp = __uint_as_float(__float_as_uint(s) + 1u);
    const float rm = __builtin_fmaf(-sm, s, q), rp = __builtin_fmaf(-sp, s, q);
    float r = (rm <= 0.0f) ? sm : s;
    return (rp > 0.0f) ? sp : r;
}
// reciprocal: v_rcp_f32 (< 1 ulp) + one Newton step with exact fma residual (Markstein); the exhaustive check
// pins it to 1.0f / b for every |b| in [2^-125, 2^125].
__device__ __forceinline__ bool rcp_fast_ok(float b) { const float a = fabsf(b); return a >= 0x1p-125f && a <= 0x1p125f; }
__device__ __forceinline__ float rcp_rn_core(float b) {
    const float y = __builtin_amdgcn_rcpf(b);
    return __builtin_fmaf(__builtin_fmaf(-b, y, 1.0f), y, y);
}
// division by a shared denominator: RN32(a / b) == RN32(a * R) with R ~ 1/b in double to 2^-51 relative,
// because a/b of two floats stays >= 2^-49 relative away from every f32 rounding boundary (proof in DESIGN.md).
__device__ __forceinline__ bool div_fast_ok(float b) { const float a = fabsf(b); return a >= 0x1p-120f && a <= 0x1p120f; }
__device__ __forceinline__ double rcp_d(float b) {
    const double d = (double)b;
    double y = __builtin_amdgcn_rcp(d);
    y = __builtin_fma(__builtin_fma(-d, y, 1.0), y, y);
    return __builtin_fma(__builtin_fma(-d, y, 1.0), y, y);
}
__device__ __forceinline__ float div_by_rcp_d(float a, double r) { return (float)((double)a * r); }

__device__ __forceinline__ float sqrt_rn(float q) {
    float s = sqrt_rn_core(q);
    if (__builtin_expect(!sqrt_fast_ok(q), 0)) s = sqrtf(q);
    return s;
}
__device__ __forceinline__ float rcp_rn(float b) {
    float y = rcp_rn_core(b);
    if (__builtin_expect(!rcp_fast_ok(b), 0)) y = 1.0f / b;
    return y;
}

__device__ __host__ __forceinline__ v3 mk(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
__device__ __forceinline__ v3 vadd(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ v3 vsub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ v3 vmul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ v3 vscale(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
// v / s componentwise: one double reciprocal shared by the three quotients (exact, see div_by_rcp_d)
__device__ __forceinline__ v3 vdivs(v3 a, float s) {
    if (__builtin_expect(div_fast_ok(s), 1)) {
        const double r = rcp_d(s);
        return mk(div_by_rcp_d(a.x, r), div_by_rcp_d(a.y, r), div_by_rcp_d(a.z, r));
    }
    return mk(a.x / s, a.y / s, a.z / s);
}

// glm compute_dot<vec3> (func_geometric.inl:48-54): (x*x' + y*y') + z*z'
__device__ __forceinline__ float vdot(v3 a, v3 b) { v3 t = vmul(a, b); return (t.x + t.y) + t.z; }
__device__ __forceinline__ float vlength(v3 a) { return sqrt_rn(vdot(a, a)); }
__device__ __forceinline__ float vdistance(v3 p0, v3 p1) { return vlength(vsub(p1, p0)); }
// glm normalize = v * (1 / sqrt(dot(v, v))) (func_geometric.inl:82-88); also hands back sqrt(dot(v, v)),
// which is glm::length(v) / glm::distance bit for bit.  One guard covers both fast forms: q in the sqrt range
// puts sqrt(q) in [2^-48, 2^64], inside the reciprocal's.
__device__ __forceinline__ v3 vnormalize_len(v3 a, float& len) {
    const float q = vdot(a, a);
    float s = sqrt_rn_core(q), y = rcp_rn_core(s);
    if (__builtin_expect(!sqrt_fast_ok(q), 0)) { s = sqrtf(q); y = 1.0f / s; }
    len = s;
    return vscale(a, y);
}
__device__ __forceinline__ v3 vnormalize(v3 a) { float l; return vnormalize_len(a, l); }
// glm mix = x * (1 - a) + y * a (func_common.inl:104-111)
__device__ __forceinline__ v3 vmix(v3 x, v3 y, float a) { return vadd(vscale(x, 1.0f - a), vscale(y, a)); }
__device__ __forceinline__ v3 vcross(v3 x, v3 y) {
    return mk(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
// quat * vec3 (type_quat.inl:347-354); q = (x, y, z, w)
__device__ __forceinline__ v3 qrotate(float4 q, v3 v) {
    v3 qv = mk(q.x, q.y, q.z);
    v3 uv = vcross(qv, v);
    v3 uuv = vcross(qv, uv);
    return vadd(v, vscale(vadd(vscale(uv, q.w), uuv), 2.0f));
}
__device__ __forceinline__ bool vany_nan(v3 a) { return __builtin_isnan(a.x) || __builtin_isnan(a.y) || __builtin_isnan(a.z); }
__device__ __forceinline__ v3 xyz(float4 f) { return mk(f.x, f.y, f.z); }

// ---- keyed RNG (include/restir_c.h header comment) --------------------------------------------------------
__device__ __host__ __forceinline__ uint32_t mix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
    return h;
}
__device__ __host__ __forceinline__ uint32_t pix_state(uint32_t key, uint32_t g) {
    return mix32(key ^ mix32(g * 0x9E3779B1u + 0x7F4A7C15u));
}
__device__ __host__ __forceinline__ uint32_t draw(uint32_t ps, uint32_t slot) { return mix32(ps + slot * 0x9E3779B9u); }
// rand() + linearMap(float(rand()), 0, RAND_MAX, 0, 1) (utils.cpp:26-31): exact (power-of-two scale)
__device__ __forceinline__ float rand01(uint32_t d) {
    float val = (float)(d >> 1);
    float ratio = (val - 0.0f) / (2147483648.0f - 0.0f);
    float scaled = ratio * (1.0f - 0.0f);
    return scaled + 0.0f;
}
__device__ __forceinline__ uint32_t uniform_index(uint32_t d, uint32_t n) { return __umulhi(d, n); }

// Reservoir::update's acceptance `u < w / wSum` (reservoir.cpp:24-28) for a u of rand01 (a multiple of 2^-31 in [0, 1))
// without the correctly rounded division where the answer is already known: the exact residual e = w - u wSum (one
// fma, its sign exact) gives w / wSum <= u (e <= 0: RN(w / wSum) <= u, false) and w / wSum > u + ulp(u) / 2
// (RN(e) > ulp(u) wSum: RN(w / wSum) >= the float after u, true).  Only the band in between (probability ~2^-24 per
// draw), u = 0, wSum outside [2^-60, 2^60] (where ulp(u) wSum could leave the normal range) and NaN operands take the
// division, under a wave-uniform branch.  tests/test_fast_accept.py checks the rule against the division on the CPU.
#ifndef ROMIS_FAST_ACCEPT
#define ROMIS_FAST_ACCEPT 1
#endif
__device__ __forceinline__ bool accept_u(float u, float w, float ws) {
#if ROMIS_FAST_ACCEPT
    const float e = __builtin_fmaf(-u, ws, w);
    const float ulp = __uint_as_float(__float_as_uint(u) + 1u) - u;
    const bool t = e > ulp * ws;
    const bool known = (t || e <= 0.0f) && u != 0.0f && ws >= 0x1p-60f && ws <= 0x1p60f;
    bool acc = t;
    if (__builtin_expect(__any(!known), 0)) {
        if (!known) acc = u < (w / ws);
    }
    return acc;
#else
    return u < (w / ws);
#endif
}
__device__ __forceinline__ int uniform_offset(uint32_t d, uint32_t r) { return (int)__umulhi(d, 2u * r + 1u) - (int)r; }

// ---- powf / expf: glibc 2.35's flt-32 algorithms, FMA objects (oracle/portable_math.h is the CPU side) -------
// The reference's std::pow(float, float) (shading.cpp:26, tone_mapping.cpp:10) and expf (tone_mapping.cpp:9)
// resolve to glibc's __powf_fma / __expf_fma on x86-64: log2 through a 16-entry {1/c, log2 c} table and a
// degree-5 polynomial, exp2 through a 32-entry 2^(i/32) table and a degree-3 polynomial, all in double with the
// fused multiply-adds of the FMA objects.  v_fma_f64 is the same single-rounding operation as vfmadd*sd, so
// the sequence below returns glibc's bits (oracle/check_libm.c: every 32-bit base for the scenes' exponents and
// every expf input, 0 mismatches; tests/test_gpu_parity.py::test_device_math_matches_oracle pins GPU = CPU).
__constant__ double kGlLog2Tab[32] = {
    0x1.661ec79f8f3bep+0, -0x1.efec65b963019p-2, 0x1.571ed4aaf883dp+0, -0x1.b0b6832d4fca4p-2,
    0x1.49539f0f010bp+0,  -0x1.7418b0a1fb77bp-2, 0x1.3c995b0b80385p+0, -0x1.39de91a6dcf7bp-2,
    0x1.30d190c8864a5p+0, -0x1.01d9bf3f2b631p-2, 0x1.25e227b0b8eap+0,  -0x1.97c1d1b3b7afp-3,
    0x1.1bb4a4a1a343fp+0, -0x1.2f9e393af3c9fp-3, 0x1.12358f08ae5bap+0, -0x1.960cbbf788d5cp-4,
    0x1.0953f419900a7p+0, -0x1.a6f9db6475fcep-5, 0x1p+0,               0x0p+0,
    0x1.e608cfd9a47acp-1, 0x1.338ca9f24f53dp-4,  0x1.ca4b31f026aap-1,  0x1.476a9543891bap-3,
    0x1.b2036576afce6p-1, 0x1.e840b4ac4e4d2p-3,  0x1.9c2d163a1aa2dp-1, 0x1.40645f0c6651cp-2,
    0x1.886e6037841edp-1, 0x1.88e9c2c1b9ff8p-2,  0x1.767dcf5534862p-1, 0x1.ce0a44eb17bccp-2,
};
__constant__ unsigned long long kGlExp2Tab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull,
};

// where a kernel keeps the two tables: the __constant__ copies, or a workgroup's LDS copy (gl_stage_tables)
struct GlTabs {
    const double* log2;                 // [16][2] {invc, logc}
    const unsigned long long* exp2;     // [32]
};
__device__ __forceinline__ GlTabs gl_global_tabs() { GlTabs t; t.log2 = kGlLog2Tab; t.exp2 = kGlExp2Tab; return t; }

__device__ __forceinline__ float gl_xflowf(uint32_t sign, float y) { return (sign ? -y : y) * y; }
__device__ __forceinline__ int gl_checkint(uint32_t iy) {
    const int e = (int)(iy >> 23 & 0xff);
    if (e < 0x7f) return 0;
    if (e > 0x7f + 23) return 2;
    if (iy & ((1u << (0x7f + 23 - e)) - 1)) return 0;
    if (iy & (1u << (0x7f + 23 - e))) return 1;
    return 2;
}
__device__ __forceinline__ bool gl_zeroinfnan(uint32_t i) { return 2u * i - 1u >= 2u * 0x7f800000u - 1u; }
__device__ __forceinline__ bool gl_issignaling(uint32_t i) { return 2u * (i ^ 0x00400000u) > 2u * 0x7fc00000u; }
// x86 x + y with a NaN operand: the first NaN operand, quieted
__device__ __forceinline__ float gl_nan_add(float x, float y) {
    const uint32_t ix = __float_as_uint(x), iy = __float_as_uint(y);
    if ((ix & 0x7fffffffu) > 0x7f800000u) return __uint_as_float(ix | 0x00400000u);
    if ((iy & 0x7fffffffu) > 0x7f800000u) return __uint_as_float(iy | 0x00400000u);
    return x + y;
}

__device__ __forceinline__ double gl_log2_inline(const GlTabs& tb, uint32_t ix) {
    const uint32_t tmp = ix - 0x3f330000u;
    const uint32_t i = (tmp >> 19) & 15u;
    const uint32_t top = tmp & 0xff800000u;
    const uint32_t iz = ix - top;
    const int k = (int32_t)top >> 23;
    const double2 c = reinterpret_cast<const double2*>(tb.log2)[i];   // {invc, logc}
    const double z = (double)__uint_as_float(iz);
    const double r = __builtin_fma(z, c.x, -1.0);
    const double y0 = c.y + (double)k;
    const double r2 = r * r;
    const double y = __builtin_fma(r, 0x1.27616c9496e0bp-2, -0x1.71969a075c67ap-2);
    const double p = __builtin_fma(r, 0x1.ec70a6ca7baddp-2, -0x1.7154748bef6c8p-1);
    const double r4 = r2 * r2;
    double q = __builtin_fma(r, 0x1.71547652ab82bp+0, y0);
    q = __builtin_fma(r2, p, q);
    return __builtin_fma(y, r4, q);
}

__device__ __forceinline__ double gl_exp2_scaled(const GlTabs& tb, unsigned long long ki, double r, double c0, double c1,
                                                 double c2) {
    unsigned long long t = tb.exp2[ki & 31u];
    t += ki << 47;
    const double s = __longlong_as_double((long long)t);
    const double z = __builtin_fma(r, c0, c1);
    const double r2 = r * r;
    double y = __builtin_fma(r, c2, 1.0);
    y = __builtin_fma(z, r2, y);
    return y * s;
}

// exp2_inline (e_powf.c) rounded to float: kd = ylogx + SHIFT rounds ylogx to k/32
__device__ __forceinline__ float gl_exp2_inline(const GlTabs& tb, double ylogx, uint32_t sign_bias) {
    double kd = ylogx + 0x1.8p+47;
    const unsigned long long ki = (unsigned long long)__double_as_longlong(kd);
    kd -= 0x1.8p+47;
    const double r = ylogx - kd;
    return (float)gl_exp2_scaled(tb, ki + sign_bias, r, 0x1.c6af84b912394p-5, 0x1.ebfce50fac4f3p-3,
                                 0x1.62e42ff0c52d6p-1);
}

// __powf (e_powf.c) with the caller's table location
__device__ __forceinline__ float gl_powf(const GlTabs& tb, float x, float y) {
    uint32_t sign_bias = 0;
    uint32_t ix = __float_as_uint(x);
    const uint32_t iy = __float_as_uint(y);
    if (__builtin_expect(ix - 0x00800000u >= 0x7f800000u - 0x00800000u || gl_zeroinfnan(iy), 0)) {
        if (gl_zeroinfnan(iy)) {
            if (2u * iy == 0u) return gl_issignaling(ix) ? gl_nan_add(x, y) : 1.0f;
            if (ix == 0x3f800000u) return gl_issignaling(iy) ? gl_nan_add(x, y) : 1.0f;
            if (2u * ix > 2u * 0x7f800000u || 2u * iy > 2u * 0x7f800000u) return gl_nan_add(x, y);
            if (2u * ix == 2u * 0x3f800000u) return 1.0f;
            if ((2u * ix < 2u * 0x3f800000u) == !(iy & 0x80000000u)) return 0.0f;
            return y * y;
        }
        if (gl_zeroinfnan(ix)) {
            float x2 = x * x;
            if ((ix & 0x80000000u) && gl_checkint(iy) == 1) x2 = -x2;
            return (iy & 0x80000000u) ? 1.0f / x2 : x2;
        }
        if (ix & 0x80000000u) {
            const int yint = gl_checkint(iy);
            if (yint == 0) return __uint_as_float(0xffc00000u);
            if (yint == 1) sign_bias = 0x10000u;
            ix &= 0x7fffffffu;
        }
        if (ix < 0x00800000u) {
            ix = __float_as_uint(__uint_as_float(ix) * 0x1p23f);
            ix &= 0x7fffffffu;
            ix -= 23u << 23;
        }
    }
    const double logx = gl_log2_inline(tb, ix);
    const double ylogx = (double)y * logx;
    if (__builtin_expect(((unsigned long long)__double_as_longlong(ylogx) >> 47 & 0xffffu) >= 0x80bfu, 0)) {
        if (ylogx > 0x1.fffffffd1d571p+6) return gl_xflowf(sign_bias, 0x1p97f);
        if (ylogx <= -150.0) return gl_xflowf(sign_bias, 0x1p-95f);
        if (ylogx < -149.0) return gl_xflowf(sign_bias, 0x1.4p-75f);
    }
    return gl_exp2_inline(tb, ylogx, sign_bias);
}

// __expf (e_expf.c)
__device__ __forceinline__ float gl_expf(const GlTabs& tb, float x) {
    const uint32_t ux = __float_as_uint(x);
    const double xd = (double)x;
    const uint32_t abstop = (ux >> 20) & 0x7ffu;
    if (__builtin_expect(abstop >= 0x42au, 0)) {
        if (ux == 0xff800000u) return 0.0f;
        if (abstop >= 0x7f8u) return gl_nan_add(x, x);
        if (x > 0x1.62e42ep6f) return gl_xflowf(0, 0x1p97f);
        if (x < -0x1.9fe368p6f) return gl_xflowf(0, 0x1p-95f);
        if (x < -0x1.9d1d9ep6f) return gl_xflowf(0, 0x1.4p-75f);
    }
    double kd = __builtin_fma(0x1.71547652b82fep+5, xd, 0x1.8p+52);
    const unsigned long long ki = (unsigned long long)__double_as_longlong(kd);
    kd -= 0x1.8p+52;
    const double r = __builtin_fma(0x1.71547652b82fep+5, xd, -kd);
    return (float)gl_exp2_scaled(tb, ki, r, 0x1.c6af84b912394p-20, 0x1.ebfce50fac4f3p-13, 0x1.62e42ff0c52d6p-6);
}

// the call sites that do not stage the tables
__device__ __noinline__ float pm_powf_general(float x, float y) { return gl_powf(gl_global_tabs(), x, y); }
__device__ __forceinline__ float pm_powf(float x, float y) { return gl_powf(gl_global_tabs(), x, y); }
__device__ __forceinline__ float pm_expf(float x) { return gl_expf(gl_global_tabs(), x); }

}  // namespace romis

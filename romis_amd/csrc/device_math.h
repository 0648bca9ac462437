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
#if defined(ROMIS_ABL_RNG)
__device__ __host__ __forceinline__ uint32_t draw(uint32_t ps, uint32_t slot) { uint32_t h = ps + slot * 0x9E3779B9u; return h ^ (h >> 15); }
#else
__device__ __host__ __forceinline__ uint32_t draw(uint32_t ps, uint32_t slot) { return mix32(ps + slot * 0x9E3779B9u); }
#endif
// rand() + linearMap(float(rand()), 0, RAND_MAX, 0, 1) (utils.cpp:26-31): exact (power-of-two scale)
__device__ __forceinline__ float rand01(uint32_t d) {
    float val = (float)(d >> 1);
    float ratio = (val - 0.0f) / (2147483648.0f - 0.0f);
    float scaled = ratio * (1.0f - 0.0f);
    return scaled + 0.0f;
}
__device__ __forceinline__ uint32_t uniform_index(uint32_t d, uint32_t n) { return __umulhi(d, n); }
__device__ __forceinline__ int uniform_offset(uint32_t d, uint32_t r) { return (int)__umulhi(d, 2u * r + 1u) - (int)r; }

// ---- portable powf / expf (same algorithm as oracle/portable_math.h, evaluated in double) -----------------
__device__ __forceinline__ double pm_ldexp1(int n) { return __longlong_as_double((long long)(n + 1023) << 52); }

__device__ __forceinline__ double pm_log_d(double a) {
    unsigned long long b = (unsigned long long)__double_as_longlong(a);
    int e = (int)((b >> 52) & 0x7FF) - 1023;
    double m = __longlong_as_double((long long)((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull));
    if (m > 1.4142135623730951) { m = m * 0.5; e = e + 1; }
    double s = (m - 1.0) / (m + 1.0);
    double s2 = s * s;
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

__device__ __forceinline__ double pm_exp_d(double z) {
    double kf = floor(z * 1.4426950408889634074 + 0.5);
    int k = (int)kf;
    double r = (z - kf * 0.693147180369123816490) - kf * 1.90821492927058770002e-10;
    double p = 1.0 / 6227020800.0;
    p = 1.0 / 479001600.0 + r * p;
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
    int k1 = k / 2, k2 = k - k / 2;
    return (p * pm_ldexp1(k1)) * pm_ldexp1(k2);
}

__device__ __forceinline__ bool pm_is_int(float y) { return y == truncf(y); }
__device__ __forceinline__ bool pm_is_odd_int(float y) {
    if (!pm_is_int(y) || fabsf(y) >= 16777216.0f) return false;
    long long i = (long long)y;
    return (i & 1) != 0;
}

__device__ __noinline__ float pm_powf_general(float x, float y) {
    if (y == 0.0f) return 1.0f;
    if (x == 1.0f) return 1.0f;
    if (__builtin_isnan(x) || __builtin_isnan(y)) return x + y;
    bool yint = pm_is_int(y), yodd = pm_is_odd_int(y);
    if (x == 0.0f) {
        if (y < 0.0f) return yodd ? copysignf(__builtin_inff(), x) : __builtin_inff();
        return yodd ? x : 0.0f;
    }
    if (__builtin_isinf(y)) {
        float ax = fabsf(x);
        if (ax == 1.0f) return 1.0f;
        return ((ax < 1.0f) == (y < 0.0f)) ? __builtin_inff() : 0.0f;
    }
    if (__builtin_isinf(x)) {
        if (x > 0.0f) return y < 0.0f ? 0.0f : __builtin_inff();
        if (yodd) return y < 0.0f ? -0.0f : -__builtin_inff();
        return y < 0.0f ? 0.0f : __builtin_inff();
    }
    if (x < 0.0f && !yint) return __builtin_nanf("");
    double sign = (x < 0.0f && yodd) ? -1.0 : 1.0;
    double ax = fabs((double)x);
    double r;
    if (yint && fabsf(y) <= 1048576.0f) {
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
        if (z > 89.0) r = __builtin_inf();
        else if (z < -104.0) r = 0.0;
        else r = pm_exp_d(z);
    }
    return (float)(sign * r);
}

__device__ __forceinline__ float pm_powf(float x, float y) { return pm_powf_general(x, y); }

__device__ __forceinline__ float pm_expf(float x) {
    if (__builtin_isnan(x)) return x;
    if (x > 89.0f) return __builtin_inff();
    if (x < -104.0f) return 0.0f;
    return (float)pm_exp_d((double)x);
}

}  // namespace romis

// kernels_common.h -- the device side shared by the frame kernels (kernels.hip) and the R-MIS / R-OMIS kernels
// (mis.hip): BVH traversal, the pixel shading context and target pdf (computeShading, shading.cpp:7-34), glibc's
// powf, reservoir state, tile / work mappings.  One translation unit per kernel family, compiled side by side.
#pragma once
#include "device_math.h"
#include "restir_c.h"
#include "restir_types.h"

#include <float.h>

namespace romis {

#define ROMIS_FLT_MAX 3.402823466e+38F
#define ROMIS_FLT_MIN 1.175494351e-38F

// ---------------------------------------------------------------------------------------------------------
// Ray / triangle, Moller-Trumbore, hit iff 0 < t <= tfar (Embree's (tnear, tfar] convention; the oracle
// restates the same routine).
__device__ __forceinline__ bool tri_hit(float4 v0, float4 e1_, float4 e2_, v3 o, v3 d, float tfar, float& t_out,
                                        float& u_out, float& v_out) {
    v3 e1 = xyz(e1_), e2 = xyz(e2_);
    v3 pvec = vcross(d, e2);
    float det = vdot(e1, pvec);
    if (det == 0.0f) return false;
    const float inv = rcp_rn(det);   // == 1.0f / det (the exact fast form, library division outside its range)
    v3 tvec = vsub(o, xyz(v0));
    float u = vdot(tvec, pvec) * inv;
    if (!(u >= 0.0f && u <= 1.0f)) return false;
    v3 qvec = vcross(tvec, e1);
    float v = vdot(d, qvec) * inv;
    if (!(v >= 0.0f && u + v <= 1.0f)) return false;
    float t = vdot(e2, qvec) * inv;
    if (!(t > 0.0f && t <= tfar)) return false;
    t_out = t; u_out = u; v_out = v;
    return true;
}

// tri_hit without early exits: the same expressions (u, v, t computed for every triangle), the decision as a
// predicate; straight-line code for the closest-hit leaf loop
__device__ __forceinline__ bool tri_test(float4 v0, float4 e1_, float4 e2_, v3 o, v3 d, float tfar, float& t, float& u,
                                         float& v) {
    const v3 e1 = xyz(e1_), e2 = xyz(e2_);
    const v3 pvec = vcross(d, e2);
    const float det = vdot(e1, pvec);
    const float inv = rcp_rn(det);
    const v3 tvec = vsub(o, xyz(v0));
    u = vdot(tvec, pvec) * inv;
    const v3 qvec = vcross(tvec, e1);
    v = vdot(d, qvec) * inv;
    t = vdot(e2, qvec) * inv;
    return det != 0.0f && (u >= 0.0f && u <= 1.0f) && (v >= 0.0f && u + v <= 1.0f) && (t > 0.0f && t <= tfar);
}

// The same test as an any-hit predicate without early exits (shadow rays): the same float expressions, so the
// same decision, but straight-line code the compiler can interleave across a leaf's triangles.
__device__ __forceinline__ bool tri_any(float4 v0, float4 e1_, float4 e2_, v3 o, v3 d, float tfar) {
    const v3 e1 = xyz(e1_), e2 = xyz(e2_);
    const v3 pvec = vcross(d, e2);
    const float det = vdot(e1, pvec);
    const float inv = rcp_rn(det);
    const v3 tvec = vsub(o, xyz(v0));
    const float u = vdot(tvec, pvec) * inv;
    const v3 qvec = vcross(tvec, e1);
    const float v = vdot(d, qvec) * inv;
    const float t = vdot(e2, qvec) * inv;
    return det != 0.0f && (u >= 0.0f && u <= 1.0f) && (v >= 0.0f && u + v <= 1.0f) && (t > 0.0f && t <= tfar);
}

// Conservative slab test (boxes are padded on the host, the interval is widened): it may accept extra boxes,
// never reject one that holds a valid hit, so traversal results equal the brute-force oracle.
__device__ __forceinline__ bool box_hit(float4 lo, float4 hi, v3 o, v3 invd, float tmax_box) {
    float tx0 = (lo.x - o.x) * invd.x, tx1 = (hi.x - o.x) * invd.x;
    float ty0 = (lo.y - o.y) * invd.y, ty1 = (hi.y - o.y) * invd.y;
    float tz0 = (lo.z - o.z) * invd.z, tz1 = (hi.z - o.z) * invd.z;
    float tmin = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
    float tmax = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tmax_box));
    return tmin <= tmax;
}

__device__ __forceinline__ v3 safe_inv(v3 d) {
    return mk(1.0f / (d.x == 0.0f ? copysignf(1e-30f, d.x) : d.x), 1.0f / (d.y == 0.0f ? copysignf(1e-30f, d.y) : d.y),
              1.0f / (d.z == 0.0f ? copysignf(1e-30f, d.z) : d.z));
}

__device__ __forceinline__ float widen(float t) { return t * 1.0001f + 1e-4f; }

// The traversal arrays, either the global copies or the workgroup's LDS copy.
struct Bvh {
    const float4* nodes;
    const float4* v0;
    const float4* e1;
    const float4* e2;
    uint32_t num_nodes;
};

__device__ __forceinline__ Bvh global_bvh(const SceneDev& s) {
    Bvh b;
    b.nodes = s.nodes; b.v0 = s.tri_v0; b.e1 = s.tri_e1; b.e2 = s.tri_e2; b.num_nodes = s.num_nodes;
    return b;
}

// Copy nodes + triangles into LDS (every thread of the block participates; ends with a barrier).  nodes = false: the
// triangles alone, at the same offsets (a block whose rays all test candidate lists, primary.tl)
__device__ __forceinline__ Bvh stage_bvh(const SceneDev& s, float4* lds, bool nodes = true) {
    const uint32_t nn = 2u * s.num_nodes, nt = s.num_tris;
    if (nodes)
        for (uint32_t i = threadIdx.x; i < nn; i += blockDim.x) lds[i] = s.nodes[i];
    for (uint32_t i = threadIdx.x; i < nt; i += blockDim.x) {
        lds[nn + i] = s.tri_v0[i];
        lds[nn + nt + i] = s.tri_e1[i];
        lds[nn + 2 * nt + i] = s.tri_e2[i];
    }
    __syncthreads();
    Bvh b;
    b.nodes = lds; b.v0 = lds + nn; b.e1 = lds + nn + nt; b.e2 = lds + nn + 2 * nt; b.num_nodes = s.num_nodes;
    return b;
}

// any hit in (0, tfar] -- EmbreeInterface::anyHit (embree_interface.cpp:58-62)
__device__ __forceinline__ bool occluded(const Bvh& b, v3 o, v3 d, float tfar) {
    v3 invd = safe_inv(d);
    float tb = widen(tfar);
    uint32_t i = 0;
    while (i < b.num_nodes) {
        float4 lo = b.nodes[2 * i], hi = b.nodes[2 * i + 1];
        uint32_t miss = __float_as_uint(lo.w), leaf = __float_as_uint(hi.w);
        if (box_hit(lo, hi, o, invd, tb)) {
            if (leaf) {
                uint32_t first = leaf & 0xFFFFFFu, cnt = leaf >> 24;
                for (uint32_t k = 0; k < cnt; k += 2) {   // two triangles per step (leaves hold 2 by default)
                    bool h = tri_any(b.v0[first + k], b.e1[first + k], b.e2[first + k], o, d, tfar);
                    if (k + 1 < cnt) h = tri_any(b.v0[first + k + 1], b.e1[first + k + 1], b.e2[first + k + 1], o, d, tfar) || h;
                    if (h) return true;
                }
                i = miss;
            } else {
                i = i + 1;
            }
        } else {
            i = miss;
        }
    }
    return false;
}

// The shadow rays' traversal arrays over the 16-byte nodes (SceneDev::nodes_q), global or the workgroup's LDS copy.
struct BvhQ {
    const uint4* nodes;
    const float4* v0;
    const float4* e1;
    const float4* e2;
    uint32_t num_nodes;
    v3 lo, s;   // coordinate = lo + q * s per axis
};

// Copy the 16-byte nodes + triangles into LDS (every thread of the block participates; ends with a barrier).
__device__ __forceinline__ BvhQ stage_bvh_q(const SceneDev& s, float4* lds) {
    const uint32_t nn = s.num_nodes, nt = s.num_tris;
    uint4* ln = reinterpret_cast<uint4*>(lds);
    for (uint32_t i = threadIdx.x; i < nn; i += blockDim.x) ln[i] = s.nodes_q[i];
    for (uint32_t i = threadIdx.x; i < nt; i += blockDim.x) {
        lds[nn + i] = s.tri_v0[i];
        lds[nn + nt + i] = s.tri_e1[i];
        lds[nn + 2 * nt + i] = s.tri_e2[i];
    }
    __syncthreads();
    BvhQ b;
    b.nodes = ln; b.v0 = lds + nn; b.e1 = lds + nn + nt; b.e2 = lds + nn + 2 * nt; b.num_nodes = nn;
    b.lo = xyz(s.q_lo); b.s = xyz(s.q_s);
    return b;
}

// occluded over the 16-byte nodes: the same threaded walk, one 16-byte node read per step instead of two.  The slab
// distances of a grid coordinate lo + q s are fma(q, s / d, (lo - o) / d): the quantized box contains the padded float
// box (snapped outward, bvh padding 1e-5 of the scene size beyond the triangles, grid step 1.5e-5 of it), and the
// rounding of either test is ~2^-22 of the scene size, so every box holding a hit the float test accepts is accepted
// here; the result, any exact triangle hit in
// (0, tfar] among the accepted leaves, is occluded's (render_utils.cpp:54-65 -> utils.cpp:41-56).
__device__ __forceinline__ bool occluded_q(const BvhQ& b, v3 o, v3 d, float tfar) {
    const v3 invd = safe_inv(d);
    const float tb = widen(tfar);
    const v3 A = mk(b.s.x * invd.x, b.s.y * invd.y, b.s.z * invd.z);
    const v3 C = mk((b.lo.x - o.x) * invd.x, (b.lo.y - o.y) * invd.y, (b.lo.z - o.z) * invd.z);
    uint32_t i = 0;
    while (i < b.num_nodes) {
        const uint4 n = b.nodes[i];
        const float tx0 = __builtin_fmaf((float)(n.x & 0xFFFFu), A.x, C.x), tx1 = __builtin_fmaf((float)(n.y >> 16), A.x, C.x);
        const float ty0 = __builtin_fmaf((float)(n.x >> 16), A.y, C.y), ty1 = __builtin_fmaf((float)(n.z & 0xFFFFu), A.y, C.y);
        const float tz0 = __builtin_fmaf((float)(n.y & 0xFFFFu), A.z, C.z), tz1 = __builtin_fmaf((float)(n.z >> 16), A.z, C.z);
        const float tmin = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
        const float tmax = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tb));
        const uint32_t cnt = n.w >> 28, miss = n.w & 0xFFFFu;
        if (tmin <= tmax) {
            if (cnt) {
                const uint32_t first = (n.w >> 16) & 0xFFFu;
                for (uint32_t k = 0; k < cnt; k += 2) {   // two triangles per step, as occluded
                    bool h = tri_any(b.v0[first + k], b.e1[first + k], b.e2[first + k], o, d, tfar);
                    if (k + 1 < cnt) h = tri_any(b.v0[first + k + 1], b.e1[first + k + 1], b.e2[first + k + 1], o, d, tfar) || h;
                    if (h) return true;
                }
                i = miss;
            } else {
                i = i + 1;
            }
        } else {
            i = miss;
        }
    }
    return false;
}

// testVisibilityLightSample (utils.cpp:41-56) over the 16-byte nodes
__device__ __forceinline__ bool visible_q(const BvhQ& b, v3 P, v3 y) {
    v3 dir = vnormalize(vsub(y, P));
    v3 P2 = vadd(P, vscale(dir, 1e-3f));
    float tfar = vdistance(P2, y);
    return !occluded_q(b, P2, dir, tfar);
}

// closest hit: minimal t, lowest original triangle index on ties
__device__ __forceinline__ bool closest(const Bvh& b, v3 o, v3 d, float& t_best, float& u_best, float& v_best,
                                        uint32_t& tri_best) {
    v3 invd = safe_inv(d);
    bool found = false;
    t_best = ROMIS_FLT_MAX;
    tri_best = 0xFFFFFFFFu;
    uint32_t i = 0;
    while (i < b.num_nodes) {
        float4 lo = b.nodes[2 * i], hi = b.nodes[2 * i + 1];
        uint32_t miss = __float_as_uint(lo.w), leaf = __float_as_uint(hi.w);
        if (box_hit(lo, hi, o, invd, widen(t_best))) {
            if (leaf) {
                uint32_t first = leaf & 0xFFFFFFu, cnt = leaf >> 24;
                for (uint32_t k = 0; k < cnt; k++) {
                    const float4 v0 = b.v0[first + k];
                    float t, u, v;
                    const bool h = tri_test(v0, b.e1[first + k], b.e2[first + k], o, d, ROMIS_FLT_MAX, t, u, v);
                    const uint32_t orig = __float_as_uint(v0.w);
                    if (h && (!found || t < t_best || (t == t_best && orig < tri_best))) {
                        found = true; t_best = t; u_best = u; v_best = v; tri_best = orig;
                    }
                }
                i = miss;
            } else {
                i = i + 1;
            }
        } else {
            i = miss;
        }
    }
    return found;
}

// closest() over a list of candidate triangles (indices into the traversal arrays): the same tests with the same
// selection rule (minimal t, lowest original index on ties), which does not depend on the order the triangles are
// tested in -- so any list that holds every triangle a ray can hit gives closest()'s result (round 6, primary.tl)
// (the list: four segments of 64 entries, cnt[w] used in segment w; the triangles indexed as the traversal arrays)
__device__ __forceinline__ bool closest_list(const Bvh& b, const uint16_t* tl, const uint32_t* cnt, v3 o, v3 d,
                                             float& t_best, float& u_best, float& v_best, uint32_t& tri_best) {
    bool found = false;
    t_best = ROMIS_FLT_MAX;
    tri_best = 0xFFFFFFFFu;
    for (uint32_t w = 0; w < 4u; w++)
    for (uint32_t k = 0; k < cnt[w]; k++) {
        const uint32_t i = tl[64u * w + k];
        const float4 v0 = b.v0[i];
        float t, u, v;
        const bool h = tri_test(v0, b.e1[i], b.e2[i], o, d, ROMIS_FLT_MAX, t, u, v);
        const uint32_t orig = __float_as_uint(v0.w);
        if (h && (!found || t < t_best || (t == t_best && orig < tri_best))) {
            found = true; t_best = t; u_best = u; v_best = v; tri_best = orig;
        }
    }
    return found;
}

// testVisibilityLightSample (utils.cpp:41-56)
__device__ __forceinline__ bool visible(const Bvh& b, v3 P, v3 y) {
    v3 dir = vnormalize(vsub(y, P));
    v3 P2 = vadd(P, vscale(dir, 1e-3f));
    float tfar = vdistance(P2, y);
    return !occluded(b, P2, dir, tfar);
}

// ---------------------------------------------------------------------------------------------------------
// Pixel shading context
struct Px {
    v3 P, N, V;
    float t;
    uint32_t mat;
    float4 kd_sh;   // diffuseAlbedo.xyz (kd, or the kdTexture texel -- apply_albedo), shininess
    float4 ks_pm;   // ks.xyz, bits(pow mode)
    float4 pw;      // (pow underflow threshold, bits(shininess class), transparency, bits(kd_texture))
};

// acquireTexel's index (texture.cpp:5-6): the float product texCoord * (size - 1) truncated toward zero;
// products outside [0, size - 1] (an out-of-bounds read in the reference) clamp to the edge texel
__device__ __forceinline__ uint32_t texel_index(float c, uint32_t n) {
    const float v = c * (float)((int)n - 1);
    if (!(v >= 0.0f)) return 0u;
    if (v >= (float)(n - 1u)) return n - 1u;
    return (uint32_t)v;
}

// diffuseAlbedo (utils.cpp:33-37): with texture mapping on and a kdTexture on the material, the texel at the
// hit's texCoord (the G-buffer plane s.gbuf_uv, view pixel p) replaces kd as the diffuse colour
__device__ __forceinline__ void apply_albedo(const SceneDev& s, Px& r, size_t p) {
    const uint32_t tex = __float_as_uint(r.pw.w);
    if (s.tex_on && tex) {
        const float2 tc = s.gbuf_uv[p];
        const uint4 dim = s.tex_dims[tex - 1u];   // width, height, first texel
        const float4 t = s.tex_texels[dim.z + texel_index(tc.y, dim.y) * dim.x + texel_index(tc.x, dim.x)];
        r.kd_sh.x = t.x; r.kd_sh.y = t.y; r.kd_sh.z = t.z;
    }
}

__device__ __forceinline__ Px make_px(const SceneDev& s, float4 a, float4 b, v3 origin, size_t p) {
    Px r;
    r.N = xyz(a); r.t = a.w;
    r.P = xyz(b);
    uint32_t m = __float_as_uint(b.w);
    if (m >= s.num_materials) m = s.num_materials - 1;
    r.mat = m;
    r.kd_sh = s.materials[3 * m];
    r.ks_pm = s.materials[3 * m + 1];
    r.pw = s.materials[3 * m + 2];
    r.V = vnormalize(vsub(origin, r.P));
    apply_albedo(s, r, p);
    return r;
}

__device__ __forceinline__ size_t gidx(const Region& rg, size_t p) { return p * rg.ps; }
__device__ __forceinline__ size_t ridx(const Region& rg, uint32_t j, size_t p) { return (size_t)j * rg.js + p * rg.ps; }

__device__ __forceinline__ Px load_px(const SceneDev& s, const Region& rg, const float4* __restrict__ n_t,
                                      const float4* __restrict__ p_mat, size_t p, v3 origin) {
    return make_px(s, n_t[gidx(rg, p)], p_mat[p], origin, p);
}

// std::pow(cosTheta, shininess) (shading.cpp:26) = glibc's powf (device_math.h gl_powf), specialised per
// material with the exponent's classes precomputed on the host (restir.cpp put_material, ROMIS_PWC_*):
//  - ks == 0 skips it (the product with ks is the same +-0 the reference gets after its NaN clean-up --
//    DESIGN.md "Floating point");
//  - |x| below the material's threshold is glibc's own underflow exit (+-0, negative for a negative base and an
//    odd integer exponent), decided before the log2 / exp2 evaluation;
//  - y = +-0 / NaN / +-inf are glibc's zeroinfnan(y) returns; otherwise of its special cases only a NaN base
//    (whose NaN the caller's clean-up zeroes whatever its payload: cosTheta is never a signalling NaN), a
//    negative base (invalid unless y is an integer, sign from y's parity) and a zero / subnormal base remain.
// material_pow in two parts.  pow_pre decides every case glibc settles without its log2 / exp2 core (returns
// true with the power in pw); otherwise it returns false with the core's input in job: the (subnormal-adjusted)
// bits of |x| and, in bit 31, glibc's sign_bias (negative base, odd integer exponent).  pow_core(job, y) is the
// rest of __powf.  (Evaluating only the cores some lane needs, wave-compacted through LDS across batches of
// candidates, was measured slower in RIS: 345 -> 393-591 us, the batch state costing occupancy -- DESIGN §6.)
__device__ __forceinline__ bool pow_pre(float x, const Px& px, float& pw, uint32_t& job) {
    const uint32_t mode = __float_as_uint(px.ks_pm.w);
    if (mode != ROMIS_POW_GLIBC) {
        // ROMIS_POW_SKIP, or ROMIS_POW_SIMPLE: every base glibc settles before its core is under the threshold
        // (+-0, NaN passed through) or a negative base with a non-integer exponent (invalid), as selects
        const uint32_t cls = __float_as_uint(px.pw.y);
        const float ax = fabsf(x);
        const bool neg_odd = __builtin_signbit(x) && (cls & ROMIS_PWC_ODD);
        const bool under = !(ax >= px.pw.x);
        const bool invalid = x < 0.0f && !(cls & ROMIS_PWC_INT);
        float r = under ? (__builtin_isnan(x) ? x : (neg_odd ? -0.0f : 0.0f)) : __uint_as_float(0xffc00000u);
        const bool skip = mode == ROMIS_POW_SKIP;
        pw = skip ? 1.0f : r;
        job = __float_as_uint(ax) | (neg_odd ? 0x80000000u : 0u);
        return skip || under || invalid;
    }
    const uint32_t cls = __float_as_uint(px.pw.y);
    const float ax = fabsf(x);
    if (__builtin_expect(cls & ROMIS_PWC_SPECIAL, 0)) {
        if (cls & ROMIS_PWC_ZERO) pw = 1.0f;
        else if (cls & ROMIS_PWC_NAN) pw = x == 1.0f ? 1.0f : __builtin_nanf("");
        else if (__builtin_isnan(x)) pw = x;
        else if (ax == 1.0f) pw = 1.0f;
        else pw = ((ax < 1.0f) == ((cls & ROMIS_PWC_PINF) != 0u)) ? 0.0f : __builtin_inff();
        return true;
    }
    const bool neg_odd = __builtin_signbit(x) && (cls & ROMIS_PWC_ODD);
    if (!(ax >= px.pw.x)) { pw = __builtin_isnan(x) ? x : (neg_odd ? -0.0f : 0.0f); return true; }
    if (x < 0.0f && !(cls & ROMIS_PWC_INT)) { pw = __uint_as_float(0xffc00000u); return true; }
    uint32_t ix = __float_as_uint(ax);
    if (__builtin_expect(ix < 0x00800000u, 0)) {
        if (ix == 0u) {
            const float z = neg_odd ? -0.0f : 0.0f;
            pw = (cls & ROMIS_PWC_NEG) ? 1.0f / z : z;
            return true;
        }
        ix = (__float_as_uint(ax * 0x1p23f) & 0x7fffffffu) - (23u << 23);
    }
    job = ix | (neg_odd ? 0x80000000u : 0u);
    return false;
}

__device__ __forceinline__ float pow_core(const GlTabs& tb, uint32_t job, float y) {
    const double ylogx = (double)y * gl_log2_inline(tb, job & 0x7fffffffu);
    const uint32_t sign_bias = (job >> 31) ? 0x10000u : 0u;
    if (__builtin_expect(((unsigned long long)__double_as_longlong(ylogx) >> 47 & 0xffffu) >= 0x80bfu, 0)) {
        if (ylogx > 0x1.fffffffd1d571p+6) return gl_xflowf(sign_bias, 0x1p97f);
        if (ylogx <= -150.0) return gl_xflowf(sign_bias, 0x1p-95f);
        if (ylogx < -149.0) return gl_xflowf(sign_bias, 0x1.4p-75f);
    }
    return gl_exp2_inline(tb, ylogx, sign_bias);
}

__device__ __forceinline__ float material_pow(const GlTabs& tb, float x, const Px& px) {
    float pw;
    uint32_t job;
    return pow_pre(x, px, pw, job) ? pw : pow_core(tb, job, px.kd_sh.w);
}

// computeShading (shading.cpp:7-34) in two parts around the power.  shade_pre: the light direction and distance,
// dotNL (a back-facing light, dotNL < 0, shades to exactly 0) and the power's argument cosTheta.
struct ShadePre {
    float d, dotNL, cosTheta;
};
#ifndef ROMIS_SKIP_COS
#define ROMIS_SKIP_COS 1
#endif
__device__ __forceinline__ ShadePre shade_pre(const Px& px, v3 lpos) {
    ShadePre r;
    v3 L = vnormalize_len(vsub(lpos, px.P), r.d);   // d = glm::distance(hitPos, lightPos), the length normalize() takes
    r.dotNL = vdot(px.N, L);
    r.cosTheta = 0.0f;
    if (r.dotNL < 0.0f) return r;
    // ks = 0 (ROMIS_POW_SKIP): the power, and so R and cosTheta, never reach the result (pow_pre returns 1 for any
    // argument) -- skipped, ROMIS_SKIP_COS (7 of the 8 Cornell materials)
    if (ROMIS_SKIP_COS && __float_as_uint(px.ks_pm.w) == ROMIS_POW_SKIP) return r;
    v3 R = vnormalize(vsub(vscale(px.N, 2.0f * r.dotNL), L));
    r.cosTheta = vdot(R, px.V);
    return r;
}
// shade_post: the terms, the reference's NaN clean-up and the distance falloff
__device__ __forceinline__ v3 shade_post(const SceneDev& s, const Px& px, v3 lcol, float dotNL, float d, float pw) {
    v3 diffuse = vscale(vmul(lcol, xyz(px.kd_sh)), dotNL);
    v3 specular = vscale(vmul(lcol, xyz(px.ks_pm)), pw);
    // The reference zeroes a term holding a NaN.  When every colour x reflectance product is finite (host
    // check, SceneDev::shade_finite), a term can only hold one through a non-finite dotNL / pow factor, so
    // the six per-component tests run only for lanes where one of those two is non-finite.
    if (!(s.shade_finite && __builtin_isfinite(dotNL) && __builtin_isfinite(pw))) {
        if (vany_nan(diffuse)) diffuse = mk(0.0f, 0.0f, 0.0f);
        if (vany_nan(specular)) specular = mk(0.0f, 0.0f, 0.0f);
    }
    if (fabsf(d) < 1e-5f) d = 1.0f;
    return vdivs(vadd(diffuse, specular), d * d);
}

// computeShading (shading.cpp:7-34), general form: every IEEE special case, any material
__device__ __forceinline__ v3 shade_ref(const SceneDev& s, const FeaturesDev& f, const Px& px, v3 lpos, v3 lcol,
                                        const GlTabs& tb = gl_global_tabs()) {
    if (!f.shading) return xyz(s.materials[3 * px.mat]);   // material.kd, not the albedo (shading.cpp:8)
    const ShadePre sp = shade_pre(px, lpos);
    if (sp.dotNL < 0.0f) return mk(0.0f, 0.0f, 0.0f);
    return shade_post(s, px, lcol, sp.dotNL, sp.d, material_pow(tb, sp.cosTheta, px));
}

__device__ __forceinline__ v3 shade(const SceneDev& s, const FeaturesDev& f, const Px& px, v3 lpos, v3 lcol,
                                    const GlTabs& tb = gl_global_tabs()) {
    return shade_ref(s, f, px, lpos, lcol, tb);
}

// target pdf = glm::length(computeShading(...)) (light.cpp:84, reservoir.cpp:49)
__device__ __forceinline__ float target_pdf(const SceneDev& s, const FeaturesDev& f, const Px& px, v3 lpos, v3 lcol,
                                            const GlTabs& tb = gl_global_tabs()) {
    return vlength(shade_ref(s, f, px, lpos, lcol, tb));
}

// target_pdf(...) > 0.0f, exactly, without the tail of computeShading where the comparison is decided before it
// (the unbiased combine's Z, reservoir.cpp:84-96, needs only the sign).  For a ks = 0 material (ROMIS_POW_SKIP:
// the specular term is a +-0 vector) in a scene whose colour x reflectance products are finite, with
// a finite dotNL >= 0: the shaded vector is v_c = RN(RN(A_c dotNL) / D), A_c = lcol_c kd_c, D = RN(d' d') (d' = 1
// below 1e-5); p = sqrt(sum RN(v_c^2)) is > 0 iff some RN(v_c^2) > 0, i.e. some |v_c| > 2^-75.  RN is monotone, so
// max |v_c| = RN(e / D) with e = RN(max |A_c| dotNL); e > 2^-60 D decides true and e < 2^-90 D false (2^15 of margin
// against any rounding); anything else -- other materials, non-finite or tiny values -- takes the full evaluation.
__device__ __forceinline__ bool target_pdf_positive(const SceneDev& s, const FeaturesDev& f, const Px& px, v3 lpos, v3 lcol,
                                                    const GlTabs& tb) {
    if (f.shading && s.shade_finite && __float_as_uint(px.ks_pm.w) == ROMIS_POW_SKIP) {
        const ShadePre sp = shade_pre(px, lpos);
        if (sp.dotNL < 0.0f) return false;   // computeShading's back-facing exit: the zero vector
        if (__builtin_isfinite(sp.dotNL)) {
            const float A = fmaxf(fmaxf(fabsf(lcol.x * px.kd_sh.x), fabsf(lcol.y * px.kd_sh.y)), fabsf(lcol.z * px.kd_sh.z));
            const float e = A * sp.dotNL;
            const float dd = fabsf(sp.d) < 1e-5f ? 1.0f : sp.d;
            const float D = dd * dd;
            if (e > 0x1p-60f * D) return true;
            if (e < 0x1p-90f * D) return false;
        }
    }
    return target_pdf(s, f, px, lpos, lcol, tb) > 0.0f;
}

// The block's LDS copy of powf's two tables (512 B): every p-hat evaluation indexes them twice per lane, and from
// __constant__ memory each index is a vector-memory round trip in the middle of the dependent chain (two per
// target pdf); from LDS it is a ds_read.  Every thread of the block must call this (it ends with a barrier).
template <bool SYNC = true>
__device__ __forceinline__ GlTabs gl_stage_tables() {
    __shared__ double s_gl_log2[32];
    __shared__ unsigned long long s_gl_exp2[32];
    if (threadIdx.x < 32u) {
        s_gl_log2[threadIdx.x] = kGlLog2Tab[threadIdx.x];
        s_gl_exp2[threadIdx.x] = kGlExp2Tab[threadIdx.x];
    }
    if (SYNC) __syncthreads();   // SYNC = false: the caller's next barrier precedes every table read
    GlTabs t;
    t.log2 = s_gl_log2;
    t.exp2 = s_gl_exp2;
    return t;
}
// The same copy by one LDS-DMA instruction of wave 0 (lanes 0-15 the log2 table, 16-31 the exp2 table, 16 B each):
// no VGPR round trip and no wait of its own -- the register-staged form above waits for its loads right where it is
// issued, before the block's own loads go out.  The caller's s_waitcnt vmcnt(0) + barrier make it visible.
__device__ __forceinline__ GlTabs gl_stage_tables_dma() {
    __shared__ __attribute__((aligned(16))) unsigned long long s_gl_tab[64];
    if (threadIdx.x < 32u) {
        const unsigned long long* src = threadIdx.x < 16u
                                            ? reinterpret_cast<const unsigned long long*>(kGlLog2Tab) + 2u * threadIdx.x
                                            : kGlExp2Tab + 2u * (threadIdx.x - 16u);
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)s_gl_tab, 16, 0, 0);
    }
    GlTabs t;
    t.log2 = reinterpret_cast<const double*>(s_gl_tab);
    t.exp2 = s_gl_tab + 32;
    return t;
}

// ---------------------------------------------------------------------------------------------------------
// Reservoir state (reservoir.h:28-73), one sub-reservoir
struct Sub {
    v3 pos, col;
    float W;
    uint32_t M;
    float wsum, chosen;
    // target pdf of the held sample at the combining pixel, cached when the sample was accepted: the
    // final W (reservoir.cpp:61-64, light.cpp:90-93) re-evaluates exactly that value, so it is reused
    float pd;
    bool has_pd;
};

__device__ __forceinline__ void sub_init(Sub& r) {
    r.pos = mk(0.0f, 0.0f, 0.0f); r.col = mk(0.0f, 0.0f, 0.0f);
    r.W = 0.0f; r.M = 1u; r.wsum = ROMIS_FLT_MIN; r.chosen = 0.0f;
    r.pd = 0.0f; r.has_pd = false;
}

// Reservoir::update (reservoir.cpp:10-32)
__device__ __forceinline__ void sub_take(Sub& r, v3 pos, v3 col, float w, float u, float pd) {
    r.M += 1u;
    r.wsum += w;
    if (accept_u(u, w, r.wsum)) { r.pos = pos; r.col = col; r.chosen = w; r.pd = pd; r.has_pd = true; }
}

template <int NT>
__device__ __forceinline__ uint32_t res_update(Sub* r, uint32_t N, v3 pos, v3 col, float w, float u, float pd) {
    if (NT == 1) {
        sub_take(r[0], pos, col, w, u, pd);
        return 0;
    }
    uint32_t k = 0;
    float best = ROMIS_FLT_MAX;
    const uint32_t n = NT > 0 ? (uint32_t)NT : N;
    if (NT > 0) {
        // compile-time N: every sub-reservoir updated by selects, no dynamic register indexing (predicated
        // sub_take calls were merged back into one r[k] store by the compiler, which put r[] in scratch memory)
#pragma unroll
        for (uint32_t j = 0; j < (uint32_t)(NT > 0 ? NT : 1); j++)
            if (r[j].wsum < best) { k = j; best = r[j].wsum; }
        float ws = r[0].wsum;
#pragma unroll
        for (uint32_t j = 1; j < (uint32_t)(NT > 0 ? NT : 1); j++) ws = (j == k) ? r[j].wsum : ws;
        ws += w;                            // sub_take's wsum += w on the routed one
        const bool acc = accept_u(u, w, ws);      // ... and its acceptance test
#pragma unroll
        for (uint32_t j = 0; j < (uint32_t)(NT > 0 ? NT : 1); j++) {
            const bool sel = j == k, take = sel && acc;
            r[j].M += sel ? 1u : 0u;
            r[j].wsum = sel ? ws : r[j].wsum;
            r[j].pos = mk(take ? pos.x : r[j].pos.x, take ? pos.y : r[j].pos.y, take ? pos.z : r[j].pos.z);
            r[j].col = mk(take ? col.x : r[j].col.x, take ? col.y : r[j].col.y, take ? col.z : r[j].col.z);
            r[j].chosen = take ? w : r[j].chosen;
            r[j].pd = take ? pd : r[j].pd;
            r[j].has_pd = take || r[j].has_pd;
        }
    } else {
        for (uint32_t j = 0; j < n; j++)
            if (r[j].wsum < best) { k = j; best = r[j].wsum; }
        sub_take(r[k], pos, col, w, u, pd);
    }
    return k;
}

template <int NT>
__device__ __forceinline__ void macc_add(uint32_t* macc, uint32_t k, uint32_t m) {
    if (NT > 0) {
#pragma unroll
        for (uint32_t j = 0; j < (uint32_t)(NT > 0 ? NT : 1); j++)
            if (j == k) macc[j] += m;
    } else {
        macc[k] += m;
    }
}

__device__ __forceinline__ float contribution_weight(float p, uint32_t M, float wsum) {
    if (p == 0.0f) return 0.0f;
    return (rcp_rn(p) * rcp_rn((float)M)) * wsum;   // rcp_rn(b) == 1.0f / b bit for bit (device_math.h)
}

__device__ __forceinline__ Sub sub_from(float4 fa, float4 fb) {
    Sub r;
    r.pos = xyz(fa); r.W = fa.w;
    r.col = xyz(fb); r.M = __float_as_uint(fb.w);
    r.wsum = 0.0f; r.chosen = 0.0f;
    r.pd = 0.0f; r.has_pd = false;
    return r;
}

__device__ __forceinline__ void sub_load(Sub& r, const float4* __restrict__ a, const float4* __restrict__ b, size_t i) {
    r = sub_from(a[i], b[i]);
}

__device__ __forceinline__ void sub_store(const Sub& r, float4* __restrict__ a, float4* __restrict__ b,
                                          float2* __restrict__ dbg, size_t i, size_t idbg) {
    a[i] = make_float4(r.pos.x, r.pos.y, r.pos.z, r.W);
    b[i] = make_float4(r.col.x, r.col.y, r.col.z, __uint_as_float(r.M));
    if (dbg) dbg[idbg] = make_float2(r.wsum, r.chosen);
}

// Neighbour (x + dx, y + dy) clamped to the image (render_utils.cpp:109-110), then -- defensively -- to the
// stored view (the host guarantees the view holds every reachable neighbour; this only prevents a fault).
__device__ __forceinline__ size_t neighbour_index(const Region& rg, uint32_t x, uint32_t y, int dx, int dy) {
    int nx = min(max((int)x + dx, 0), (int)rg.W - 1);
    int ny = min(max((int)y + dy, 0), (int)rg.H - 1);
    nx = min(max(nx, (int)rg.vx0), (int)(rg.vx0 + rg.vw) - 1);
    ny = min(max(ny, (int)rg.vy0), (int)(rg.vy0 + rg.vh) - 1);
    return (size_t)(ny - (int)rg.vy0) * rg.vw + (size_t)(nx - (int)rg.vx0);
}

// ---------------------------------------------------------------------------------------------------------
// Work mapping.  Tiles of 32x8 pixels, one 256-lane block each (a wave = 32x2 pixels).
constexpr uint32_t kTileW = 32, kTileH = 8;

__device__ __forceinline__ uint32_t num_tiles(const Region& rg) {
    return ((rg.rw + kTileW - 1) / kTileW) * ((rg.rh + kTileH - 1) / kTileH);
}

__device__ __forceinline__ bool tile_pixel_of(const Region& rg, uint32_t tile, uint32_t& x, uint32_t& y, size_t& p) {
    const uint32_t ntx = (rg.rw + kTileW - 1) / kTileW;
    const uint32_t tx = tile % ntx, ty = tile / ntx;
    if (rg.map2d == 2u) {   // each wave an 8x8 block of the 32x8 tile (a squarer gather footprint per wave)
        const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63u;
        x = rg.rx0 + tx * kTileW + w * 8u + (l & 7u);
        y = rg.ry0 + ty * kTileH + (l >> 3);
    } else {
        x = rg.rx0 + tx * kTileW + threadIdx.x % kTileW;
        y = rg.ry0 + ty * kTileH + threadIdx.x / kTileW;
    }
    if (x >= rg.rx0 + rg.rw || y >= rg.ry0 + rg.rh) return false;
    p = (size_t)(y - rg.vy0) * rg.vw + (x - rg.vx0);
    return true;
}

// Spatial pass: blocks are dealt round-robin over the 8 XCDs (blocks b and b+8 share one --
// MI355X_MICROARCH.md "Workgroup dispatch"), so block b is remapped to give each XCD one contiguous run of
// tiles, i.e. a horizontal band of the image: the rows a neighbourhood gathers then sit in that XCD's L2
// instead of being fetched by all eight (FETCH_SIZE 0.95 GB -> 0.15 GB per 1080p pass, profiles/).
__device__ __forceinline__ uint32_t xcd_banded_tile() {
    const uint32_t nb = gridDim.x, b = blockIdx.x;
    const uint32_t xcd = b % 8u, q = nb / 8u, rem = nb % 8u;
    return xcd * q + min(xcd, rem) + b / 8u;
}

__device__ __forceinline__ bool region_pixel(const Region& rg, uint32_t idx, uint32_t& x, uint32_t& y, size_t& p) {
    if (idx >= rg.rw * rg.rh) return false;
    x = rg.rx0 + idx % rg.rw;
    y = rg.ry0 + idx / rg.rw;
    p = (size_t)(y - rg.vy0) * rg.vw + (x - rg.vx0);
    return true;
}

// Work items of a launch: 32x8 tiles (map2d) or runs of 256 row-major pixels.
__device__ __forceinline__ uint32_t work_items(const Region& rg) {
    return rg.map2d ? num_tiles(rg) : (rg.rw * rg.rh + 255u) / 256u;
}
__device__ __forceinline__ bool work_pixel(const Region& rg, uint32_t item, uint32_t& x, uint32_t& y, size_t& p) {
    return rg.map2d ? tile_pixel_of(rg, item, x, y, p) : region_pixel(rg, item * 256u + threadIdx.x, x, y, p);
}

}  // namespace romis

using namespace romis;

extern __shared__ __attribute__((aligned(16))) float4 g_lds[];

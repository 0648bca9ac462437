/*
 * restir_oracle.c -- TEST INFRASTRUCTURE ONLY: the CPU restatement of the reference ReSTIR path that the
 * parity tests check the HIP kernels against.  See restir_oracle.h for the parity status of each part.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this (via ctypes).
 *
 * Floating point: C11 float arithmetic on x86-64 SSE (FLT_EVAL_METHOD 0), -ffp-contract=off, no fast-math,
 * the exact operation order of glm 0.9.9.9 as the reference instantiates it (pinned by
 * tests/test_oracle_pinning.py against the vendored glm compiled here).
 */
#include "restir_oracle.h"
#include "portable_math.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------------------------------------ */
/* glm 0.9.9.9 primitives (framework/third_party/glm/glm/detail/func_geometric.inl, func_common.inl,       */
/* type_vec3.inl, type_quat.inl).                                                                          */
typedef struct { float x, y, z; } v3;
static inline v3 mk(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
static inline v3 vadd(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vscale(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline v3 vdivs(v3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
/* compute_dot<vec3>: tmp = a * b; tmp.x + tmp.y + tmp.z (func_geometric.inl:48-54) */
static inline float vdot(v3 a, v3 b) { v3 t = vmul(a, b); return (t.x + t.y) + t.z; }
/* length = sqrt(dot(v, v)) (:8-14); distance(p0, p1) = length(p1 - p0) (:17-23) */
static inline float vlength(v3 a) { return sqrtf(vdot(a, a)); }
static inline float vdistance(v3 p0, v3 p1) { return vlength(vsub(p1, p0)); }
/* normalize = v * inversesqrt(dot(v, v)), inversesqrt = 1 / sqrt (func_geometric.inl:82-88,
 * func_exponential.inl:134-139) */
static inline v3 vnormalize(v3 a) { return vscale(a, 1.0f / sqrtf(vdot(a, a))); }
/* mix(x, y, a) = x * (1 - a) + y * a (func_common.inl:104-111) */
static inline v3 vmix(v3 x, v3 y, float a) { return vadd(vscale(x, 1.0f - a), vscale(y, a)); }
/* cross (func_geometric.inl:68-79) */
static inline v3 vcross(v3 x, v3 y) {
    return mk(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
/* quat * vec3 (type_quat.inl:347-354) */
static inline v3 qrotate(const float q[4], v3 v) {
    v3 qv = mk(q[0], q[1], q[2]);
    v3 uv = vcross(qv, v);
    v3 uuv = vcross(qv, uv);
    return vadd(v, vscale(vadd(vscale(uv, q[3]), uuv), 2.0f));
}
static inline int vany_nan(v3 a) { return isnan(a.x) || isnan(a.y) || isnan(a.z); }
static inline v3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
static inline void st3(float* p, v3 v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* ------------------------------------------------------------------------------------------------------ */
/* keyed RNG (restir_c.h header comment)                                                                   */
static inline uint32_t mix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
    return h;
}
uint32_t or_rng_key(uint32_t seed, uint32_t frame, uint32_t stage, uint32_t pass) {
    return mix32(mix32(mix32(seed ^ 0x9E3779B9u) + frame) ^ (stage * 0x01000193u + pass * 0x27D4EB2Fu));
}
static inline uint32_t pix_state(uint32_t key, uint32_t g) { return mix32(key ^ mix32(g * 0x9E3779B1u + 0x7F4A7C15u)); }
static inline uint32_t draw(uint32_t ps, uint32_t slot) { return mix32(ps + slot * 0x9E3779B9u); }
uint32_t or_rng_draw(uint32_t key, uint32_t g, uint32_t slot) { return draw(pix_state(key, g), slot); }

/* rand() stand-in + linearMap(float(rand()), 0, RAND_MAX, 0, 1) (utils.cpp:26-31; reservoir.cpp:24,
 * light.cpp:20,28-29).  RAND_MAX converts to 2147483648.0f as the float parameter domainMax. */
static inline float rand01(uint32_t d) {
    float val = (float)(d >> 1);
    float ratio = (val - 0.0f) / (2147483648.0f - 0.0f);
    float scaled = ratio * (1.0f - 0.0f);
    return scaled + 0.0f;
}
/* uniform_int_distribution<>(0, L-1) (light.cpp:51) / (-r, r) (render_utils.cpp:91) stand-ins */
static inline uint32_t uniform_index(uint32_t d, uint32_t n) { return (uint32_t)(((uint64_t)d * n) >> 32); }
static inline int uniform_offset(uint32_t d, uint32_t r) { return (int)uniform_index(d, 2u * r + 1u) - (int)r; }

/* ------------------------------------------------------------------------------------------------------ */
/* Scene: flat triangle list + material table (+1 miss material) + lights                                 */
struct or_scene {
    uint32_t num_tris;
    float* v0;   /* [T][3] */
    float* e1;   /* v1 - v0 */
    float* e2;   /* v2 - v0 */
    float* n0; float* n1; float* n2;
    uint32_t* mat;
    restir_material* materials;
    uint32_t num_materials;   /* including the miss material at the end */
    restir_light* lights;
    uint32_t num_lights;
};

or_scene* or_scene_create(const restir_mesh* meshes, uint32_t num_meshes, const restir_light* lights,
                          uint32_t num_lights) {
    or_scene* s = (or_scene*)calloc(1, sizeof(or_scene));
    uint32_t T = 0;
    for (uint32_t m = 0; m < num_meshes; m++) T += meshes[m].num_triangles;
    s->num_tris = T;
    size_t n3 = (size_t)(T ? T : 1) * 3;
    s->v0 = (float*)malloc(n3 * 4); s->e1 = (float*)malloc(n3 * 4); s->e2 = (float*)malloc(n3 * 4);
    s->n0 = (float*)malloc(n3 * 4); s->n1 = (float*)malloc(n3 * 4); s->n2 = (float*)malloc(n3 * 4);
    s->mat = (uint32_t*)malloc((T ? T : 1) * 4);
    s->num_materials = num_meshes + 1;
    s->materials = (restir_material*)calloc(s->num_materials, sizeof(restir_material));
    uint32_t t = 0;
    for (uint32_t m = 0; m < num_meshes; m++) {
        const restir_mesh* mesh = &meshes[m];
        s->materials[m] = mesh->material;
        for (uint32_t i = 0; i < mesh->num_triangles; i++, t++) {
            const uint32_t* tri = &mesh->triangles[3 * i];
            v3 a = ld3(&mesh->positions[3 * tri[0]]), b = ld3(&mesh->positions[3 * tri[1]]),
               c = ld3(&mesh->positions[3 * tri[2]]);
            st3(&s->v0[3 * t], a);
            st3(&s->e1[3 * t], vsub(b, a));
            st3(&s->e2[3 * t], vsub(c, a));
            st3(&s->n0[3 * t], ld3(&mesh->normals[3 * tri[0]]));
            st3(&s->n1[3 * t], ld3(&mesh->normals[3 * tri[1]]));
            st3(&s->n2[3 * t], ld3(&mesh->normals[3 * tri[2]]));
            s->mat[t] = m;
        }
    }
    /* HitInfo of a miss: value-initialised RayHit -> Material defaults kd 0, ks 0, shininess 1,
     * transparency 1 (mesh.h:22-27) and a zero normal. */
    restir_material* miss = &s->materials[num_meshes];
    memset(miss, 0, sizeof(*miss));
    miss->shininess = 1.0f;
    miss->transparency = 1.0f;
    s->num_lights = num_lights;
    s->lights = (restir_light*)malloc((num_lights ? num_lights : 1) * sizeof(restir_light));
    if (num_lights) memcpy(s->lights, lights, num_lights * sizeof(restir_light));
    return s;
}

void or_scene_destroy(or_scene* s) {
    if (!s) return;
    free(s->v0); free(s->e1); free(s->e2); free(s->n0); free(s->n1); free(s->n2); free(s->mat);
    free(s->materials); free(s->lights); free(s);
}
uint32_t or_scene_num_triangles(const or_scene* s) { return s->num_tris; }
uint32_t or_scene_miss_material(const or_scene* s) { return s->num_materials - 1; }

/* ------------------------------------------------------------------------------------------------------ */
/* Ray / triangle (replaces Embree 4.3.1 rtcIntersect1 / rtcOccluded1, embree_interface.cpp:58-90;        */
/* UNPINNED).  Moller-Trumbore, no culling, hit iff tnear(0) < t <= tfar; NaN-safe comparisons.            */
static inline int tri_hit(const or_scene* s, uint32_t i, v3 o, v3 d, float tfar, float* t_out, float* u_out,
                          float* v_out) {
    v3 e1 = ld3(&s->e1[3 * i]), e2 = ld3(&s->e2[3 * i]);
    v3 pvec = vcross(d, e2);
    float det = vdot(e1, pvec);
    if (det == 0.0f) return 0;
    float inv = 1.0f / det;
    v3 tvec = vsub(o, ld3(&s->v0[3 * i]));
    float u = vdot(tvec, pvec) * inv;
    if (!(u >= 0.0f && u <= 1.0f)) return 0;
    v3 qvec = vcross(tvec, e1);
    float v = vdot(d, qvec) * inv;
    if (!(v >= 0.0f && u + v <= 1.0f)) return 0;
    float t = vdot(e2, qvec) * inv;
    if (!(t > 0.0f && t <= tfar)) return 0;
    *t_out = t; *u_out = u; *v_out = v;
    return 1;
}

/* closest hit: minimal t, lowest triangle index on ties */
static int closest_hit(const or_scene* s, v3 o, v3 d, float* t, float* u, float* v, uint32_t* tri) {
    int found = 0;
    float bt = FLT_MAX;
    for (uint32_t i = 0; i < s->num_tris; i++) {
        float ti, ui, vi;
        if (tri_hit(s, i, o, d, FLT_MAX, &ti, &ui, &vi) && (!found || ti < bt)) {
            found = 1; bt = ti; *t = ti; *u = ui; *v = vi; *tri = i;
        }
    }
    return found;
}

static int any_hit(const or_scene* s, v3 o, v3 d, float tfar) {
    for (uint32_t i = 0; i < s->num_tris; i++) {
        float ti, ui, vi;
        if (tri_hit(s, i, o, d, tfar, &ti, &ui, &vi)) return 1;
    }
    return 0;
}

/* testVisibilityLightSample (utils.cpp:41-56): P' = P + normalize(y - P) * 1e-3, tfar = distance(P', y). */
static int visible(const or_scene* s, v3 P, v3 y) {
    v3 dir = vnormalize(vsub(y, P));
    v3 P2 = vadd(P, vscale(dir, 1e-3f));   /* SHADOW_RAY_EPSILON (utils.h:16) */
    float tfar = vdistance(P2, y);
    return !any_hit(s, P2, dir, tfar);
}

/* ------------------------------------------------------------------------------------------------------ */
/* Camera (trackball.cpp:20-29 ctor, :75-78 position, :105-114 generateRay; glm::quat(euler) type_quat.inl:208-217) */
void or_camera_derive(const restir_camera* cam, restir_camera_frame* out) {
    float hh = tanf(cam->fovy / 2.0f);
    float hw = cam->aspect * hh;
    float hx = cam->rotation[0] * 0.5f, hy = cam->rotation[1] * 0.5f, hz = cam->rotation[2] * 0.5f;
    float cx = cosf(hx), cy = cosf(hy), cz = cosf(hz);
    float sx = sinf(hx), sy = sinf(hy), sz = sinf(hz);
    float q[4];
    q[3] = cx * cy * cz + sx * sy * sz;
    q[0] = sx * cy * cz - cx * sy * sz;
    q[1] = cx * sy * cz + sx * cy * sz;
    q[2] = cx * cy * sz - sx * sy * cz;
    v3 origin = vadd(ld3(cam->look_at), qrotate(q, mk(0.0f, 0.0f, -cam->distance)));
    st3(out->origin, origin);
    memcpy(out->quat, q, sizeof(q));
    out->half_w = hw;
    out->half_h = hh;
}

static v3 camera_dir(const restir_camera_frame* cam, uint32_t x, uint32_t y, uint32_t W, uint32_t H) {
    float nx = (float)x / (float)W * 2.0f - 1.0f;    /* render_utils.cpp:24-25 */
    float ny = (float)y / (float)H * 2.0f - 1.0f;
    v3 csd = vnormalize(mk(-nx * cam->half_w, ny * cam->half_h, 1.0f));
    return qrotate(cam->quat, csd);
}

/* genPrimaryRayHits (render_utils.cpp:13-34) with closestHit's attribute interpolation
 * (embree_interface.cpp:64-90; rtcInterpolate0 restated as (1-u-v) a0 + u a1 + v a2, UNPINNED). */
void or_primary(const or_scene* s, const restir_camera_frame* cam, uint32_t W, uint32_t H, or_rect view,
                or_rect rect, float* n_t, float* p_mat) {
    v3 o = ld3(cam->origin);
#pragma omp parallel for schedule(guided)
    for (int yy = 0; yy < (int)rect.h; yy++) {
        uint32_t y = rect.y0 + (uint32_t)yy;
        for (uint32_t x = rect.x0; x < rect.x0 + rect.w; x++) {
            size_t p = (size_t)(y - view.y0) * view.w + (x - view.x0);
            v3 d = camera_dir(cam, x, y, W, H);
            float t = FLT_MAX, u = 0.0f, v = 0.0f;
            uint32_t tri = 0;
            v3 n = mk(0.0f, 0.0f, 0.0f);
            uint32_t m = s->num_materials - 1;
            if (closest_hit(s, o, d, &t, &u, &v, &tri)) {
                float w0 = (1.0f - u) - v;
                n = vadd(vadd(vscale(ld3(&s->n0[3 * tri]), w0), vscale(ld3(&s->n1[3 * tri]), u)),
                         vscale(ld3(&s->n2[3 * tri]), v));
                m = s->mat[tri];
            } else {
                t = FLT_MAX;
            }
            v3 P = vadd(o, vscale(d, t));   /* ray.origin + (ray.t * ray.direction) */
            n_t[4 * p + 0] = n.x; n_t[4 * p + 1] = n.y; n_t[4 * p + 2] = n.z; n_t[4 * p + 3] = t;
            p_mat[4 * p + 0] = P.x; p_mat[4 * p + 1] = P.y; p_mat[4 * p + 2] = P.z; p_mat[4 * p + 3] = u2f(m);
        }
    }
}

/* ------------------------------------------------------------------------------------------------------ */
/* Shading / target function                                                                             */
typedef struct {
    v3 P, N, V;      /* V = normalize(o - P) is light-independent (hoisted; same bits) */
    const restir_material* mat;
    float t;
} or_px;

static inline or_px load_px(const or_scene* s, const float* n_t, const float* p_mat, size_t p, v3 origin) {
    or_px r;
    r.N = ld3(&n_t[4 * p]);
    r.t = n_t[4 * p + 3];
    r.P = ld3(&p_mat[4 * p]);
    uint32_t m = f2u(p_mat[4 * p + 3]);
    if (m >= s->num_materials) m = s->num_materials - 1;
    r.mat = &s->materials[m];
    r.V = vnormalize(vsub(origin, r.P));
    return r;
}

/* computeShading (shading.cpp:7-34); diffuseAlbedo = kd (utils.cpp:33-37, no textures carried). */
static v3 shade(const restir_features* f, const or_px* px, v3 lpos, v3 lcol) {
    v3 kd = ld3(px->mat->kd);
    if (!f->enable_shading) return kd;
    v3 L = vnormalize(vsub(lpos, px->P));
    float dotNL = vdot(px->N, L);
    if (dotNL < 0.0f) return mk(0.0f, 0.0f, 0.0f);
    v3 R = vnormalize(vsub(vscale(px->N, 2.0f * dotNL), L));
    float cosTheta = vdot(R, px->V);
    v3 diffuse = vscale(vmul(lcol, kd), dotNL);
    v3 specular = vscale(vmul(lcol, ld3(px->mat->ks)), pm_powf(cosTheta, px->mat->shininess));
    if (vany_nan(diffuse)) diffuse = mk(0.0f, 0.0f, 0.0f);
    if (vany_nan(specular)) specular = mk(0.0f, 0.0f, 0.0f);
    float d = vdistance(px->P, lpos);
    if (fabsf(d) < 1e-5f) d = 1.0f;   /* zeroWithinEpsilon, ZERO_EPSILON (utils.cpp:25, utils.h:19) */
    return vdivs(vadd(diffuse, specular), d * d);
}

/* targetPDF = length(computeShading) (reservoir.cpp:106-109) */
static inline float target_pdf(const restir_features* f, const or_px* px, v3 lpos, v3 lcol) {
    return vlength(shade(f, px, lpos, lcol));
}

float or_target_pdf(const or_scene* s, const restir_features* f, const float origin[3], const float n_t[4],
                    const float p_mat[4], const float lpos[3], const float lcol[3]) {
    or_px px = load_px(s, n_t, p_mat, 0, ld3(origin));
    return target_pdf(f, &px, ld3(lpos), ld3(lcol));
}

/* ------------------------------------------------------------------------------------------------------ */
/* Reservoir (reservoir.h:18-73)                                                                          */
typedef struct {
    v3 pos, col;
    float W;
    uint32_t M;        /* sampleNums (size_t in the reference) */
    float wsum, chosen;
} or_sub;

/* Reservoir(N) ctor (reservoir.h:29-32): M = 1, wSum = FLT_MIN, chosen = 0, sample = 0, W = 0 */
static inline void res_init(or_sub* r, uint32_t N) {
    for (uint32_t j = 0; j < N; j++) {
        r[j].pos = mk(0.0f, 0.0f, 0.0f); r[j].col = mk(0.0f, 0.0f, 0.0f);
        r[j].W = 0.0f; r[j].M = 1u; r[j].wsum = FLT_MIN; r[j].chosen = 0.0f;
    }
}

/* Reservoir::update (reservoir.cpp:10-32) with u = the draw for this call. */
static inline uint32_t res_update(or_sub* r, uint32_t N, v3 pos, v3 col, float w, float u) {
    uint32_t k = 0;
    float best = FLT_MAX;
    for (uint32_t j = 0; j < N; j++) {
        if (r[j].wsum < best) { k = j; best = r[j].wsum; }
    }
    r[k].M += 1u;
    r[k].wsum += w;
    if (u < (w / r[k].wsum)) { r[k].pos = pos; r[k].col = col; r[k].chosen = w; }
    return k;
}

static inline void res_load(or_sub* r, uint32_t N, const float* a, const float* b, size_t p, size_t npx) {
    for (uint32_t j = 0; j < N; j++) {
        const float* pa = &a[4 * (j * npx + p)];
        const float* pb = &b[4 * (j * npx + p)];
        r[j].pos = ld3(pa); r[j].W = pa[3];
        r[j].col = ld3(pb); r[j].M = f2u(pb[3]);
        r[j].wsum = 0.0f; r[j].chosen = 0.0f;
    }
}

static inline void res_store(const or_sub* r, uint32_t N, float* a, float* b, float* dbg, size_t p, size_t npx) {
    for (uint32_t j = 0; j < N; j++) {
        float* pa = &a[4 * (j * npx + p)];
        float* pb = &b[4 * (j * npx + p)];
        st3(pa, r[j].pos); pa[3] = r[j].W;
        st3(pb, r[j].col); pb[3] = u2f(r[j].M);
        if (dbg) { dbg[2 * (j * npx + p)] = r[j].wsum; dbg[2 * (j * npx + p) + 1] = r[j].chosen; }
    }
}

/* W = (1/p) * (1/M) * wSum, p == 0 -> 0 (light.cpp:90-93, reservoir.cpp:61-64) */
static inline float contribution_weight(float p, uint32_t M, float wsum) {
    if (p == 0.0f) return 0.0f;
    return ((1.0f / p) * (1.0f / (float)M)) * wsum;
}

/* ------------------------------------------------------------------------------------------------------ */
/* genCanonicalSamples (light.cpp:39-99) over rect, via genInitialSamples (render_utils.cpp:36-52).       */
void or_ris(const or_scene* s, const restir_features* f, uint32_t key, const float origin_[3], uint32_t W,
            uint32_t H, or_rect view, or_rect rect, const float* n_t, const float* p_mat, float* res_a,
            float* res_b, float* res_dbg) {
    (void)H;
    const uint32_t N = f->num_samples_in_reservoir;
    const size_t npx = (size_t)view.w * view.h;
    const v3 origin = ld3(origin_);
    const uint32_t L = s->num_lights;
#pragma omp parallel for schedule(guided)
    for (int yy = 0; yy < (int)rect.h; yy++) {
        uint32_t y = rect.y0 + (uint32_t)yy;
        or_sub r[RESTIR_MAX_N];
        for (uint32_t x = rect.x0; x < rect.x0 + rect.w; x++) {
            size_t p = (size_t)(y - view.y0) * view.w + (x - view.x0);
            res_init(r, N);
            if (L != 0) {
                or_px px = load_px(s, n_t, p_mat, p, origin);
                uint32_t ps = pix_state(key, y * W + x);
                for (uint32_t j = 0; j < N; j++) r[j].M = 0u;   /* light.cpp:58-60 */
                for (uint32_t c = 0; c < f->initial_light_samples; c++) {
                    const restir_light* light = &s->lights[uniform_index(draw(ps, 4u * c), L)];
                    v3 pos, col;
                    if (light->type == RESTIR_LIGHT_POINT) {
                        pos = ld3(light->p0); col = ld3(light->c0);
                    } else if (light->type == RESTIR_LIGHT_SEGMENT) {
                        /* sampleSegmentLight (light.cpp:19-23) */
                        float fr = rand01(draw(ps, 4u * c + 1u));
                        pos = vmix(ld3(light->p0), ld3(light->p1), fr);
                        col = vmix(ld3(light->c0), ld3(light->c1), fr);
                    } else {
                        /* sampleParallelogramLight (light.cpp:27-34) */
                        float a = rand01(draw(ps, 4u * c + 1u));
                        float b = rand01(draw(ps, 4u * c + 2u));
                        pos = vadd(vadd(ld3(light->p0), vscale(ld3(light->p1), a)), vscale(ld3(light->p2), b));
                        v3 l01 = vmix(ld3(light->c0), ld3(light->c1), a);
                        v3 l23 = vmix(ld3(light->c2), ld3(light->c3), a);
                        col = vmix(l01, l23, b);
                    }
                    float w = target_pdf(f, &px, pos, col) / (1.0f / (float)L);   /* light.cpp:80 */
                    res_update(r, N, pos, col, w, rand01(draw(ps, 4u * c + 3u)));
                }
                for (uint32_t j = 0; j < N; j++) {   /* light.cpp:85-95 */
                    if (f->initial_samples_visibility_check && !visible(s, px.P, r[j].pos)) {
                        r[j].W = 0.0f;
                    } else {
                        r[j].W = contribution_weight(target_pdf(f, &px, r[j].pos, r[j].col), r[j].M, r[j].wsum);
                    }
                }
            }
            res_store(r, N, res_a, res_b, res_dbg, p, npx);
        }
    }
}

/* ------------------------------------------------------------------------------------------------------ */
/* Reservoir::combineBiased (reservoir.cpp:40-66) into `out` (already initialised with Reservoir(N)).     */
static void combine_biased(const restir_features* f, const or_px* cur, const or_sub* stream, uint32_t nres,
                           uint32_t N, or_sub* out, uint32_t ps, uint32_t slot0) {
    uint32_t macc[RESTIR_MAX_N];
    for (uint32_t j = 0; j < N; j++) macc[j] = 0u;
    uint32_t t = 0;
    for (uint32_t i = 0; i < nres; i++) {
        for (uint32_t j = 0; j < N; j++) {
            const or_sub* in = &stream[i * N + j];
            float p = target_pdf(f, cur, in->pos, in->col);
            float w = (p * in->W) * (float)in->M;
            uint32_t k = res_update(out, N, in->pos, in->col, w, rand01(draw(ps, slot0 + t)));
            t++;
            macc[k] += in->M;
        }
    }
    for (uint32_t j = 0; j < N; j++) out[j].M = macc[j];
    for (uint32_t j = 0; j < N; j++)
        out[j].W = contribution_weight(target_pdf(f, cur, out[j].pos, out[j].col), out[j].M, out[j].wsum);
}

/* temporalReuse (render_utils.cpp:142-177) */
void or_temporal(const or_scene* s, const restir_features* f, uint32_t key, const float origin_[3], uint32_t W,
                 uint32_t H, or_rect view, or_rect rect, const float* n_t, const float* p_mat,
                 const float* cur_a, const float* cur_b, const float* prev_a, const float* prev_b,
                 float* out_a, float* out_b, float* out_dbg) {
    (void)H;
    const uint32_t N = f->num_samples_in_reservoir;
    const size_t npx = (size_t)view.w * view.h;
    const v3 origin = ld3(origin_);
#pragma omp parallel for schedule(guided)
    for (int yy = 0; yy < (int)rect.h; yy++) {
        uint32_t y = rect.y0 + (uint32_t)yy;
        or_sub stream[2 * RESTIR_MAX_N];
        or_sub out[RESTIR_MAX_N];
        for (uint32_t x = rect.x0; x < rect.x0 + rect.w; x++) {
            size_t p = (size_t)(y - view.y0) * view.w + (x - view.x0);
            or_px px = load_px(s, n_t, p_mat, p, origin);
            res_load(&stream[0], N, cur_a, cur_b, p, npx);
            res_load(&stream[N], N, prev_a, prev_b, p, npx);
            uint64_t mcur = 0, mprev = 0;
            for (uint32_t j = 0; j < N; j++) { mcur += stream[j].M; mprev += stream[N + j].M; }
            uint64_t C = (uint64_t)f->temporal_clamp_m * mcur + 1u;
            if (mprev > C) {
                for (uint32_t j = 0; j < N; j++) {
                    if (stream[N + j].M == 0u) continue;
                    /* wSums[j] *= C / M (integer division) has no effect on the output: combineBiased
                     * never reads an input's wSum. */
                    stream[N + j].M = (uint32_t)C;
                }
            }
            res_init(out, N);
            combine_biased(f, &px, stream, 2, N, out, pix_state(key, y * W + x), 0u);
            res_store(out, N, out_a, out_b, out_dbg, p, npx);
        }
    }
}

/* spatialReuse, one pass (render_utils.cpp:96-139) */
int or_spatial_pass(const or_scene* s, const restir_features* f, uint32_t key, const float origin_[3], uint32_t W,
                    uint32_t H, or_rect view, or_rect rect, const float* n_t, const float* p_mat,
                    const float* in_a, const float* in_b, float* out_a, float* out_b, float* out_dbg) {
    const uint32_t N = f->num_samples_in_reservoir;
    const uint32_t K = f->num_neighbours_to_sample;
    const uint32_t R = f->spatial_resample_radius;
    const size_t npx = (size_t)view.w * view.h;
    const v3 origin = ld3(origin_);
    int bad = 0;
#pragma omp parallel for schedule(guided) reduction(| : bad)
    for (int yy = 0; yy < (int)rect.h; yy++) {
        uint32_t y = rect.y0 + (uint32_t)yy;
        or_sub* stream = (or_sub*)malloc(sizeof(or_sub) * (size_t)(K + 1) * N);
        size_t* where = (size_t*)malloc(sizeof(size_t) * (K + 1));
        or_sub out[RESTIR_MAX_N];
        for (uint32_t x = rect.x0; x < rect.x0 + rect.w; x++) {
            size_t p = (size_t)(y - view.y0) * view.w + (x - view.x0);
            or_px cur = load_px(s, n_t, p_mat, p, origin);
            uint32_t ps = pix_state(key, y * W + x);
            uint32_t nsel = 0;
            for (uint32_t n = 0; n < K; n++) {
                int nx = (int)x + uniform_offset(draw(ps, 2u * n), R);
                int ny = (int)y + uniform_offset(draw(ps, 2u * n + 1u), R);
                nx = nx < 0 ? 0 : (nx > (int)W - 1 ? (int)W - 1 : nx);   /* std::clamp to the image */
                ny = ny < 0 ? 0 : (ny > (int)H - 1 ? (int)H - 1 : ny);
                if (nx < (int)view.x0 || nx >= (int)(view.x0 + view.w) || ny < (int)view.y0 ||
                    ny >= (int)(view.y0 + view.h)) { bad = 1; continue; }
                size_t q = (size_t)(ny - (int)view.y0) * view.w + (size_t)(nx - (int)view.x0);
                if (!f->unbiased_combination) {   /* render_utils.cpp:114-118 */
                    float tn = n_t[4 * q + 3];
                    float depthFracDiff = fabsf(1.0f - (tn / cur.t));
                    float normalsDotProd = vdot(ld3(&n_t[4 * q]), cur.N);
                    if (depthFracDiff > 0.1f || normalsDotProd < 0.90630778703f) continue;
                }
                res_load(&stream[nsel * N], N, in_a, in_b, q, npx);
                where[nsel] = q;
                nsel++;
            }
            res_load(&stream[nsel * N], N, in_a, in_b, p, npx);   /* current last (:124) */
            where[nsel] = p;
            nsel++;
            res_init(out, N);
            const uint32_t slot0 = 2u * K;
            if (!f->unbiased_combination) {
                combine_biased(f, &cur, stream, nsel, N, out, ps, slot0);
            } else {
                /* Reservoir::combineUnbiased (reservoir.cpp:68-104) */
                uint32_t macc[RESTIR_MAX_N];
                for (uint32_t j = 0; j < N; j++) macc[j] = 0u;
                uint32_t t = 0;
                for (uint32_t i = 0; i < nsel; i++) {
                    for (uint32_t j = 0; j < N; j++) {
                        const or_sub* in = &stream[i * N + j];
                        float pd = target_pdf(f, &cur, in->pos, in->col);
                        float w = (pd * in->W) * (float)in->M;
                        uint32_t k = res_update(out, N, in->pos, in->col, w, rand01(draw(ps, slot0 + t)));
                        t++;
                        macc[k] += in->M;
                    }
                }
                for (uint32_t j = 0; j < N; j++) out[j].M = macc[j];
                uint64_t Z[RESTIR_MAX_N];
                for (uint32_t j = 0; j < N; j++) Z[j] = 0u;
                for (uint32_t i = 0; i < nsel; i++) {
                    or_px rp = load_px(s, n_t, p_mat, where[i], origin);
                    uint64_t tot = 0;
                    for (uint32_t j = 0; j < N; j++) tot += stream[i * N + j].M;
                    for (uint32_t j = 0; j < N; j++) {
                        float pd = target_pdf(f, &rp, out[j].pos, out[j].col);
                        if (f->spatial_reuse_visibility_check) pd *= visible(s, rp.P, out[j].pos) ? 1.0f : 0.0f;
                        if (pd > 0.0f) Z[j] += tot;
                    }
                }
                for (uint32_t j = 0; j < N; j++) {
                    float pc = target_pdf(f, &cur, out[j].pos, out[j].col);
                    if (pc == 0.0f || Z[j] == 0u) out[j].W = 0.0f;
                    else out[j].W = ((1.0f / pc) * (1.0f / (float)Z[j])) * out[j].wsum;
                }
            }
            res_store(out, N, out_a, out_b, out_dbg, p, npx);
        }
        free(stream);
        free(where);
    }
    return bad ? -1 : 0;
}

/* ------------------------------------------------------------------------------------------------------ */
/* exposureToneMapping (tone_mapping.cpp:8-11) */
static v3 tonemap(v3 c, float exposure, float gamma) {
    v3 e = vscale(mk(-c.x, -c.y, -c.z), exposure);
    v3 mapped = mk(1.0f - pm_expf(e.x), 1.0f - pm_expf(e.y), 1.0f - pm_expf(e.z));
    float g = 1.0f / gamma;
    return mk(pm_powf(mapped.x, g), pm_powf(mapped.y, g), pm_powf(mapped.z, g));
}
void or_tonemap(const float c[3], float exposure, float gamma, float out[3]) {
    st3(out, tonemap(ld3(c), exposure, gamma));
}

/* final loop of renderReSTIR (render.cpp:45-57) + finalShading (render_utils.cpp:54-65) + setPixel y-flip
 * (screen.cpp:37-43) */
void or_final(const or_scene* s, const restir_features* f, const float origin_[3], uint32_t W, uint32_t H,
              or_rect view, or_rect rect, const float* n_t, const float* p_mat, const float* res_a,
              const float* res_b, float* rgb) {
    (void)W; (void)H;
    const uint32_t N = f->num_samples_in_reservoir;
    const size_t npx = (size_t)view.w * view.h;
    const v3 origin = ld3(origin_);
#pragma omp parallel for schedule(guided)
    for (int yy = 0; yy < (int)rect.h; yy++) {
        uint32_t y = rect.y0 + (uint32_t)yy;
        or_sub r[RESTIR_MAX_N];
        for (uint32_t x = rect.x0; x < rect.x0 + rect.w; x++) {
            size_t p = (size_t)(y - view.y0) * view.w + (x - view.x0);
            or_px px = load_px(s, n_t, p_mat, p, origin);
            res_load(r, N, res_a, res_b, p, npx);
            v3 color = mk(0.0f, 0.0f, 0.0f);
            for (uint32_t j = 0; j < N; j++) {
                v3 sc = visible(s, px.P, r[j].pos) ? shade(f, &px, r[j].pos, r[j].col) : mk(0.0f, 0.0f, 0.0f);
                sc = vscale(sc, r[j].W);
                color = vadd(color, sc);
            }
            color = vdivs(color, (float)N);
            if (f->enable_tone_mapping) color = tonemap(color, f->exposure, f->gamma);
            size_t row = (size_t)(rect.h - 1u - (uint32_t)yy);   /* row 0 = top of rect */
            st3(&rgb[3 * (row * rect.w + (x - rect.x0))], color);
        }
    }
}

/* ------------------------------------------------------------------------------------------------------ */
int or_render_frame(const or_scene* s, const restir_camera* cam, const restir_features* f, uint32_t seed,
                    uint32_t frame, uint32_t W, uint32_t H, or_rect view, or_rect rect, const float* prev_a,
                    const float* prev_b, float* n_t, float* p_mat, float* out_a, float* out_b, float* rgb,
                    int threads) {
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
    const uint32_t N = f->num_samples_in_reservoir;
    if (N == 0 || N > RESTIR_MAX_N) return -2;
    const size_t n4 = (size_t)view.w * view.h * N * 4;
    restir_camera_frame cf;
    or_camera_derive(cam, &cf);
    or_primary(s, &cf, W, H, view, view, n_t, p_mat);
    or_ris(s, f, or_rng_key(seed, frame, RESTIR_STAGE_RIS, 0), cf.origin, W, H, view, view, n_t, p_mat,
           out_a, out_b, NULL);
    float* ta = (float*)malloc(n4 * 4);
    float* tb = (float*)malloc(n4 * 4);
    int rc = 0;
    if (f->temporal_reuse && prev_a && prev_b) {
        or_temporal(s, f, or_rng_key(seed, frame, RESTIR_STAGE_TEMPORAL, 0), cf.origin, W, H, view, view, n_t,
                    p_mat, out_a, out_b, prev_a, prev_b, ta, tb, NULL);
        memcpy(out_a, ta, n4 * 4);
        memcpy(out_b, tb, n4 * 4);
    }
    if (f->spatial_reuse) {
        for (uint32_t pass = 0; pass < f->spatial_resampling_passes; pass++) {
            /* pass p must be valid on rect grown by (P-1-p) r (ghost zones; whole view when rect == view) */
            uint32_t g = (f->spatial_resampling_passes - 1u - pass) * f->spatial_resample_radius;
            uint32_t x0 = rect.x0 > view.x0 + g ? rect.x0 - g : view.x0;
            uint32_t y0 = rect.y0 > view.y0 + g ? rect.y0 - g : view.y0;
            uint32_t x1 = rect.x0 + rect.w + g < view.x0 + view.w ? rect.x0 + rect.w + g : view.x0 + view.w;
            uint32_t y1 = rect.y0 + rect.h + g < view.y0 + view.h ? rect.y0 + rect.h + g : view.y0 + view.h;
            or_rect pr = {x0, y0, x1 - x0, y1 - y0};
            memcpy(ta, out_a, n4 * 4);
            memcpy(tb, out_b, n4 * 4);
            if (or_spatial_pass(s, f, or_rng_key(seed, frame, RESTIR_STAGE_SPATIAL, pass), cf.origin, W, H, view,
                                pr, n_t, p_mat, ta, tb, out_a, out_b, NULL) != 0)
                rc = -1;
        }
    }
    free(ta);
    free(tb);
    or_final(s, f, cf.origin, W, H, view, rect, n_t, p_mat, out_a, out_b, rgb);
    return rc;
}

/* ------------------------------------------------------------------------------------------------------ */
void or_glm_probe(const float a_[3], const float b_[3], float t, const float e[3], float out[24]) {
    v3 a = ld3(a_), b = ld3(b_);
    restir_camera cam;
    memset(&cam, 0, sizeof(cam));
    cam.rotation[0] = e[0]; cam.rotation[1] = e[1]; cam.rotation[2] = e[2];
    cam.fovy = 1.0f; cam.aspect = 1.0f;
    restir_camera_frame cf;
    or_camera_derive(&cam, &cf);
    memcpy(&out[0], cf.quat, 16);
    st3(&out[4], vnormalize(a));
    out[7] = vdot(a, b);
    out[8] = vlength(a);
    out[9] = vdistance(a, b);
    st3(&out[10], vcross(a, b));
    st3(&out[13], vmix(a, b, t));
    st3(&out[16], qrotate(cf.quat, b));
    out[19] = 0.0f;
}
float or_powf(float x, float y) { return pm_powf(x, y); }
float or_expf(float x) { return pm_expf(x); }

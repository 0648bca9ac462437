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

/* CPU-baseline timing mode (or_set_rng_mode(1)): the reference's own generators (oracle/ref_rng.cpp --
 * per-pixel std::random_device + std::mt19937 + uniform_int_distribution, process-wide rand()) replace the keyed
 * draws at the same call sites.  Not reproducible, never used for parity: bench.py times it beside the keyed mode. */
void or_refrng_pixel_seed(void);
int or_refrng_uniform(int lo, int hi);
void or_refrng_shared_seed(void);
int or_refrng_shared_uniform(int lo, int hi);
float or_refrng_rand01(void);
static int g_ref_rng = 0;
void or_set_rng_mode(int mode) { g_ref_rng = mode != 0; }
#define U01(ps, slot) (g_ref_rng ? or_refrng_rand01() : rand01(draw((ps), (slot))))

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
    /* textures (Material::kdTexture images) and per-triangle texture coordinates t0, t1, t2 ([T][2] each) */
    uint32_t num_textures;
    uint32_t* tex_w; uint32_t* tex_h;
    float** tex_rgb;
    float* tc0; float* tc1; float* tc2;
    /* the G-buffer's texCoord plane of the following stage calls (or_scene_bind_uv), indexed like n_t / p_mat */
    const float* uv;
};

or_scene* or_scene_create_textured(const restir_mesh* meshes, uint32_t num_meshes, const restir_light* lights,
                                   uint32_t num_lights, const restir_texture* textures, uint32_t num_textures) {
    or_scene* s = (or_scene*)calloc(1, sizeof(or_scene));
    s->num_textures = num_textures;
    s->tex_w = (uint32_t*)calloc(num_textures ? num_textures : 1, 4);
    s->tex_h = (uint32_t*)calloc(num_textures ? num_textures : 1, 4);
    s->tex_rgb = (float**)calloc(num_textures ? num_textures : 1, sizeof(float*));
    for (uint32_t i = 0; i < num_textures; i++) {
        const size_t n = (size_t)textures[i].width * textures[i].height * 3;
        s->tex_w[i] = textures[i].width;
        s->tex_h[i] = textures[i].height;
        s->tex_rgb[i] = (float*)malloc((n ? n : 1) * 4);
        if (n) memcpy(s->tex_rgb[i], textures[i].rgb, n * 4);
    }
    uint32_t T = 0;
    for (uint32_t m = 0; m < num_meshes; m++) T += meshes[m].num_triangles;
    s->num_tris = T;
    size_t n3 = (size_t)(T ? T : 1) * 3;
    s->v0 = (float*)malloc(n3 * 4); s->e1 = (float*)malloc(n3 * 4); s->e2 = (float*)malloc(n3 * 4);
    s->n0 = (float*)malloc(n3 * 4); s->n1 = (float*)malloc(n3 * 4); s->n2 = (float*)malloc(n3 * 4);
    s->mat = (uint32_t*)malloc((T ? T : 1) * 4);
    size_t n2 = (size_t)(T ? T : 1) * 2;
    s->tc0 = (float*)calloc(n2, 4); s->tc1 = (float*)calloc(n2, 4); s->tc2 = (float*)calloc(n2, 4);
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
            if (mesh->texcoords)
                for (int k = 0; k < 2; k++) {
                    s->tc0[2 * t + k] = mesh->texcoords[2 * tri[0] + k];
                    s->tc1[2 * t + k] = mesh->texcoords[2 * tri[1] + k];
                    s->tc2[2 * t + k] = mesh->texcoords[2 * tri[2] + k];
                }
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

or_scene* or_scene_create(const restir_mesh* meshes, uint32_t num_meshes, const restir_light* lights,
                          uint32_t num_lights) {
    return or_scene_create_textured(meshes, num_meshes, lights, num_lights, NULL, 0);
}

void or_scene_bind_uv(or_scene* s, const float* uv) { s->uv = uv; }

void or_scene_destroy(or_scene* s) {
    if (!s) return;
    for (uint32_t i = 0; i < s->num_textures; i++) free(s->tex_rgb[i]);
    free(s->tex_w); free(s->tex_h); free(s->tex_rgb); free(s->tc0); free(s->tc1); free(s->tc2);
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
void or_primary_uv(const or_scene* s, const restir_camera_frame* cam, uint32_t W, uint32_t H, or_rect view,
                   or_rect rect, float* n_t, float* p_mat, float* uv) {
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
            float tc[2] = {0.0f, 0.0f};   /* a miss keeps the value-initialised HitInfo::texCoord */
            uint32_t m = s->num_materials - 1;
            if (closest_hit(s, o, d, &t, &u, &v, &tri)) {
                float w0 = (1.0f - u) - v;
                n = vadd(vadd(vscale(ld3(&s->n0[3 * tri]), w0), vscale(ld3(&s->n1[3 * tri]), u)),
                         vscale(ld3(&s->n2[3 * tri]), v));
                /* texCoord: rtcInterpolate0 of vertex attribute slot 1 (embree_interface.cpp:80-81), the same
                 * (1-u-v) t0 + u t1 + v t2 form as the normal */
                for (int k = 0; k < 2; k++)
                    tc[k] = (s->tc0[2 * tri + k] * w0 + s->tc1[2 * tri + k] * u) + s->tc2[2 * tri + k] * v;
                m = s->mat[tri];
            } else {
                t = FLT_MAX;
            }
            v3 P = vadd(o, vscale(d, t));   /* ray.origin + (ray.t * ray.direction) */
            n_t[4 * p + 0] = n.x; n_t[4 * p + 1] = n.y; n_t[4 * p + 2] = n.z; n_t[4 * p + 3] = t;
            p_mat[4 * p + 0] = P.x; p_mat[4 * p + 1] = P.y; p_mat[4 * p + 2] = P.z; p_mat[4 * p + 3] = u2f(m);
            if (uv) { uv[2 * p] = tc[0]; uv[2 * p + 1] = tc[1]; }
        }
    }
}

void or_primary(const or_scene* s, const restir_camera_frame* cam, uint32_t W, uint32_t H, or_rect view,
                or_rect rect, float* n_t, float* p_mat) {
    or_primary_uv(s, cam, W, H, view, rect, n_t, p_mat, NULL);
}

/* acquireTexel (texture.cpp:4-9): size_t discreteX = texCoord.x * (width - 1) -- the float product truncated
 * toward zero -- and memoryLoc = discreteY * width + discreteX into the row-major pixels.  Products outside
 * [0, width - 1] read out of bounds in the reference (UB); they clamp to the edge texel here. */
static inline uint32_t texel_index(float c, uint32_t n) {
    float v = c * (float)((int)n - 1);
    if (!(v >= 0.0f)) return 0u;
    if (v >= (float)(n - 1)) return n - 1;
    return (uint32_t)v;
}
static const float* acquire_texel(const or_scene* s, uint32_t tex, const float* tc) {
    uint32_t w = s->tex_w[tex], h = s->tex_h[tex];
    size_t loc = (size_t)texel_index(tc[1], h) * w + texel_index(tc[0], w);
    return &s->tex_rgb[tex][3 * loc];
}
void or_acquire_texel(const or_scene* s, uint32_t tex, const float tc[2], float out[3]) {
    const float* t = acquire_texel(s, tex, tc);
    out[0] = t[0]; out[1] = t[1]; out[2] = t[2];
}

/* ------------------------------------------------------------------------------------------------------ */
/* Shading / target function                                                                             */
typedef struct {
    v3 P, N, V;      /* V = normalize(o - P) is light-independent (hoisted; same bits) */
    const restir_material* mat;
    float t;
    const float* texel;   /* acquireTexel at the hit's texCoord when the material has a kdTexture, else NULL */
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
    r.texel = NULL;
    if (s->uv && r.mat->kd_texture && r.mat->kd_texture <= s->num_textures)
        r.texel = acquire_texel(s, r.mat->kd_texture - 1u, &s->uv[2 * p]);
    return r;
}

/* computeShading (shading.cpp:7-34); diffuseAlbedo (utils.cpp:33-37): the texel when texture mapping is on
 * and the material has a kdTexture, else kd.  With shading off the reference returns material.kd itself. */
static v3 shade(const restir_features* f, const or_px* px, v3 lpos, v3 lcol) {
    if (!f->enable_shading) return ld3(px->mat->kd);
    v3 kd = (f->enable_texture_mapping && px->texel) ? ld3(px->texel) : ld3(px->mat->kd);
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
                if (g_ref_rng) or_refrng_pixel_seed();   /* light.cpp:49-51 */
                for (uint32_t j = 0; j < N; j++) r[j].M = 0u;   /* light.cpp:58-60 */
                for (uint32_t c = 0; c < f->initial_light_samples; c++) {
                    const uint32_t li = g_ref_rng ? (uint32_t)or_refrng_uniform(0, (int)L - 1) : uniform_index(draw(ps, 4u * c), L);
                    const restir_light* light = &s->lights[li];
                    v3 pos, col;
                    if (light->type == RESTIR_LIGHT_POINT) {
                        pos = ld3(light->p0); col = ld3(light->c0);
                    } else if (light->type == RESTIR_LIGHT_SEGMENT) {
                        /* sampleSegmentLight (light.cpp:19-23) */
                        float fr = U01(ps, 4u * c + 1u);
                        pos = vmix(ld3(light->p0), ld3(light->p1), fr);
                        col = vmix(ld3(light->c0), ld3(light->c1), fr);
                    } else {
                        /* sampleParallelogramLight (light.cpp:27-34) */
                        float a = U01(ps, 4u * c + 1u);
                        float b = U01(ps, 4u * c + 2u);
                        pos = vadd(vadd(ld3(light->p0), vscale(ld3(light->p1), a)), vscale(ld3(light->p2), b));
                        v3 l01 = vmix(ld3(light->c0), ld3(light->c1), a);
                        v3 l23 = vmix(ld3(light->c2), ld3(light->c3), a);
                        col = vmix(l01, l23, b);
                    }
                    float w = target_pdf(f, &px, pos, col) / (1.0f / (float)L);   /* light.cpp:80 */
                    res_update(r, N, pos, col, w, U01(ps, 4u * c + 3u));
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
            uint32_t k = res_update(out, N, in->pos, in->col, w, U01(ps, slot0 + t));
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
    if (g_ref_rng) or_refrng_shared_seed();
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
            for (uint32_t n = 0; n < K; n++) {   /* the shared generator of render_utils.cpp:89-91 */
                int nx = (int)x + (g_ref_rng ? or_refrng_shared_uniform(-(int)R, (int)R) : uniform_offset(draw(ps, 2u * n), R));
                int ny = (int)y + (g_ref_rng ? or_refrng_shared_uniform(-(int)R, (int)R) : uniform_offset(draw(ps, 2u * n + 1u), R));
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
                        uint32_t k = res_update(out, N, in->pos, in->col, w, U01(ps, slot0 + t));
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
    /* textured scenes: the G-buffer's texCoord plane, bound for every stage of the frame */
    float* uv = s->num_textures ? (float*)calloc((size_t)view.w * view.h * 2, 4) : NULL;
    const float* bound = s->uv;
    or_primary_uv(s, &cf, W, H, view, view, n_t, p_mat, uv);
    if (uv) ((or_scene*)s)->uv = uv;
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
    ((or_scene*)s)->uv = bound;
    free(uv);
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
void or_powf_n(const float* x, const float* y, float* out, size_t n) {
    for (size_t i = 0; i < n; i++) out[i] = pm_powf(x[i], y[i]);
}
void or_expf_n(const float* x, float* out, size_t n) {
    for (size_t i = 0; i < n; i++) out[i] = pm_expf(x[i]);
}

/* ====================================================================================================== */
/* R-MIS / R-OMIS (render.cpp:64-265, render_utils.cpp:68-85 / 179-257, neighbour_selection.cpp:7-122,     */
/* render_utils.h:52).  Whole images only: grids are [H][W] row-major, pixel index p = y * W + x.           */

/* HitInfo::geometryId: the mesh index (rtcAttachGeometry order, embree_interface.cpp:46-47, one material per
 * mesh); a primary miss keeps the value-initialised HitInfo of genPrimaryRayHits (render_utils.cpp:15): 0. */
static inline uint32_t geom_id(const or_scene* s, const float* p_mat, size_t p) {
    uint32_t m = f2u(p_mat[4 * p + 3]);
    return m + 1u >= s->num_materials ? 0u : m;
}

/* areSimilar (neighbour_selection.cpp:7-22), lhs = the canonical pixel, rhs = the neighbour.  The normal test
 * compares the dot product with the RADIANS field (maxDiffCos is computed and unused), as the reference does. */
static int are_similar(const or_scene* s, const restir_features* f, const float* n_t, const float* p_mat, size_t l,
                       size_t r) {
    if (f->neighbour_same_geometry && geom_id(s, p_mat, l) != geom_id(s, p_mat, r)) return 0;
    float depthFracDiff = fabsf(1.0f - (n_t[4 * l + 3] / n_t[4 * r + 3]));
    if (depthFracDiff > f->neighbour_max_depth_difference_fraction) return 0;
    float normalsDotProd = vdot(ld3(&n_t[4 * l]), ld3(&n_t[4 * r]));
    if (normalsDotProd < f->neighbour_max_normal_angle_difference_radians) return 0;
    return 1;
}

typedef struct { int x0, y0, x1, y1; } or_win;

/* Walk pixel p's window in indicesSimilarity's order (y outer, x inner, the pixel itself skipped) and append the
 * members of one class (similar = 1 / dissimilar = 0): all of them, or std::sample's selection sampling of
 * `want` of the class's `len` members (member i is kept iff U{0..len-1-i}, keyed slot i, < the number still
 * needed; the walk stops when none is needed). */
static uint32_t emit_class(const or_scene* s, const restir_features* f, const float* n_t, const float* p_mat,
                           uint32_t W, or_win w, size_t p, int cls, uint64_t len, uint64_t want, int take_all,
                           uint32_t ps, uint32_t* out, size_t npx, uint32_t n) {
    uint64_t needed = take_all ? len : (want < len ? want : len);
    uint64_t i = 0;
    for (int ny = w.y0; ny <= w.y1 && needed; ny++) {
        for (int nx = w.x0; nx <= w.x1 && needed; nx++) {
            size_t q = (size_t)ny * W + (size_t)nx;
            if (q == p || are_similar(s, f, n_t, p_mat, p, q) != cls) continue;
            int keep = take_all || uniform_index(draw(ps, (uint32_t)i), (uint32_t)(len - i)) < needed;
            if (keep) { out[(size_t)(1u + n) * npx + p] = (uint32_t)q; n++; needed--; }
            i++;
        }
    }
    return n;
}

uint32_t or_mis_capacity(const restir_features* f, uint32_t W, uint32_t H) {
    uint32_t k1 = f->num_neighbours_to_sample + 1u;
    if (f->neighbour_selection_strategy == RESTIR_NEIGHBOURS_RANDOM ||
        f->neighbour_selection_strategy == RESTIR_NEIGHBOURS_SIMILAR)
        return k1;
    uint64_t side = 2ull * f->spatial_resample_radius + 1ull;
    uint64_t win = (side < W ? side : W) * (side < H ? side : H);
    return win > k1 ? (uint32_t)win : k1;
}

/* generateResampleIndicesGrid (neighbour_selection.cpp:107-122): nbr[0][p] = neighbourhood size, nbr[1 + i][p] =
 * its i-th pixel (the pixel itself first).  indicesRandom (:24-43): candidate n draws x then y uniformly in the
 * clamped window; indicesSimilarity (:45-105): the similar / dissimilar classes of the window, sampled per the
 * strategy -- including the reference's size arithmetic (Dissimilar takes `k - similar.size()` of the similar
 * class as size_t, i.e. all of them when that wraps; EqualSimilarDissimilar in uint32_t). */
void or_neighbours(const or_scene* s, const restir_features* f, uint32_t key_similar, uint32_t key_dissimilar,
                   uint32_t W, uint32_t H, const float* n_t, const float* p_mat, uint32_t cap, uint32_t* nbr) {
    const size_t npx = (size_t)W * H;
    const uint32_t k = f->num_neighbours_to_sample;
    const int rc = (int)f->spatial_resample_radius;
#pragma omp parallel for schedule(guided)
    for (int yy = 0; yy < (int)H; yy++) {
        for (int x = 0; x < (int)W; x++) {
            const size_t p = (size_t)yy * W + (size_t)x;
            const uint32_t ps_s = pix_state(key_similar, (uint32_t)p), ps_d = pix_state(key_dissimilar, (uint32_t)p);
            or_win w = {x - rc > 0 ? x - rc : 0, yy - rc > 0 ? yy - rc : 0,
                        x + rc < (int)W - 1 ? x + rc : (int)W - 1, yy + rc < (int)H - 1 ? yy + rc : (int)H - 1};
            uint32_t n = 0;
            nbr[npx + p] = (uint32_t)p;
            n = 1;
            if (f->neighbour_selection_strategy == RESTIR_NEIGHBOURS_RANDOM) {
                for (uint32_t c = 0; c < k; c++) {
                    uint32_t nx = (uint32_t)w.x0 + uniform_index(draw(ps_s, 2u * c), (uint32_t)(w.x1 - w.x0 + 1));
                    uint32_t ny = (uint32_t)w.y0 + uniform_index(draw(ps_s, 2u * c + 1u), (uint32_t)(w.y1 - w.y0 + 1));
                    nbr[(size_t)(1u + n) * npx + p] = ny * W + nx;
                    n++;
                }
            } else {
                uint64_t S = 0, D = 0;
                for (int ny = w.y0; ny <= w.y1; ny++)
                    for (int nx = w.x0; nx <= w.x1; nx++) {
                        size_t q = (size_t)ny * W + (size_t)nx;
                        if (q == p) continue;
                        if (are_similar(s, f, n_t, p_mat, p, q)) S++; else D++;
                    }
                switch (f->neighbour_selection_strategy) {
                case RESTIR_NEIGHBOURS_SIMILAR:
                    if (S < k) {
                        n = emit_class(s, f, n_t, p_mat, W, w, p, 1, S, 0, 1, ps_s, nbr, npx, n);
                        n = emit_class(s, f, n_t, p_mat, W, w, p, 0, D, (uint64_t)k - S, 0, ps_d, nbr, npx, n);
                    } else {
                        n = emit_class(s, f, n_t, p_mat, W, w, p, 1, S, k, 0, ps_s, nbr, npx, n);
                    }
                    break;
                case RESTIR_NEIGHBOURS_DISSIMILAR:
                    if (D < k) {
                        n = emit_class(s, f, n_t, p_mat, W, w, p, 0, D, 0, 1, ps_d, nbr, npx, n);
                        n = emit_class(s, f, n_t, p_mat, W, w, p, 1, S, (uint64_t)k - S, 0, ps_s, nbr, npx, n);
                    } else {
                        n = emit_class(s, f, n_t, p_mat, W, w, p, 0, D, k, 0, ps_d, nbr, npx, n);
                    }
                    break;
                default: {   /* EqualSimilarDissimilar (uint32_t arithmetic as written) */
                    uint32_t sS = (k / 2u) + 1u < (uint32_t)S ? (k / 2u) + 1u : (uint32_t)S;
                    uint32_t desired = k - sS;
                    if ((uint64_t)desired > D) sS = (uint32_t)((uint64_t)sS + ((uint64_t)k - D - sS));
                    n = emit_class(s, f, n_t, p_mat, W, w, p, 1, S, sS, 0, ps_s, nbr, npx, n);
                    n = emit_class(s, f, n_t, p_mat, W, w, p, 0, D, (uint32_t)(k - sS), 0, ps_d, nbr, npx, n);
                } break;
                }
            }
            (void)cap;
            nbr[p] = n;
        }
    }
}

/* One pixel's reservoir (N sub-reservoirs) with the debug planes (wSum, chosenSampleWeight). */
static inline void res_load_dbg(or_sub* r, uint32_t N, const float* a, const float* b, const float* dbg, size_t p,
                                size_t npx) {
    res_load(r, N, a, b, p, npx);
    for (uint32_t j = 0; j < N; j++) { r[j].wsum = dbg[2 * (j * npx + p)]; r[j].chosen = dbg[2 * (j * npx + p) + 1]; }
}

/* One R-MIS iteration's pixel loop (render.cpp:76-112): acc[3][W*H] += the pixel's MIS estimate over its
 * neighbourhood's reservoirs (this iteration's genInitialSamples). */
void or_rmis_accumulate(const or_scene* s, const restir_features* f, const float origin_[3], uint32_t W, uint32_t H,
                        const float* n_t, const float* p_mat, const uint32_t* nbr, const float* res_a,
                        const float* res_b, float* acc) {
    const size_t npx = (size_t)W * H;
    const uint32_t N = f->num_samples_in_reservoir;
    const v3 origin = ld3(origin_);
#pragma omp parallel for schedule(guided)
    for (int yy = 0; yy < (int)H; yy++) {
        or_sub r[RESTIR_MAX_N];
        for (uint32_t x = 0; x < W; x++) {
            const size_t p = (size_t)yy * W + x;
            or_px cur = load_px(s, n_t, p_mat, p, origin);
            const uint32_t c = nbr[p];
            v3 finalColor = mk(0.0f, 0.0f, 0.0f);
            for (uint32_t i = 0; i < c; i++) {
                const size_t q = nbr[(size_t)(1u + i) * npx + p];
                res_load(r, N, res_a, res_b, q, npx);
                for (uint32_t j = 0; j < N; j++) {
                    float misWeight;
                    if (f->mis_weight_rmis == RESTIR_MIS_EQUAL) {
                        misWeight = 1.0f / (float)c;
                    } else {   /* generalisedBalanceHeuristic (render_utils.cpp:179-187) */
                        float numerator = target_pdf(f, &cur, r[j].pos, r[j].col);
                        float denominator = FLT_MIN;
                        for (uint32_t i2 = 0; i2 < c; i2++) {
                            or_px px2 = load_px(s, n_t, p_mat, nbr[(size_t)(1u + i2) * npx + p], origin);
                            denominator += target_pdf(f, &px2, r[j].pos, r[j].col);
                        }
                        misWeight = numerator / denominator;
                    }
                    v3 sc = visible(s, cur.P, r[j].pos) ? shade(f, &cur, r[j].pos, r[j].col) : mk(0.0f, 0.0f, 0.0f);
                    v3 t = vscale(vscale(sc, misWeight), r[j].W);   /* misWeight * sampleColor * outputWeight */
                    finalColor = vadd(finalColor, vdivs(t, (float)N));
                }
            }
            acc[p] += finalColor.x; acc[npx + p] += finalColor.y; acc[2 * npx + p] += finalColor.z;
        }
    }
}

/* ---- Eigen 3 CompleteOrthogonalDecomposition<MatrixXf>::solve (render_utils.h:52), scalar restatement ---- *
 * ColPivHouseholderQR::computeInPlace (ColPivHouseholderQR.h:482-571), CompleteOrthogonalDecomposition::
 * computeInPlace / _solve_impl / applyZAdjointOnTheLeftInPlace (CompleteOrthogonalDecomposition.h:430-560),
 * makeHouseholder / applyHouseholderOnTheLeft / OnTheRight (Householder.h, HouseholderSequence.h:361-412), the
 * upper-triangular back substitution (TriangularSolverVector.h, one panel for n <= 16), with the reductions
 * (norms, the Householder dot products) in Eigen's SIMD packet order below: bit-exact with the reference's
 * vendored Eigen on every system of tests/golden/cod_fixtures.json (oracle/_ref/cod_ref); the device is
 * bit-exact with this. */
#define OR_COD_MAX 8
/* Eigen's reductions of n products a[i] * b[i] with SSE2 Packet4f arithmetic (the image's x86-64 default; no FMA:
 * pmadd = padd(pmul)).  Contiguous operands only; predux(p) = (p0 + p2) + (p1 + p3) (PacketMath.h:987-998).
 * redux: DenseBase::redux, LinearVectorizedTraversal with alignedStart 0 (a cwise expression has no direct access,
 *   Redux.h:205-250): first packet loaded, a second one for 8+ elements, then the scalar tail; n < 4: in order.
 * gemv: one row of general_matrix_vector_product<RowMajor> (GeneralMatrixVector.h:327-515): a zeroed packet
 *   accumulates the 4-blocks, predux, then the tail onto it (so an all-tail row starts from +0). */
static float or_dot_redux(const float* a, int sa, const float* b, int sb, int n) {
    if (n < 4) {
        float r = a[0] * b[0];
        for (int i = 1; i < n; i++) r = r + a[i * sa] * b[i * sb];
        return r;
    }
    float p[4], q[4];
    const int full = n / 4 * 4, end2 = n / 8 * 8;
    for (int l = 0; l < 4; l++) p[l] = a[l * sa] * b[l * sb];
    if (full > 4) {
        for (int l = 0; l < 4; l++) q[l] = a[(4 + l) * sa] * b[(4 + l) * sb];
        for (int i = 8; i < end2; i += 8)
            for (int l = 0; l < 4; l++) {
                p[l] = p[l] + a[(i + l) * sa] * b[(i + l) * sb];
                q[l] = q[l] + a[(i + 4 + l) * sa] * b[(i + 4 + l) * sb];
            }
        for (int l = 0; l < 4; l++) p[l] = p[l] + q[l];
        if (full > end2)
            for (int l = 0; l < 4; l++) p[l] = p[l] + a[(end2 + l) * sa] * b[(end2 + l) * sb];
    }
    float r = (p[0] + p[2]) + (p[1] + p[3]);
    for (int i = full; i < n; i++) r = r + a[i * sa] * b[i * sb];
    return r;
}
static float or_dot_gemv(const float* a, const float* b, int n) {
    float c[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    int j = 0;
    for (; j + 4 <= n; j += 4)
        for (int l = 0; l < 4; l++) c[l] = c[l] + a[j + l] * b[j + l];
    float r = (c[0] + c[2]) + (c[1] + c[3]);
    for (; j < n; j++) r = r + a[j] * b[j];
    return r;
}
/* squaredNorm: vectorised over a contiguous segment, in index order over a strided one (a row of the
 * column-major matrix has no packet access: DefaultTraversal) */
static float or_sqnorm(const float* v, int n, int stride) {
    if (stride == 1) return or_dot_redux(v, 1, v, 1, n);
    float s = v[0] * v[0];
    for (int i = 1; i < n; i++) s = s + v[i * stride] * v[i * stride];
    return s;
}
/* makeHouseholder on v[0], v[stride], ... (m entries): essential written over v[stride..], returns tau, beta */
static void or_make_householder(float* v, int m, int stride, float* tau, float* beta) {
    float tailSqNorm = m == 1 ? 0.0f : or_sqnorm(v + stride, m - 1, stride);
    float c0 = v[0];
    if (tailSqNorm <= FLT_MIN) {
        *tau = 0.0f;
        *beta = c0;
        for (int i = 1; i < m; i++) v[i * stride] = 0.0f;
    } else {
        float b = sqrtf(c0 * c0 + tailSqNorm);
        if (c0 >= 0.0f) b = -b;
        for (int i = 1; i < m; i++) v[i * stride] = v[i * stride] / (c0 - b);
        *tau = (b - c0) / b;
        *beta = b;
    }
}
/* H = I - tau [1 e][1 e]^T from the left on the rows r0..r0+m-1 of columns c0..c0+nc-1 of column-major M (ld).
 * tmp = essential^* bottom is, by Eigen's compile-time product selection: a row-major GEMV when bottom is a
 * matrix block (the QR sweep, OR_HH_GEMV), an inner product (redux) when it is a vector block (Q^* applied to
 * the right-hand side, OR_HH_DOT), in index order when the essential part is a strided row (Z^*, OR_HH_SEQ). */
enum { OR_HH_GEMV = 0, OR_HH_DOT = 1, OR_HH_SEQ = 2 };
static void or_householder_left(float* M, int ld, int r0, int c0, int m, int nc, const float* e, int estride, float tau,
                                int kind) {
    if (m == 1) {
        for (int j = 0; j < nc; j++) M[r0 + (c0 + j) * ld] *= 1.0f - tau;
        return;
    }
    if (tau == 0.0f) return;
    for (int j = 0; j < nc; j++) {
        float* col = &M[(c0 + j) * ld + r0];
        float t;
        if (kind == OR_HH_GEMV) {
            t = or_dot_gemv(e, col + 1, m - 1);
        } else if (kind == OR_HH_DOT) {
            t = or_dot_redux(e, 1, col + 1, 1, m - 1);
        } else {
            t = e[0] * col[1];
            for (int i = 1; i < m - 1; i++) t = t + e[i * estride] * col[1 + i];
        }
        t += col[0];
        col[0] -= tau * t;
        for (int i = 0; i < m - 1; i++) col[1 + i] -= (tau * e[i * estride]) * t;
    }
}
/* H from the right on rows r0..r0+nr-1 of columns c0..c0+m-1: tmp = right * essential is a column-major GEMV,
 * each row summed in index order onto a zeroed accumulator */
static void or_householder_right(float* M, int ld, int r0, int c0, int nr, int m, const float* e, int estride, float tau) {
    if (m == 1) {
        for (int i = 0; i < nr; i++) M[r0 + i + c0 * ld] *= 1.0f - tau;
        return;
    }
    if (tau == 0.0f) return;
    for (int i = 0; i < nr; i++) {
        float t = 0.0f;
        for (int j = 0; j < m - 1; j++) t = t + M[r0 + i + (c0 + 1 + j) * ld] * e[j * estride];
        t += M[r0 + i + c0 * ld];
        M[r0 + i + c0 * ld] -= tau * t;
        for (int j = 0; j < m - 1; j++) M[r0 + i + (c0 + 1 + j) * ld] -= (tau * t) * e[j * estride];
    }
}

void or_cod_solve(uint32_t n_, const float* A, const float* b, float* x) {
    const int n = (int)n_;
    float qr[OR_COD_MAX * OR_COD_MAX], hc[OR_COD_MAX], zc[OR_COD_MAX], nU[OR_COD_MAX], nD[OR_COD_MAX];
    int tr[OR_COD_MAX], perm[OR_COD_MAX];
    memcpy(qr, A, (size_t)n * n * sizeof(float));
    for (int k = 0; k < n; k++) { nD[k] = sqrtf(or_sqnorm(&qr[k * n], n, 1)); nU[k] = nD[k]; }
    float mx = nU[0];
    for (int k = 1; k < n; k++) if (nU[k] > mx) mx = nU[k];
    const float eps = FLT_EPSILON;
    const float threshold_helper = (mx * eps) * (mx * eps) / (float)n;
    const float norm_downdate_threshold = sqrtf(eps);
    int nonzero = n;
    float maxpivot = 0.0f;
    for (int k = 0; k < n; k++) {
        int bi = k;
        float bv = nU[k];
        for (int j = k + 1; j < n; j++) if (nU[j] > bv) { bv = nU[j]; bi = j; }
        if (nonzero == n && bv * bv < threshold_helper * (float)(n - k)) nonzero = k;
        tr[k] = bi;
        if (k != bi) {
            for (int i = 0; i < n; i++) { float t = qr[i + k * n]; qr[i + k * n] = qr[i + bi * n]; qr[i + bi * n] = t; }
            float t = nU[k]; nU[k] = nU[bi]; nU[bi] = t;
            t = nD[k]; nD[k] = nD[bi]; nD[bi] = t;
        }
        float beta;
        or_make_householder(&qr[k + k * n], n - k, 1, &hc[k], &beta);
        qr[k + k * n] = beta;
        if (fabsf(beta) > maxpivot) maxpivot = fabsf(beta);
        or_householder_left(qr, n, k, k + 1, n - k, n - k - 1, &qr[k + 1 + k * n], 1, hc[k], OR_HH_GEMV);
        for (int j = k + 1; j < n; j++) {
            if (nU[j] != 0.0f) {
                float temp = fabsf(qr[k + j * n]) / nU[j];
                temp = (1.0f + temp) * (1.0f - temp);
                temp = temp < 0.0f ? 0.0f : temp;
                float ratio = nU[j] / nD[j];
                float temp2 = temp * (ratio * ratio);
                if (temp2 <= norm_downdate_threshold) {
                    nD[j] = sqrtf(or_sqnorm(&qr[k + 1 + j * n], n - k - 1, 1));
                    nU[j] = nD[j];
                } else {
                    nU[j] *= sqrtf(temp);
                }
            }
        }
    }
    for (int k = 0; k < n; k++) perm[k] = k;
    for (int k = 0; k < n; k++) { int t = perm[k]; perm[k] = perm[tr[k]]; perm[tr[k]] = t; }
    /* ColPivHouseholderQR::rank() (ColPivHouseholderQR.h:255-264), threshold() = epsilon * diagonalSize */
    const float pre = fabsf(maxpivot) * (eps * (float)n);
    int rank = 0;
    for (int i = 0; i < nonzero; i++) rank += fabsf(qr[i + i * n]) > pre;
    /* CompleteOrthogonalDecomposition::computeInPlace: zero R12 from the right */
    if (rank < n) {
        for (int k = rank - 1; k >= 0; k--) {
            if (k != rank - 1)
                for (int i = 0; i <= k; i++) { float t = qr[i + k * n]; qr[i + k * n] = qr[i + (rank - 1) * n]; qr[i + (rank - 1) * n] = t; }
            float beta;
            or_make_householder(&qr[k + (rank - 1) * n], n - rank + 1, n, &zc[k], &beta);
            qr[k + (rank - 1) * n] = beta;
            if (k > 0) or_householder_right(qr, n, 0, rank - 1, k, n - rank + 1, &qr[k + rank * n], n, zc[k]);
            if (k != rank - 1)
                for (int i = 0; i <= k; i++) { float t = qr[i + k * n]; qr[i + k * n] = qr[i + (rank - 1) * n]; qr[i + (rank - 1) * n] = t; }
        }
    }
    /* _solve_impl: rank() again, now over the decomposition's T11 diagonal (|beta| >= the old pivot: the same
     * count, re-evaluated as the reference does) */
    {
        int r2 = 0;
        for (int i = 0; i < nonzero; i++) r2 += fabsf(qr[i + i * n]) > pre;
        rank = r2;
    }
    float c[OR_COD_MAX], y[OR_COD_MAX];
    if (rank == 0) { for (int i = 0; i < n; i++) x[i] = 0.0f; return; }
    for (int i = 0; i < n; i++) c[i] = b[i];
    for (int k = 0; k < rank; k++)   /* Q^* c: H_0 first */
        or_householder_left(c, n, k, 0, n - k, 1, &qr[k + 1 + k * n], 1, hc[k], OR_HH_DOT);
    for (int i = 0; i < n; i++) y[i] = i < rank ? c[i] : 0.0f;
    for (int i = rank - 1; i >= 0; i--) {   /* upper-triangular back substitution, column sweep */
        if (y[i] != 0.0f) {
            y[i] /= qr[i + i * n];
            for (int j = 0; j < i; j++) y[j] -= y[i] * qr[j + i * n];
        }
    }
    if (rank < n) {   /* applyZAdjointOnTheLeftInPlace */
        for (int k = 0; k < rank; k++) {
            if (k != rank - 1) { float t = y[k]; y[k] = y[rank - 1]; y[rank - 1] = t; }
            or_householder_left(y, n, rank - 1, 0, n - rank + 1, 1, &qr[k + rank * n], n, zc[k], OR_HH_SEQ);
            if (k != rank - 1) { float t = y[k]; y[k] = y[rank - 1]; y[rank - 1] = t; }
        }
    }
    for (int i = 0; i < n; i++) x[perm[i]] = y[i];
}

/* arbitraryUnbiasedContributionWeightReciprocal (render_utils.cpp:245-257) for sample (pos, col) against
 * distribution pixel q's reservoir sub sampleIdx */
static inline float aucw_reciprocal(const or_scene* s, const restir_features* f, const or_px* qpx, const or_sub* qr,
                                    v3 pos, v3 col) {
    float targetPdfValue = target_pdf(f, qpx, pos, col);
    if (targetPdfValue == 0.0f) return 0.0f;
    float mockSampleWeight = targetPdfValue / (1.0f / (float)s->num_lights);
    float arbitraryWeight = ((1.0f / targetPdfValue) * (1.0f / (float)qr->M)) * ((qr->wsum - qr->chosen) + mockSampleWeight);
    return 1.0f / arbitraryWeight;
}

/* One R-OMIS iteration's pixel loop (render.cpp:139-231): the technique matrix / contribution vectors (and the
 * progressive estimator's alphas and colour) of acc, layout as RESTIR_BUF_MIS_ACC. */
void or_romis_accumulate(const or_scene* s, const restir_features* f, const float origin_[3], uint32_t W, uint32_t H,
                         const float* n_t, const float* p_mat, const uint32_t* nbr, const float* res_a,
                         const float* res_b, const float* res_dbg, uint32_t iteration, float* acc) {
    const size_t npx = (size_t)W * H;
    const uint32_t N = f->num_samples_in_reservoir;
    const uint32_t T = f->num_neighbours_to_sample + 1u;
    const int32_t totalSamples = (int32_t)(T * N);
    const int32_t fractionOfTotalSamples = (int32_t)N / (int32_t)T;
    const v3 origin = ld3(origin_);
    float* Am = acc;
    float* Bv = acc + (size_t)T * T * npx;
    float* Al = Bv + (size_t)3 * T * npx;
    float* Col = Al + (size_t)3 * T * npx;
#pragma omp parallel for schedule(guided)
    for (int yy = 0; yy < (int)H; yy++) {
        or_sub r[RESTIR_MAX_N], rd[RESTIR_MAX_N];
        for (uint32_t x = 0; x < W; x++) {
            const size_t p = (size_t)yy * W + x;
            or_px cur = load_px(s, n_t, p_mat, p, origin);
            float A[OR_COD_MAX * OR_COD_MAX], bb[3][OR_COD_MAX], al[3][OR_COD_MAX];
            for (uint32_t e = 0; e < T * T; e++) A[e] = Am[e * npx + p];
            for (uint32_t c = 0; c < 3; c++)
                for (uint32_t i = 0; i < T; i++) { bb[c][i] = Bv[(c * T + i) * npx + p]; al[c][i] = Al[(c * T + i) * npx + p]; }
            v3 fc = mk(Col[p], Col[npx + p], Col[2 * npx + p]);
            if (f->use_progressive_romis && iteration >= 1u && iteration % f->progressive_update_mod == 0u)
                for (uint32_t c = 0; c < 3; c++) or_cod_solve(T, A, bb[c], al[c]);
            for (uint32_t pi = 0; pi < T; pi++) {
                if (f->use_progressive_romis) fc = vadd(fc, mk(al[0][pi], al[1][pi], al[2][pi]));
                const size_t q = nbr[(size_t)(1u + pi) * npx + p];
                res_load(r, N, res_a, res_b, q, npx);
                for (uint32_t si = 0; si < N; si++) {
                    float v[OR_COD_MAX];
                    for (uint32_t d = 0; d < T; d++) {
                        const size_t qd = nbr[(size_t)(1u + d) * npx + p];
                        or_px dpx = load_px(s, n_t, p_mat, qd, origin);
                        res_load_dbg(rd, N, res_a, res_b, res_dbg, qd, npx);
                        v[d] = aucw_reciprocal(s, f, &dpx, &rd[si], r[si].pos, r[si].col);
                    }
                    v3 sc = visible(s, cur.P, r[si].pos) ? shade(f, &cur, r[si].pos, r[si].col) : mk(0.0f, 0.0f, 0.0f);
                    if (f->use_progressive_romis) {
                        v3 sa = mk(0.0f, 0.0f, 0.0f);
                        float sf = FLT_MIN;
                        for (uint32_t d = 0; d < T; d++) {
                            sa = vadd(sa, vscale(mk(al[0][d], al[1][d], al[2][d]), v[d]));
                            sf += (float)fractionOfTotalSamples * v[d];
                        }
                        v3 term = vsub(vdivs(sc, sf), vdivs(sa, sf));
                        float inv = 1.0f / (float)totalSamples;
                        fc = vadd(fc, mk(inv * term.x, inv * term.y, inv * term.z));
                    }
                    float scaleFactor = FLT_MIN;
                    for (uint32_t d = 0; d < T; d++) scaleFactor += (float)N * v[d];
                    scaleFactor = 1.0f / scaleFactor;
                    for (uint32_t d = 0; d < T; d++) v[d] *= scaleFactor;
                    for (uint32_t j = 0; j < T; j++)
                        for (uint32_t i = 0; i < T; i++) A[i + j * T] += v[i] * v[j];
                    for (uint32_t row = 0; row < T; row++) {
                        float scaleColVecConst = scaleFactor * v[row];
                        bb[0][row] += sc.x * scaleColVecConst;
                        bb[1][row] += sc.y * scaleColVecConst;
                        bb[2][row] += sc.z * scaleColVecConst;
                    }
                }
            }
            for (uint32_t e = 0; e < T * T; e++) Am[e * npx + p] = A[e];
            for (uint32_t c = 0; c < 3; c++)
                for (uint32_t i = 0; i < T; i++) { Bv[(c * T + i) * npx + p] = bb[c][i]; Al[(c * T + i) * npx + p] = al[c][i]; }
            Col[p] = fc.x; Col[npx + p] = fc.y; Col[2 * npx + p] = fc.z;
        }
    }
}

/* Screen output of R-MIS / progressive R-OMIS (combineToScreen, render_utils.cpp:68-85) or the direct R-OMIS
 * estimator (render.cpp:234-263: per-pixel solves, component sums, tone map).  rgb [H][W][3], row 0 = top. */
void or_mis_finish(const restir_features* f, uint32_t W, uint32_t H, const float* acc, float* rgb) {
    const size_t npx = (size_t)W * H;
    const uint32_t T = f->num_neighbours_to_sample + 1u;
    const int romis = f->ray_trace_mode == RESTIR_MODE_ROMIS;
    const int direct = romis && !f->use_progressive_romis;
    const float* col = romis ? acc + (size_t)(T * T + 6u * T) * npx : acc;
#pragma omp parallel for schedule(guided)
    for (int yy = 0; yy < (int)H; yy++) {
        for (uint32_t x = 0; x < W; x++) {
            const size_t p = (size_t)yy * W + x;
            v3 c;
            if (direct) {
                float A[OR_COD_MAX * OR_COD_MAX], bb[OR_COD_MAX], xs[3][OR_COD_MAX];
                for (uint32_t e = 0; e < T * T; e++) A[e] = acc[e * npx + p];
                for (uint32_t ch = 0; ch < 3; ch++) {
                    for (uint32_t i = 0; i < T; i++) bb[i] = acc[(T * T + ch * T + i) * npx + p];
                    or_cod_solve(T, A, bb, xs[ch]);
                }
                c = mk(0.0f, 0.0f, 0.0f);
                for (uint32_t row = 0; row < T; row++) { c.x += xs[0][row]; c.y += xs[1][row]; c.z += xs[2][row]; }
            } else {
                c = vdivs(mk(col[p], col[npx + p], col[2 * npx + p]), (float)f->max_iterations_mis);
            }
            if (f->enable_tone_mapping) c = tonemap(c, f->exposure, f->gamma);
            st3(&rgb[3 * ((size_t)(H - 1u - (uint32_t)yy) * W + x)], c);
        }
    }
}

uint32_t or_mis_acc_rows(const restir_features* f) {
    const uint32_t T = f->num_neighbours_to_sample + 1u;
    return f->ray_trace_mode == RESTIR_MODE_ROMIS ? T * T + 6u * T + 3u : 3u;
}

/* renderRMIS / renderROMIS (render.cpp:64-265) over the whole W x H image; rgb [H][W][3], row 0 = top. */
int or_render_mis(const or_scene* s, const restir_camera* cam, const restir_features* f, uint32_t seed, uint32_t frame,
                  uint32_t W, uint32_t H, float* rgb, int threads) {
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
    const uint32_t N = f->num_samples_in_reservoir;
    if (N == 0 || N > RESTIR_MAX_N) return -2;
    const size_t npx = (size_t)W * H;
    restir_camera_frame cf;
    or_camera_derive(cam, &cf);
    float* n_t = (float*)malloc(npx * 16);
    float* p_mat = (float*)malloc(npx * 16);
    or_rect view = {0, 0, W, H};
    float* uv = s->num_textures ? (float*)calloc(npx * 2, 4) : NULL;
    const float* bound = s->uv;
    or_primary_uv(s, &cf, W, H, view, view, n_t, p_mat, uv);
    if (uv) ((or_scene*)s)->uv = uv;
    const uint32_t cap = or_mis_capacity(f, W, H);
    uint32_t* nbr = (uint32_t*)calloc((size_t)(1u + cap) * npx, 4);
    or_neighbours(s, f, or_rng_key(seed, frame, RESTIR_STAGE_NEIGHBOURS, 0), or_rng_key(seed, frame, RESTIR_STAGE_NEIGHBOURS, 1),
                  W, H, n_t, p_mat, cap, nbr);
    const size_t rows = or_mis_acc_rows(f);
    float* acc = (float*)calloc(rows * npx, 4);
    float* a = (float*)malloc(npx * N * 16);
    float* b = (float*)malloc(npx * N * 16);
    float* d = (float*)malloc(npx * N * 8);
    int rc = 0;
    for (uint32_t it = 0; it < f->max_iterations_mis; it++) {
        or_ris(s, f, or_rng_key(seed, frame, RESTIR_STAGE_RIS, it), cf.origin, W, H, view, view, n_t, p_mat, a, b, d);
        if (f->ray_trace_mode == RESTIR_MODE_ROMIS)
            or_romis_accumulate(s, f, cf.origin, W, H, n_t, p_mat, nbr, a, b, d, it, acc);
        else
            or_rmis_accumulate(s, f, cf.origin, W, H, n_t, p_mat, nbr, a, b, acc);
    }
    or_mis_finish(f, W, H, acc, rgb);
    ((or_scene*)s)->uv = bound;
    free(uv);
    free(n_t); free(p_mat); free(nbr); free(acc); free(a); free(b); free(d);
    return rc;
}

/*
 * restir_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C11) of the reference's ReSTIR hot path, used as the parity checker by tests/,
 * by __graft_entry__.smoke() and as bench.py's cpu_baseline ("port").  The product (libromis_amd.so) never
 * links, loads or calls anything here.  Each function cites the reference file:line it restates.
 *
 * Parity status (see DESIGN.md "Oracle"):
 *  - scene inputs (loadMesh/loadScenePrebuilt/regularLightGrid), tone mapping and every glm primitive used
 *    below are PINNED against the reference's own translation units compiled here (oracle/_ref, fixtures in
 *    tests/golden/ref_fixtures.json);
 *  - the reservoir arithmetic itself (reservoir.cpp, light.cpp, render_utils.cpp, shading.cpp) is a
 *    line-by-line restatement whose parity against the reference binary is UNPINNED: those translation units
 *    include embree4/rtcore.h / <format> / GL/glu.h, which this image lacks, and the reference holds no tests
 *    or golden vectors;
 *  - visibility (Embree rtcOccluded1 / rtcIntersect1, Embree 4.3.1, not vendored) is restated as
 *    Moller-Trumbore with Embree's (tnear, tfar] convention: parity vs Embree UNPINNED;
 *  - powf/expf use the portable double-evaluated implementations below (shared with the device code) in
 *    place of glibc's, so oracle and device agree bit-for-bit; they track glibc within the 1e-5 tolerance.
 */
#ifndef RESTIR_ORACLE_H
#define RESTIR_ORACLE_H

#include <stdint.h>
#include "../include/restir_c.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_scene or_scene;

/* A rectangle of the global image, in global pixel coordinates (y = 0 bottom). */
typedef struct or_rect { uint32_t x0, y0, w, h; } or_rect;

or_scene* or_scene_create(const restir_mesh* meshes, uint32_t num_meshes, const restir_light* lights,
                          uint32_t num_lights);
or_scene* or_scene_create_textured(const restir_mesh* meshes, uint32_t num_meshes, const restir_light* lights,
                                   uint32_t num_lights, const restir_texture* textures, uint32_t num_textures);
/* the G-buffer texCoord plane ([pixels][2], indexed like n_t / p_mat) the following stage calls read; NULL = none */
void      or_scene_bind_uv(or_scene* s, const float* uv);
void      or_acquire_texel(const or_scene* s, uint32_t texture, const float tc[2], float out[3]);
void      or_scene_destroy(or_scene* s);
uint32_t  or_scene_num_triangles(const or_scene* s);
uint32_t  or_scene_miss_material(const or_scene* s);

/* keyed RNG (restir_c.h header comment) */
uint32_t or_rng_key(uint32_t seed, uint32_t frame, uint32_t stage, uint32_t pass);
uint32_t or_rng_draw(uint32_t key, uint32_t global_pixel, uint32_t slot);

/* primitives exposed for the pinning tests */
void  or_glm_probe(const float a[3], const float b[3], float t, const float e[3], float out[24]);
void  or_tonemap(const float c[3], float exposure, float gamma, float out[3]);
float or_powf(float x, float y);
float or_expf(float x);
void or_powf_n(const float* x, const float* y, float* out, size_t n);
void or_expf_n(const float* x, float* out, size_t n);
void  or_camera_derive(const restir_camera* cam, restir_camera_frame* out);
float or_target_pdf(const or_scene* s, const restir_features* f, const float origin[3],
                    const float n_t[4], const float p_mat[4], const float lpos[3], const float lcol[3]);

/* Passes.  All grids cover `view` (row-major, index (y - view.y0) * view.w + (x - view.x0)); reservoir
 * planes are [N][view pixels]; each pass writes only the pixels of `rect` (a sub-rectangle of view). */
void or_primary(const or_scene* s, const restir_camera_frame* cam, uint32_t W, uint32_t H, or_rect view,
                or_rect rect, float* n_t, float* p_mat);
void or_primary_uv(const or_scene* s, const restir_camera_frame* cam, uint32_t W, uint32_t H, or_rect view,
                   or_rect rect, float* n_t, float* p_mat, float* uv);
void or_ris(const or_scene* s, const restir_features* f, uint32_t key, const float origin[3], uint32_t W,
            uint32_t H, or_rect view, or_rect rect, const float* n_t, const float* p_mat, float* res_a,
            float* res_b, float* res_dbg);
void or_temporal(const or_scene* s, const restir_features* f, uint32_t key, const float origin[3], uint32_t W,
                 uint32_t H, or_rect view, or_rect rect, const float* n_t, const float* p_mat,
                 const float* cur_a, const float* cur_b, const float* prev_a, const float* prev_b,
                 float* out_a, float* out_b, float* out_dbg);
/* One spatial pass: neighbours from (in_a, in_b); returns 0, or -1 if a neighbour fell outside `view`. */
int  or_spatial_pass(const or_scene* s, const restir_features* f, uint32_t key, const float origin[3],
                     uint32_t W, uint32_t H, or_rect view, or_rect rect, const float* n_t, const float* p_mat,
                     const float* in_a, const float* in_b, float* out_a, float* out_b, float* out_dbg);
/* Final shading + tone map.  rgb is [rect.h][rect.w][3] with row 0 = TOP of rect (Screen layout). */
void or_final(const or_scene* s, const restir_features* f, const float origin[3], uint32_t W, uint32_t H,
              or_rect view, or_rect rect, const float* n_t, const float* p_mat, const float* res_a,
              const float* res_b, float* rgb);

/* Whole frame over `view` (renderReSTIR, render.cpp:28-62), owned pixels = rect.  prev_a/prev_b may be
 * NULL.  Final reservoirs are written to out_a/out_b (view layout); rgb is rect-sized.  Returns 0 on
 * success.  `threads` > 0 sets the OpenMP thread count (CPU baseline). */
int or_render_frame(const or_scene* s, const restir_camera* cam, const restir_features* f, uint32_t seed,
                    uint32_t frame, uint32_t W, uint32_t H, or_rect view, or_rect rect, const float* prev_a,
                    const float* prev_b, float* n_t, float* p_mat, float* out_a, float* out_b, float* rgb,
                    int threads);

/* R-MIS / R-OMIS (render.cpp:64-265) over a whole W x H image (pixel index p = y * W + x).  Buffer layouts are
 * RESTIR_BUF_MIS_NBR ([1 + cap][W*H] uint32) and RESTIR_BUF_MIS_ACC ([or_mis_acc_rows][W*H] float). */
uint32_t or_mis_capacity(const restir_features* f, uint32_t W, uint32_t H);
uint32_t or_mis_acc_rows(const restir_features* f);
void or_neighbours(const or_scene* s, const restir_features* f, uint32_t key_similar, uint32_t key_dissimilar,
                   uint32_t W, uint32_t H, const float* n_t, const float* p_mat, uint32_t cap, uint32_t* nbr);
void or_rmis_accumulate(const or_scene* s, const restir_features* f, const float origin[3], uint32_t W, uint32_t H,
                        const float* n_t, const float* p_mat, const uint32_t* nbr, const float* res_a,
                        const float* res_b, float* acc);
void or_romis_accumulate(const or_scene* s, const restir_features* f, const float origin[3], uint32_t W, uint32_t H,
                         const float* n_t, const float* p_mat, const uint32_t* nbr, const float* res_a,
                         const float* res_b, const float* res_dbg, uint32_t iteration, float* acc);
void or_mis_finish(const restir_features* f, uint32_t W, uint32_t H, const float* acc, float* rgb);
/* Eigen CompleteOrthogonalDecomposition<MatrixXf>(A).solve(b), n <= 8, A column-major (scalar restatement). */
void or_cod_solve(uint32_t n, const float* A, const float* b, float* x);
int  or_render_mis(const or_scene* s, const restir_camera* cam, const restir_features* f, uint32_t seed,
                   uint32_t frame, uint32_t W, uint32_t H, float* rgb, int threads);

#ifdef __cplusplus
}
#endif
#endif

// restir_types.h -- device-side data layout shared by the kernels (kernels.hip) and the host launcher
// (restir.cpp).  See DESIGN.md "Data layout in HBM".
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define RESTIR_MAX_N_DEV 32u

// material pow modes (std::pow(cosTheta, shininess), shading.cpp:26)
#define ROMIS_POW_SKIP 0u      // ks == 0: the specular term is +-0 whatever pow returns
#define ROMIS_POW_GLIBC 1u     // glibc's powf specialised to the material's exponent (kernels.hip material_pow)
#define ROMIS_POW_SIMPLE 2u    // ROMIS_POW_GLIBC for a finite exponent y > 0 whose underflow threshold is >= 2^-126:
                               // a zero or subnormal base is always under the threshold, so the cases before the
                               // log2 / exp2 core reduce to three selects (pow_pre)
// exponent classes of ROMIS_POW_GLIBC (materials[3m + 2].y)
#define ROMIS_PWC_ODD 1u       // glibc checkint(y) == 1: odd integer
#define ROMIS_PWC_INT 2u       // checkint(y) != 0: integer
#define ROMIS_PWC_NEG 4u       // y < 0
#define ROMIS_PWC_ZERO 8u      // y == +-0
#define ROMIS_PWC_NAN 16u      // y is NaN
#define ROMIS_PWC_PINF 32u     // y == +inf
#define ROMIS_PWC_NINF 64u     // y == -inf
#define ROMIS_PWC_SPECIAL (ROMIS_PWC_ZERO | ROMIS_PWC_NAN | ROMIS_PWC_PINF | ROMIS_PWC_NINF)

namespace romis {

// Scene as the kernels see it.  All arrays are device pointers, 16-byte aligned float4 records.
struct SceneDev {
    // Threaded (stackless) BVH, depth-first order, 2 float4 per node:
    //   nodes[2i]   = (lo.xyz, bits(miss link))       miss link = next node when the box is missed / leaf done
    //   nodes[2i+1] = (hi.xyz, bits(leaf))            leaf = 0 for inner nodes (child = i + 1), else
    //                                                  (count << 24) | first triangle (BVH order)
    const float4* nodes;
    uint32_t num_nodes;
    // The same nodes for shadow rays, 16 bytes each (kernels_common.h occluded_q): the padded box snapped outward to a
    // 16-bit grid over the root box -- x = lo.x | lo.y << 16, y = lo.z | hi.x << 16, z = hi.y | hi.z << 16, coordinate
    // = q_lo + q * q_s -- and w = miss link | first triangle << 16 | count << 28 (count 0: inner node).  nodes_q_ok = 0
    // when the tree does not fit (>= 65,536 nodes, a leaf past triangle 4,096 or of > 15 triangles).
    const uint4* nodes_q;
    uint32_t nodes_q_ok;
    float4 q_lo, q_s;
    // Triangles in BVH order (Moller-Trumbore operands, e1 = v1 - v0, e2 = v2 - v0 computed on the host):
    //   tri_v0.w = bits(original triangle index) -- closest-hit ties resolve to the lowest original index
    const float4* tri_v0;
    const float4* tri_e1;
    const float4* tri_e2;
    // Shading attributes by ORIGINAL triangle index: vertex normals, n0.w = bits(material index)
    const float4* tri_n0;
    const float4* tri_n1;
    const float4* tri_n2;
    uint32_t num_tris;
    // Materials: 3 float4 each: (kd.xyz, shininess), (ks.xyz, bits(pow mode)),
    // (pow underflow threshold, bits(shininess class ROMIS_PWC_*), transparency, 0).  Last entry = miss material.
    const float4* materials;
    uint32_t num_materials;
    // Lights: 7 float4 each: (p0.xyz, bits(type)), (p1.xyz, 0), (p2.xyz, 0), c0, c1, c2, c3
    const float4* lights;
    uint32_t num_lights;
    uint32_t light_types;      // bit t set <=> a light of type t is present
    float light_scale;         // L when 1/L is a power of two (then p / (1/L) == p * L exactly), else 0
    const float4* light_c2;    // compact table, two planes: row 0 of every light's record (p0 / position), then row 3
                               // (first colour) -- light i's rows at [i] and [num_lights + i]
    uint32_t lights_grid;      // every light a parallelogram with light 0's edges (rows 1, 2) and c0 = c1 = c2 = c3
    const float4* light_c4;    // rows 0..3 of every light's record (v0, edge01, edge02, c0): the kLtPgram table
    uint32_t lights_pgram;     // every light a parallelogram with c0 = c1 = c2 = c3
    // a light grid (lights_grid) laid out as regularLightGrid does (scene.cpp:5-28): light i's corner is
    // (start + s01 * float(i / ny)) + s02 * float(i % ny) bit for bit (host-verified), ny a power of two -- the RIS
    // kernels' kLtRegular form computes the corner and reads only the colour (light_col: c0 of every light)
    uint32_t lights_regular;
    uint32_t grid_ny_log2;
    float4 grid_start, grid_s01, grid_s02;   // .xyz
    const float4* light_col;
    uint32_t lights_finite;    // every light coordinate / colour is finite
    uint32_t shade_finite;     // every light colour x material kd / ks product is finite (shade()'s NaN tests)
    uint32_t normals_bounded;  // every vertex normal component finite with |n| <= 2^125: interpolated normals are
                               // finite, so a miss pixel's zero normal rejects every neighbour (dot = +-0)
    uint32_t miss_shade_zero;  // the miss material's kd and ks are 0 and every light colour is finite with |c| <= 2^126
                               // (so every light sample's colour, a convex mix, is finite): a miss pixel shades any
                               // light sample to +-0 (k_final's miss shortcut)
    // Textures (Material::kdTexture): texels as float4 (rgb, 0), all images back to back; tex_dims[i] =
    // (width, height, first texel, 0); per-triangle texture coordinates by original index, 2 float4 each:
    // (t0.xy, t1.xy), (t2.xy, 0, 0).  materials[3m + 2].w = bits(kd_texture), 0 = none.
    const float4* tex_texels;
    const uint4* tex_dims;
    const float4* tri_uv;
    uint32_t num_textures;
    // per launch (set by the host for the view being rendered): the G-buffer texCoord plane (nullptr for scenes
    // without textures; k_primary writes it, everything else reads it) and whether diffuseAlbedo reads
    // textures (Features::enableTextureMapping and num_textures > 0)
    float2* gbuf_uv;
    uint32_t tex_on;
};

// Image region bookkeeping: global image W x H (y = 0 bottom), storage view (the computed region, row-major)
// and the rectangle a pass writes.
struct Region {
    uint32_t W, H;
    uint32_t vx0, vy0, vw, vh;
    uint32_t rx0, ry0, rw, rh;
    uint32_t map2d;   // work item = a 32x8 tile (1: waves 32x2, 2: waves 8x8) or 256 row-major pixels (0)
    // Record layout of the G-buffer n_t and reservoir (res_a, res_b) arrays: element (j, p) of view pixel p
    // lives at index j * js + p * ps.  SoA planes: ps = 1, js = view pixels.  Per-pixel records
    // [n_t, a_0, b_0, a_1, b_1, ...] (restir_render): ps = 1 + 2N, js = 2, with res_a = rec + 1, res_b = rec + 2.
    uint32_t ps, js;
    uint32_t xcd_rows;   // the lean spatial passes' XCD tile order (xcd_tile); 0 elsewhere
    uint32_t xcd_cols;   // chunk width in tiles (xcd_tile); 0 = the whole row of tiles
};

// Background tiles (restir_render, N <= 2, no temporal reuse): the fused primary + RIS kernel writes one byte per
// 32 x 8 tile of its region (the view), 0 when every pixel of the tile is a primary-ray miss whose RIS reservoir is
// known -- the miss material, P not NaN, finite lights, L != 0: (0, 0, 0, W = 0), (0, 0, 0, M = f.M) in sub-reservoir
// 0 and M = 0 in sub-reservoir 1, pdf 0 -- and
// 1 otherwise.  The spatial passes and final shading then write such tiles' known results without reading them.
// m: the M every such pixel holds at the pass's input (0: flags unused by this launch).
struct MissTiles {
    const uint8_t* flags;
    uint32_t m;
    uint32_t gbuf;   // 1: RIS did not store background tiles' G-buffer records either (a biased pass fixes its window up)
};

// Sample handles (N = 1, point-light scenes, kernels.hip k_spatial1h): per view pixel the held sample's W (w) and
// M | light index << 24 (m; index L = the initial zero sample), written beside the reservoir planes by the producer.
// The predecessor grid of a temporal pass fused into primary rays + RIS (launch_primary_ris_temporal)
struct TemporalIn {
    const float4* pa;
    const float4* pb;
    uint32_t key;   // the temporal stage's RNG key
    // N = 1 point lights: the predecessor's sample handles (W, M | light index << 24), read instead of (pa, pb) -- the
    // light table rebuilds the sample (restir_render's frame handles; nullptr: the reservoir planes)
    const float* hw;
    const uint32_t* hm;
};

struct Handles {
    float* w;
    uint32_t* m;
    uint32_t res_dead;   // (an output) the handles are the reservoir planes' only reader: RIS / the pass skips their stores
};

// Launch-shape knobs (restir_set_tuning); they never change results, only speed.
constexpr uint32_t kXcdRowsAuto = 255u;
constexpr uint32_t kXcdColsAuto = 255u;
struct Tuning {
    uint32_t primary_lds = 1;      // stage the BVH in LDS when it fits
    uint32_t ris_lds = 1;          // stage the light table in LDS when it fits
    uint32_t ris_compact = 1;      // N <= 2: compact light tables for point-light-only scenes and light grids (_pt /
                                   // _grid RIS kernels, kernels.hip ris_light_form)
    uint32_t miss_tiles = 1;       // restir_render: background-tile flags (MissTiles) from RIS to the spatial passes
                                   // and final shading
    uint32_t miss_gbuf = 2;        // RIS skips background tiles' G-buffer stores: 0 never, 1 whenever the passes and final
                                   // shading allow, 2 (auto) the same but biased passes only from 2048 px wide (their
                                   // window fix-up's per-entry flag loads outweigh the saved stores at 1080p)
    uint32_t ris_late = 1;         // fused primary + RIS, one tile per block: stage the light table only for tiles with
                                   // a pixel that runs the candidate loop (0: every tile, before the primary rays)
    uint32_t spatial_xcd_rows = 255; // lean passes: XCD x takes every 8th chunk of this many tile rows (0: one band;
                                     // 255 = kXcdRowsAuto: as many as keep a chunk's records in one XCD's L2)
    uint32_t spatial_xcd_cols = 255; // chunk width in tiles (0: full rows); 2-D chunks keep the +-R window rows of
                                     // consecutive tile rows in the XCD's L2.  255 = kXcdColsAuto: the N = 1 biased
                                     // pass on 32 x 8 tiles takes 8 tile rows x a third of the tile row when the row
                                     // has >= 24 tiles (C2: 1.20 -> 1.0x traffic, same time), full rows elsewhere
    uint32_t fuse_primary_ris = 1; // restir_render: k_primary_ris instead of k_primary + k_ris when the BVH fits LDS
    uint32_t spatial_lean = 1;     // the lean N = 1 / 2 passes (0: the general kernels)
    uint32_t spatial_th = 0;       // N = 1 biased ntl pass: tile height in 8-row units (1: 32x8, 2: 32x16 k_spatial1_ntl_t2; 0: by width)
    uint32_t fuse_temporal = 1;    // restir_render with a predecessor: temporal reuse inside the fused RIS kernel
    uint32_t spatial_handles = 1;  // restir_render, N = 1 biased, point lights: the passes read sample handles (k_spatial1h)
    uint32_t spatial_n2h = 1;      // N = 2 biased passes over point lights read 16-byte handle records (k_spatial2hg)
    uint32_t spatial_gather = 1;   // the point-light handle pass on 32 x 16 tiles gathers the accepted neighbours' handles
                                   // (k_spatial1hg_t2: 34 KB of LDS, four blocks per CU) instead of staging the handle
                                   // windows in LDS (k_spatial1h_t2: 49.5 KB, three blocks); C2 65.7 -> 64.9 us (round 6)
    uint32_t timing_mask = 0xFFFFFFFFu;   // kernels (bit = RESTIR_K_*) bracketed by HIP events when timing is on
    uint32_t timing_every = 1;     // events on every n-th launch of a timed kernel (the others launch plain)
    uint32_t timing_fence = 0;     // 1: timing events with the default system-scope release (a cache writeback after
                                   // the timed kernel: 6.7 + 4.6 us of stream gaps per C2 frame, profiles/r4); 0:
                                   // hipEventDisableSystemFence (read only after a stream synchronisation)
    uint32_t records = 0;          // frame path: per-pixel records (1) or SoA planes (0); planes measured faster
    uint32_t bvh_max_leaf = 2;     // triangles per BVH leaf (used by restir_set_scene); 2 beat 1/4/8 (kbench)
    uint32_t final_lds = 1;
    uint32_t final_miss = 1;       // k_final_n*_sorted: primary-ray misses read p_mat + (pos, W) only (SceneDev::miss_shade_zero)
    uint32_t final_qbvh = 2;       // k_final_n*_sorted: shadow rays over the 16-byte nodes (SceneDev::nodes_q) when they fit;
                                   // 2 (auto): at N = 2 (C2 N = 2 final 153.6 -> 145.8 us; N = 1: C2 80.0 -> 79.5, C4f
                                   // 265.8 -> 277.4 -- round 6, profiles/r6/probes/s7)
    uint32_t final_sort = 1;       // N = 1: bin each tile's shadow rays by target before tracing (-2.4 %, r2ah)
    uint32_t primary_tl = 1;       // fused primary + RIS, one tile per block: the primary rays test the tile's candidate
                                   // triangles (tile_triangles) instead of walking the BVH
    uint32_t mis_chunk = 0;        // R-OMIS samples per k_romis_samples / k_romis_accum pair; 0 = the scratch budget
};

// Halo segments of one exchange (restir_halo_plan), pixel prefix offsets into the packed buffer.
#define RESTIR_MAX_HALO_SEGS 8u
struct HaloSegs {
    uint32_t n;
    uint32_t x0[RESTIR_MAX_HALO_SEGS], y0[RESTIR_MAX_HALO_SEGS], w[RESTIR_MAX_HALO_SEGS], h[RESTIR_MAX_HALO_SEGS];
    uint32_t px0[RESTIR_MAX_HALO_SEGS + 1];   // px0[i] = pixels before segment i; px0[n] = total
};

struct CameraDev {
    float4 quat;      // x, y, z, w
    float origin[3];
    float half_w, half_h;
};

// The Features subset the kernels read.
struct FeaturesDev {
    uint32_t M, N, K, R;
    uint32_t clamp_m;
    uint32_t initial_vis, unbiased, spatial_vis, shading, tone_map;
    float gamma, exposure;
    uint32_t texture;         // enableTextureMapping
    // R-MIS / R-OMIS and the neighbour-selection heuristic (common.h:110-121)
    uint32_t mode;            // restir_mode
    uint32_t strategy;        // restir_neighbour_strategy
    uint32_t same_geom;
    float depth_frac, normal_rad;
    uint32_t mis_weight;      // restir_mis_weight
    uint32_t progressive, prog_mod, iterations;
};

}  // namespace romis

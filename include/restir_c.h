/*
 * restir_c.h -- C ABI of the MI355X-native ReSTIR direct-lighting sampler (libromis_amd.so).
 *
 * Drop-in boundary for the reference's ReSTIR render entry:
 *   renderRayTraced(prevGrid, Scene, Trackball, EmbreeInterface, Screen, Features)   src/rendering/render.cpp:268-290
 *   renderReSTIR   (prevGrid, Scene, Trackball, EmbreeInterface, Screen, Features)   src/rendering/render.cpp:28-62
 * Plain pointers and sizes only: no C++ / torch types cross this line.  The C++ wrapper that keeps the
 * reference's call surface (value-typed grids, exceptions) is include/romis_amd/restir.hpp.
 *
 * Conventions (mirroring the reference):
 *  - every entry point returns restir_status; the message of the last failure on the calling thread is
 *    restir_last_error() (the C++ wrapper rethrows it as std::runtime_error, as render.cpp:99/278 do);
 *  - a context owns one HIP device, one HIP stream and all device buffers; calls on one context are
 *    serialised by the context, different contexts are independent (main.cpp:213-230 renders per thread);
 *  - a restir_frame is the device-resident replacement of std::shared_ptr<ReservoirGrid> (main.cpp:165):
 *    reference-counted, never copied to the host unless downloaded.
 *  - pixel (x, y) uses the reference's convention: y = 0 is the BOTTOM row (render_utils.cpp:24-25); the RGB
 *    image handed back is laid out like Screen's texture (screen.cpp:37-43): row 0 = TOP.
 *
 * Keyed RNG (the parity contract; the reference's rand()/random_device/mt19937 are not seedable):
 *   mix32(h)          = murmur3 fmix32
 *   key(s,f,stage,p)  = mix32(mix32(mix32(s ^ 0x9E3779B9) + f) ^ (stage * 0x01000193 + p * 0x27D4EB2F))
 *   pix(key, g)       = mix32(key ^ mix32(g * 0x9E3779B1 + 0x7F4A7C15))        g = global pixel id y*W + x
 *   draw(pix, slot)   = mix32(pix + slot * 0x9E3779B9)
 *   rand()            -> draw >> 1 ; u = linearMap(float(rand()), 0, RAND_MAX, 0, 1)   (utils.cpp:26-31)
 *   U{0..L-1}         -> (uint64(draw) * L) >> 32
 *   U{-r..r}          -> ((uint64(draw) * (2r+1)) >> 32) - r
 * stages / slots:
 *   RESTIR_STAGE_RIS      (pass 0): candidate c: light 4c, first rand 4c+1, second rand 4c+2, accept 4c+3
 *   RESTIR_STAGE_TEMPORAL (pass 0): accept of the t-th Reservoir::update = t
 *   RESTIR_STAGE_SPATIAL  (pass p): neighbour n: dx 2n, dy 2n+1; accept of the t-th update = 2k + t
 *   R-MIS / R-OMIS (restir_render with RESTIR_MODE_RMIS / ROMIS):
 *   RESTIR_STAGE_RIS      (pass i): the i-th MIS iteration's genInitialSamples, slots as above
 *   RESTIR_STAGE_NEIGHBOURS         generateResampleIndicesGrid (neighbour_selection.cpp:45-122), once per render:
 *     Random strategy (pass 0): candidate n: x 2n, y 2n+1, U{lo..hi} -> lo + ((uint64(draw) * (hi-lo+1)) >> 32)
 *     std::sample over the similar list (pass 0) / the dissimilar list (pass 1): selection sampling, the list's
 *     i-th element is kept iff U{0..len-1-i} (slot i) < the number still needed
 */
#ifndef RESTIR_C_H
#define RESTIR_C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RESTIR_ABI_VERSION 5   /* 2: restir_features gained the R-MIS / R-OMIS fields;
                                  3: textures (restir_texture, restir_material.kd_texture, restir_mesh.texcoords);
                                  4: halo passes split into interior / border, native RCCL halo transport,
                                     frame output (8-bit BMP, Features JSON record);
                                  5: the native transport's operation list (restir_halo_ops) and its record-only
                                     mode (restir_halo_record / restir_halo_log) */

#define RESTIR_STAGE_RIS      1u
#define RESTIR_STAGE_TEMPORAL 2u
#define RESTIR_STAGE_SPATIAL  3u
#define RESTIR_STAGE_NEIGHBOURS 4u
#define RESTIR_DEFAULT_SEED   0x5EED0001u
#define RESTIR_MAX_N          32u   /* numSamplesInReservoir slider range 1..32 (ui.cpp:305) */

typedef enum restir_status {
    RESTIR_OK              = 0,
    RESTIR_ERR_INVALID     = 1,  /* bad argument (null pointer, size, range) */
    RESTIR_ERR_HIP         = 2,  /* HIP runtime failure */
    RESTIR_ERR_NO_DEVICE   = 3,  /* no usable gfx950 device */
    RESTIR_ERR_STATE       = 4,  /* call out of order (e.g. render before set_scene) */
    RESTIR_ERR_UNSUPPORTED = 5,  /* feature combination not implemented (e.g. R-MIS / R-OMIS on a screen tile) */
    RESTIR_ERR_COMM        = 6   /* RCCL failure */
} restir_status;

/* RayTraceMode (src/utils/common.h:25-29): renderReSTIR, renderRMIS, renderROMIS (render.cpp:28-265). */
typedef enum restir_mode { RESTIR_MODE_RESTIR = 0, RESTIR_MODE_RMIS = 1, RESTIR_MODE_ROMIS = 2 } restir_mode;
/* MISWeightRMIS (common.h:31-34) and NeighbourSelectionStrategy (common.h:36-41) */
typedef enum restir_mis_weight { RESTIR_MIS_EQUAL = 0, RESTIR_MIS_BALANCE = 1 } restir_mis_weight;
typedef enum restir_neighbour_strategy {
    RESTIR_NEIGHBOURS_RANDOM = 0, RESTIR_NEIGHBOURS_SIMILAR = 1, RESTIR_NEIGHBOURS_DISSIMILAR = 2,
    RESTIR_NEIGHBOURS_EQUAL_SIMILAR_DISSIMILAR = 3
} restir_neighbour_strategy;

/* std::variant<PointLight, SegmentLight, ParallelogramLight> (common.h:72-87) flattened. 88 bytes. */
typedef enum restir_light_type {
    RESTIR_LIGHT_POINT = 0, RESTIR_LIGHT_SEGMENT = 1, RESTIR_LIGHT_PARALLELOGRAM = 2
} restir_light_type;
typedef struct restir_light {
    uint32_t type;
    float p0[3];   /* Point.position | Segment.endpoint0 | Parallelogram.v0     */
    float p1[3];   /*                | Segment.endpoint1 | Parallelogram.edge01 */
    float p2[3];   /*                                    | Parallelogram.edge02 */
    float c0[3];   /* Point.color    | Segment.color0    | Parallelogram.color0 */
    float c1[3];   /*                | Segment.color1    | Parallelogram.color1 */
    float c2[3];   /*                                    | Parallelogram.color2 */
    float c3[3];   /*                                    | Parallelogram.color3 */
} restir_light;

/* Image (framework/include/framework/image.h): width x height texels, row-major [y][x] with y = 0 the image
 * file's first row (Image::pixels order), each texel the stb RGB bytes / 255.0f (image.cpp:22-31). */
typedef struct restir_texture {
    uint32_t     width, height;
    const float* rgb;              /* [height][width][3] */
} restir_texture;

/* Material (framework/include/framework/mesh.h:22-34).  kd_texture = Material::kdTexture: 0 = none, else
 * 1 + an index into restir_set_scene_textured's textures (several materials may share one Image). */
typedef struct restir_material {
    float    kd[3];
    float    ks[3];
    float    shininess;
    float    transparency;
    uint32_t kd_texture;
} restir_material;

/* Mesh (mesh.h:36-43): one material per mesh, like loadMesh's per-material sub-meshes. */
typedef struct restir_mesh {
    const float*    positions;     /* [num_vertices][3] */
    const float*    normals;       /* [num_vertices][3] */
    uint32_t        num_vertices;
    const uint32_t* triangles;     /* [num_triangles][3] vertex indices */
    uint32_t        num_triangles;
    restir_material material;
    const float*    texcoords;     /* [num_vertices][2] Vertex::texCoord; NULL = (0, 0) (loadMesh's default) */
} restir_mesh;

/* Trackball state (framework/include/framework/trackball.h:13-66) as set by Trackball(window, fovy, dist)
 * + setCamera(lookAt, rotation, dist) (main.cpp:223-224). Angles in radians. */
typedef struct restir_camera {
    float fovy;
    float aspect;          /* Window::getAspectRatio() = float(w)/float(h) (window.cpp:380-385) */
    float look_at[3];
    float distance;
    float rotation[3];     /* Euler angles (x, y, z) */
} restir_camera;

/* Derived per-frame camera constants (Trackball::position / generateRay, trackball.cpp:75-78,105-114). */
typedef struct restir_camera_frame {
    float origin[3];
    float quat[4];         /* x, y, z, w of glm::quat(rotation) */
    float half_w, half_h;  /* m_halfScreenSpaceWidth / Height */
} restir_camera_frame;

/* The Features fields read on the ReSTIR path (common.h:89-136). */
typedef struct restir_features {
    uint32_t ray_trace_mode;                 /* restir_mode */
    uint32_t initial_light_samples;          /* M  */
    uint32_t num_samples_in_reservoir;       /* N  (1..RESTIR_MAX_N) */
    uint32_t num_neighbours_to_sample;       /* k  */
    uint32_t spatial_resample_radius;        /* r  */
    uint32_t spatial_resampling_passes;
    uint32_t temporal_clamp_m;
    uint8_t  initial_samples_visibility_check;
    uint8_t  unbiased_combination;
    uint8_t  spatial_reuse;
    uint8_t  spatial_reuse_visibility_check;
    uint8_t  temporal_reuse;
    uint8_t  enable_shading;
    uint8_t  enable_texture_mapping;         /* diffuseAlbedo's switch (utils.cpp:33-37) */
    uint8_t  enable_tone_mapping;
    float    gamma;
    float    exposure;
    /* R-MIS / R-OMIS parameters and the neighbour-selection heuristic (common.h:110-121) -- ABI v2 */
    uint8_t  neighbour_same_geometry;                   /* true */
    uint8_t  use_progressive_romis;                     /* false */
    uint8_t  save_alphas_visualisation;                 /* true; R-OMIS writes the per-distribution bitmaps
                                                           when the context has a renders dir
                                                           (restir_set_renders_dir) */
    uint8_t  reserved0;
    float    neighbour_max_depth_difference_fraction;   /* 0.10 */
    float    neighbour_max_normal_angle_difference_radians; /* 0.436332, compared with the normals' dot product
                                                           as areSimilar does (neighbour_selection.cpp:16-18) */
    uint32_t max_iterations_mis;                        /* 5 */
    uint32_t neighbour_selection_strategy;              /* restir_neighbour_strategy, default SIMILAR */
    uint32_t mis_weight_rmis;                           /* restir_mis_weight, default EQUAL */
    uint32_t progressive_update_mod;                    /* 1 */
} restir_features;

/* Defaults of struct Features (common.h:89-136), rayTraceMode forced to ReSTIR. */
void restir_features_default(restir_features* out);

/* Keyed RNG (see header comment). Exposed for tests and tools. */
uint32_t restir_rng_key(uint32_t seed, uint32_t frame, uint32_t stage, uint32_t pass);
uint32_t restir_rng_draw(uint32_t key, uint32_t global_pixel, uint32_t slot);

/* Host-side camera derivation, identical to the device path's constants. */
void restir_camera_derive(const restir_camera* cam, restir_camera_frame* out);

/* ---- screen tiling (multi-GPU) : pure host logic, callable without a GPU ---------------------------- */
/* Tile (tx, ty) of a tiles_x x tiles_y grid over a global width x height image.  The tile's region is
 * [x0, x0+w) x [y0, y0+h); its ghost region (what a rank must compute locally so that `passes` spatial
 * passes of radius r give bit-identical results to a single-GPU frame) is the region grown by
 * passes*r pixels, clipped to the image. */
typedef struct restir_tile {
    uint32_t global_width, global_height;
    uint32_t x0, y0, width, height;          /* owned pixels */
    uint32_t gx0, gy0, gwidth, gheight;      /* computed pixels (owned + ghost zone) */
} restir_tile;
restir_status restir_tile_plan(uint32_t global_width, uint32_t global_height, uint32_t tiles_x, uint32_t tiles_y,
                               uint32_t rank, uint32_t ghost, restir_tile* out);

/* Reservoir halo exchange between tiles (multi-GPU frames with temporal reuse).  In halo mode a
 * rank computes RIS / temporal / spatial / final only on its owned tile; before every spatial pass the
 * reservoirs within `radius` of a tile border are exchanged with the adjacent ranks.  restir_halo_plan lists,
 * for `rank`, one segment per adjacent rank (ascending rank order): `send[i]` = the rectangle of this rank's
 * owned pixels that rank send[i].rank reads, `recv[i]` = the rectangle of that rank's owned pixels this rank
 * reads.  A segment's bytes = w * h * N * 32, laid out [sub-reservoir j][pixel row-major][res_a, res_b];
 * `offset` is its byte offset in the contiguous send / recv buffer (segments back to back in list order).
 * Pure host; every rank computes the same plan.  *count: in = capacity (>= 8 suffices), out = segments. */
typedef struct restir_halo_segment {
    uint32_t rank;
    uint32_t x0, y0, width, height;          /* global pixel rectangle */
    uint64_t offset, bytes;
} restir_halo_segment;
restir_status restir_halo_plan(uint32_t global_width, uint32_t global_height, uint32_t tiles_x, uint32_t tiles_y,
                               uint32_t rank, uint32_t radius, uint32_t N, restir_halo_segment* send,
                               restir_halo_segment* recv, uint32_t* count);

/* Uneven screen tiles (cost-balanced plans for frames whose geometry is not spread evenly).  A layout
 * cuts the image into tiles_x columns at x_cuts (x_cuts[0] = 0 < x_cuts[1] < ... < x_cuts[tiles_x] = width) and
 * each column c into tiles_y rows at its own y_cuts[c] (0 = y_cuts[c][0] < ... < y_cuts[c][tiles_y] = height); rank
 * ty * tiles_x + tx owns [x_cuts[tx], x_cuts[tx + 1]) x [y_cuts[tx][ty], y_cuts[tx][ty + 1]).  One rectangle per rank,
 * every pixel owned once; with tiles_y <= 4 a rank has at most 2 + 2 tiles_y halo partners (<= 8 segments).  Any
 * layout renders bit-identically to one GPU: the spatial clamp is global (render_utils.cpp:109-110) and the RNG is
 * keyed by global pixel.  restir_layout_even is restir_tile_plan's split; restir_tile_plan / restir_halo_plan /
 * restir_halo_ops / restir_halo_begin are the _layout functions over it. */
#define RESTIR_MAX_TILES_X 16u
#define RESTIR_MAX_TILES_Y 16u
typedef struct restir_tile_layout {
    uint32_t global_width, global_height, tiles_x, tiles_y;
    uint32_t x_cuts[RESTIR_MAX_TILES_X + 1];
    uint32_t y_cuts[RESTIR_MAX_TILES_X][RESTIR_MAX_TILES_Y + 1];
} restir_tile_layout;
restir_status restir_layout_even(uint32_t global_width, uint32_t global_height, uint32_t tiles_x, uint32_t tiles_y,
                                 restir_tile_layout* out);
/* A layout balancing `cost` -- a cost_w x cost_h grid of per-cell work over the image (row-major, row 0 = the bottom
 * row, cell (i, j) = the pixels x with floor(x cost_w / width) = i and y with floor(y cost_h / height) = j, the cell's
 * cost spread evenly over them): the x cuts split the column totals into equal shares, then each column's y cuts
 * split its own row totals.  Cuts are rounded to multiples of align_x / align_y (0: 1) and keep every tile at least
 * one alignment unit wide / high.  *efficiency (may be NULL) = mean over ranks of a rank's cost / the largest. */
restir_status restir_layout_balanced(uint32_t global_width, uint32_t global_height, uint32_t tiles_x, uint32_t tiles_y,
                                     const float* cost, uint32_t cost_w, uint32_t cost_h, uint32_t align_x,
                                     uint32_t align_y, restir_tile_layout* out, double* efficiency);
/* The cost share a layout gives each rank (out[rank], summing to 1) under the same cost grid. */
restir_status restir_layout_shares(const restir_tile_layout* layout, const float* cost, uint32_t cost_w, uint32_t cost_h,
                                   double* out);
restir_status restir_layout_tile(const restir_tile_layout* layout, uint32_t rank, uint32_t ghost, restir_tile* out);
restir_status restir_layout_halo_plan(const restir_tile_layout* layout, uint32_t rank, uint32_t radius, uint32_t N,
                                      restir_halo_segment* send, restir_halo_segment* recv, uint32_t* count);

/* ---- context ----------------------------------------------------------------------------------------- */
/* (halo-mode frame functions: after the render / stage API below) */
typedef struct restir_ctx   restir_ctx;
typedef struct restir_frame restir_frame;

const char*   restir_last_error(void);
int           restir_abi_version(void);
restir_status restir_device_count(int* out);

restir_status restir_create(int device, restir_ctx** out);
void          restir_destroy(restir_ctx* ctx);
restir_status restir_set_seed(restir_ctx* ctx, uint32_t seed, uint32_t frame_index);
/* The reference's RENDERS_DIR (a build-time constant there) for this context's file side outputs; NULL or "" =
 * none (the default).  With a dir, an R-OMIS render with features->save_alphas_visualisation writes
 * visualiseAlphas' bitmaps after every iteration (render.cpp:227-229, render_utils.cpp:189-243):
 * <dir>/<"%d-%m-%Y %H-%M-%S" local time>/Distribution <i> - <Red|Green|Blue>.bmp for technique i of the k + 1,
 * each pixel mix(black, (1, .5, 0), alpha) for alpha > 0 and mix(black, (0, .5, 1), -alpha) otherwise, the
 * alphas solved from the technique matrix and contribution vectors so far -- byte for byte the reference's images
 * (iterations within one second share the folder and overwrite, as there).  The dirs are created as needed;
 * a file that cannot be written fails the render (RESTIR_ERR_INVALID). */
restir_status restir_set_renders_dir(restir_ctx* ctx, const char* dir);

/* Uploads the scene: materials, light SoA table, and the flattened BVH built on the host (replaces
 * EmbreeInterface(scene), embree_interface.cpp:14-51). */
restir_status restir_set_scene(restir_ctx* ctx, const restir_mesh* meshes, uint32_t num_meshes,
                               const restir_light* lights, uint32_t num_lights);
/* The same with the Images textured materials point at (diffuseAlbedo's kdTexture, utils.cpp:33-37): with
 * features->enable_texture_mapping (the Features default, common.h:95) a textured material's diffuse colour
 * is acquireTexel(kdTexture, the hit's interpolated texCoord) (texture.cpp:4-9, embree_interface.cpp:80-81).
 * Texture coordinates outside [0, 1] read out of bounds in the reference (its float -> size_t conversion);
 * here they clamp to the edge texel. */
restir_status restir_set_scene_textured(restir_ctx* ctx, const restir_mesh* meshes, uint32_t num_meshes,
                                        const restir_light* lights, uint32_t num_lights,
                                        const restir_texture* textures, uint32_t num_textures);

/* renderRayTraced (render.cpp:268-290) by features->ray_trace_mode:
 * RMIS / ROMIS -- renderRMIS / renderROMIS (render.cpp:64-265): primary hits -> neighbour selection grid ->
 * max_iterations_mis x (initial RIS -> per-pixel MIS combination over the pixel's neighbourhood) -> screen.
 * Whole images only (tile NULL or covering the image), no temporal predecessor, *out_next = NULL (the reference
 * returns std::nullopt).  R-OMIS needs k + 1 <= RESTIR_ROMIS_MAX_TECHNIQUES and at least k candidates in every
 * pixel's window (the reference indexes past the neighbourhood otherwise).
 * RESTIR -- renderReSTIR (render.cpp:28-62): primary hits -> initial RIS -> [temporal if prev] -> [spatial x P] ->
 * final shading + tone map.  `prev` may be NULL (no temporal predecessor).  `out_next` (nullable) receives
 * a new reference to the frame's final reservoir grid.  `out_rgb` (nullable, host, width*height*3 floats,
 * row 0 = top) -- when NULL the call only enqueues work and returns without synchronising; the image stays
 * on the device (restir_download_rgb).  `tile` (nullable) restricts the frame to one screen tile of a
 * larger image (multi-GPU); NULL = the whole width x height image.  A tiled frame's grid is defined on the owned
 * rect: its ghost ring (computed only for the owned pixels' spatial neighbourhoods) holds intermediate values. */
restir_status restir_render(restir_ctx* ctx, const restir_camera* cam, const restir_features* features,
                            uint32_t width, uint32_t height, const restir_tile* tile,
                            const restir_frame* prev, restir_frame** out_next, float* out_rgb);

restir_status restir_frame_retain(restir_frame* frame);
/* Drops a reference.  The last one hands the grid's device records back to the producing context for re-use,
 * ordered on the GPU after every kernel that wrote or read them (no host or device-wide synchronisation). */
void          restir_frame_release(restir_frame* frame);

/* The grid a frame holds -- renderReSTIR's returned ReservoirGrid (render.h:25-28, render.cpp:61) -- over the
 * frame's computed view (vw x vh pixels at (vx0, vy0) of the W x H image; the whole image for untiled frames).
 * restir_frame_info: any pointer may be NULL.  restir_frame_download copies, per sub-reservoir j and view pixel
 * p (index j * vw * vh + p, rows y = 0 bottom): outputSamples[j].position -> pos[3 i], .color -> color[3 i],
 * .W -> w[i], sampleNums[j] -> m[i]; any output may be NULL, each holds vw * vh * N entries (x3 for pos /
 * color).  Waits for the frame's producer, then copies synchronously. */
restir_status restir_frame_info(const restir_frame* frame, uint32_t* width, uint32_t* height, uint32_t* vx0,
                                uint32_t* vy0, uint32_t* vw, uint32_t* vh, uint32_t* n);
restir_status restir_frame_download(const restir_frame* frame, float* pos, float* color, float* w, uint32_t* m);
restir_status restir_synchronize(restir_ctx* ctx);

/* Last rendered image (owned pixels), host float RGB, row 0 = top. */
restir_status restir_download_rgb(restir_ctx* ctx, float* out_rgb, size_t count);

/* ---- stage-level access for parity tests and profiling ---------------------------------------------- *
 * Buffers are the device SoA layout (DESIGN.md "Data layout"), one entry per pixel of the computed region
 * (row-major, y = 0 bottom), and for reservoirs [N][pixels]:
 *   gbuf_n_t   : float4 (N.xyz, t)         gbuf_p_mat : float4 (P.xyz, bits(material index))
 *   res_a      : float4 (light pos.xyz, W) res_b      : float4 (light colour.xyz, bits(M))
 *   res_dbg    : float2 (wSum, chosenSampleWeight)
 *   gbuf_uv    : float2 (the hit's interpolated texCoord; written and read only for scenes with textures) */
typedef enum restir_buffer {
    RESTIR_BUF_GBUF_N_T   = 0,   /* read by the spatial heuristic for every neighbour: keep it compact */
    RESTIR_BUF_GBUF_P_MAT = 1,
    RESTIR_BUF_RES_A      = 2,   /* reservoir slot 0 ("current") */
    RESTIR_BUF_RES_B      = 3,
    RESTIR_BUF_RES_DBG    = 4,
    RESTIR_BUF_PREV_A     = 5,   /* reservoir slot 1 (temporal predecessor / spatial ping-pong) */
    RESTIR_BUF_PREV_B     = 6,
    RESTIR_BUF_PREV_DBG   = 7,
    RESTIR_BUF_RGB        = 8,   /* float3 per owned pixel, row 0 = top */
    /* R-MIS / R-OMIS stage buffers (restir_stage_neighbours / restir_stage_mis_accumulate):
     *   mis_nbr : uint32 [1 + cap][pixels]: row 0 = neighbourhood size c, rows 1..c = the neighbourhood's pixel
     *             indices y * width + x, the pixel itself first (cap = restir_stage_mis_capacity)
     *   mis_acc : float [rows][pixels].  R-MIS: colour sum (3 rows).  R-OMIS with T = k + 1: technique matrix A
     *             (T*T rows, element (i, j) in row i + j*T), contribution vectors b (3*T rows, colour c, technique
     *             i in row T*T + c*T + i), progressive alphas (3*T rows after b, same order), progressive colour
     *             (3 rows) */
    RESTIR_BUF_MIS_NBR    = 9,
    RESTIR_BUF_MIS_ACC    = 10,
    RESTIR_BUF_GBUF_UV    = 11
} restir_buffer;
#define RESTIR_ROMIS_MAX_TECHNIQUES 8u   /* k + 1 distributions per pixel (the technique matrix lives in registers) */

/* Allocates stage buffers for a width x height region with N sub-reservoirs (idempotent). */
restir_status restir_stage_configure(restir_ctx* ctx, uint32_t width, uint32_t height, uint32_t n);
restir_status restir_stage_upload(restir_ctx* ctx, restir_buffer which, const void* host, size_t bytes);
restir_status restir_stage_download(restir_ctx* ctx, restir_buffer which, void* host, size_t bytes);

/* Individual passes on the stage buffers (the camera supplies the ray origin every pass shades from).
 * `debug` != 0 also writes the (wSum, chosenSampleWeight) buffer of the pass output.
 *   primary  : -> GBUF_*                         ris      : GBUF -> RES_*
 *   temporal : RES_* (current) + PREV_* -> RES_*
 *   spatial  : ONE pass, RES_* -> new RES_* (the input becomes PREV_*); call once per pass with that
 *              pass's key restir_rng_key(seed, frame, RESTIR_STAGE_SPATIAL, pass)
 *   final    : RES_* -> RGB                                                                                */
restir_status restir_stage_primary(restir_ctx* ctx, const restir_camera* cam);
restir_status restir_stage_ris(restir_ctx* ctx, const restir_camera* cam, const restir_features* f, uint32_t rng_key,
                               int debug);
restir_status restir_stage_temporal(restir_ctx* ctx, const restir_camera* cam, const restir_features* f,
                                    uint32_t rng_key, int debug);
restir_status restir_stage_spatial(restir_ctx* ctx, const restir_camera* cam, const restir_features* f,
                                   uint32_t rng_key, int debug);
restir_status restir_stage_final(restir_ctx* ctx, const restir_camera* cam, const restir_features* f);

/* R-MIS / R-OMIS stages (render.cpp:64-265) on the stage buffers (the stage region is the whole image):
 *   neighbours     : GBUF -> MIS_NBR (generateResampleIndicesGrid); keys = RESTIR_STAGE_NEIGHBOURS passes 0 and 1
 *   mis_accumulate : iteration i's reservoirs RES_A / RES_B / RES_DBG (restir_stage_ris with debug != 0) + GBUF +
 *                    MIS_NBR -> MIS_ACC (features->ray_trace_mode selects R-MIS or R-OMIS; MIS_ACC is zeroed
 *                    when iteration == 0)
 *   mis_finish     : MIS_ACC -> RGB (combineToScreen, or R-OMIS's per-pixel least-squares solve)
 * restir_stage_mis_capacity: the neighbourhood capacity `cap` of MIS_NBR for these features. */
restir_status restir_stage_neighbours(restir_ctx* ctx, const restir_features* f, uint32_t key_similar,
                                      uint32_t key_dissimilar);
restir_status restir_stage_mis_accumulate(restir_ctx* ctx, const restir_camera* cam, const restir_features* f,
                                          uint32_t iteration);
restir_status restir_stage_mis_finish(restir_ctx* ctx, const restir_features* f);
restir_status restir_stage_mis_capacity(restir_ctx* ctx, const restir_features* f, uint32_t* out_cap);

/* Batched least squares as renderROMIS solves its systems (Eigen CompleteOrthogonalDecomposition::solve,
 * render_utils.h:52): for each of `count` systems x = the minimum-norm least-squares solution of A x = b, A n x n
 * column-major (n*n floats per system), b and x n floats per system; host arrays, n <= RESTIR_ROMIS_MAX_TECHNIQUES.
 * The device routine of the R-OMIS finish, exposed for the parity tests. */
restir_status restir_debug_cod_solve(restir_ctx* ctx, uint32_t n, const float* A, const float* b, float* x,
                                     size_t count);

/* Device portable powf / expf over arrays (parity of the device math with the oracle's). */
restir_status restir_debug_math(restir_ctx* ctx, const float* x, const float* y, float* out_pow, float* out_exp,
                                size_t n);

/* ---- halo-mode frames (multi-GPU tiles with temporal reuse) ----------------------------------------------
 * The stages of restir_render for rank `rank` of a tiles_x x tiles_y split, with the spatial passes' ghost
 * zone replaced by a reservoir exchange (restir_halo_plan).  Per frame:
 *   restir_halo_begin   primary rays on the tile + radius ring, RIS and temporal reuse on the owned tile;
 *                       returns the pack / unpack buffer sizes
 *   per spatial pass:   restir_halo_pack(send) -> move segment i of send to rank send[i].rank and receive
 *                       recv[i] from rank recv[i].rank (RCCL ncclSend/ncclRecv, torch.distributed, ...) ->
 *                       restir_halo_unpack(recv) -> restir_halo_spatial (or the split / native forms below)
 *   restir_halo_end     final shading of the owned tile; *out_next = the grid for the next frame's temporal reuse
 * Bit-identical to the same pixels of a single-GPU restir_render frame.  Buffers are device memory (or host
 * memory when host_memory != 0, staged by the library); pack returns after the buffer is written, unpack
 * expects the received bytes complete when called. */
restir_status restir_halo_begin(restir_ctx* ctx, const restir_camera* cam, const restir_features* features,
                                uint32_t width, uint32_t height, uint32_t tiles_x, uint32_t tiles_y, uint32_t rank,
                                const restir_frame* prev, uint64_t* send_bytes, uint64_t* recv_bytes);
/* restir_halo_begin over an uneven layout (restir_tile_layout): rank `rank`'s tile of it */
restir_status restir_halo_begin_layout(restir_ctx* ctx, const restir_camera* cam, const restir_features* features,
                                       const restir_tile_layout* layout, uint32_t rank, const restir_frame* prev,
                                       uint64_t* send_bytes, uint64_t* recv_bytes);
restir_status restir_halo_pack(restir_ctx* ctx, void* send_buf, uint64_t bytes, int host_memory);
restir_status restir_halo_unpack(restir_ctx* ctx, const void* recv_buf, uint64_t bytes, int host_memory);
restir_status restir_halo_spatial(restir_ctx* ctx);
restir_status restir_halo_end(restir_ctx* ctx, restir_frame** out_next, float* out_rgb);

/* A spatial pass in two launches, so that the exchange overlaps computation: the interior of the owned tile
 * (pixels more than `radius` from every side that faces another tile: their neighbourhoods never reach the
 * ring) reads no exchanged reservoir and may run as soon as the pass's pack is issued; the border strips run
 * after the unpack.  Per pass: pack -> spatial_interior -> (exchange) -> unpack -> spatial_border.
 * restir_halo_spatial == spatial_interior + spatial_border.  Same results either way. */
restir_status restir_halo_spatial_interior(restir_ctx* ctx);
restir_status restir_halo_spatial_border(restir_ctx* ctx);

/* Native RCCL transport of the halo (the exchange runs inside the library, no host round trip).  One rank
 * calls restir_rccl_unique_id and hands the RESTIR_RCCL_ID_BYTES bytes to every rank (any side channel);
 * every rank then calls restir_halo_attach_rccl(ctx, id, nranks, rank) once (ncclCommInitRank on the context's
 * device; the communicator lives with the context), or restir_halo_attach_comm with the caller's own
 * ncclComm_t (not owned, it must outlive the context's use).  restir_halo_pass then runs one spatial pass of
 * the frame begun by restir_halo_begin: pack on the context's stream; ncclGroupStart / ncclSend+ncclRecv per
 * plan segment / ncclGroupEnd on the context's communication stream, ordered after the pack by an event; the
 * interior pass on the context's stream concurrently with the transfer; unpack and border pass after it.
 * Nothing synchronises the host.  librccl is loaded on first use (RESTIR_ERR_UNSUPPORTED when absent). */
#define RESTIR_RCCL_ID_BYTES 128u
restir_status restir_rccl_unique_id(void* out, size_t bytes);
restir_status restir_halo_attach_rccl(restir_ctx* ctx, const void* unique_id, uint32_t nranks, uint32_t rank);
restir_status restir_halo_attach_comm(restir_ctx* ctx, void* nccl_comm);
restir_status restir_halo_pass(restir_ctx* ctx);

/* The point-to-point operations restir_halo_pass posts for every spatial pass, in posting order: one ncclSend
 * then one ncclRecv per restir_halo_plan segment, all inside one ncclGroupStart / ncclGroupEnd on the
 * communication stream.  Each: kind, peer (tile rank), byte offset into the pass's device send / receive buffer,
 * bytes, and the global pixel rectangle the bytes hold ([sub-reservoir][pixel row-major][res_a, res_b]).  Pure
 * host: restir_halo_begin builds the list restir_halo_pass posts from with this same function.  *count: in =
 * capacity (2 per segment; 16 suffices), out = operations. */
#define RESTIR_HALO_OP_SEND 0u
#define RESTIR_HALO_OP_RECV 1u
typedef struct restir_halo_op {
    uint32_t kind, peer;
    uint64_t offset, bytes;
    uint32_t x0, y0, width, height;          /* global pixel rectangle */
} restir_halo_op;
restir_status restir_halo_ops(uint32_t global_width, uint32_t global_height, uint32_t tiles_x, uint32_t tiles_y,
                              uint32_t rank, uint32_t radius, uint32_t N, restir_halo_op* ops, uint32_t* count);
restir_status restir_layout_halo_ops(const restir_tile_layout* layout, uint32_t rank, uint32_t radius, uint32_t N,
                                     restir_halo_op* ops, uint32_t* count);

/* Record-only mode of restir_halo_pass: the native transport's plumbing checked without a second GPU.  With
 * restir_halo_record(ctx, 1) a pass needs no communicator and posts no RCCL operation; it appends every step it
 * issues to the context's log instead -- on the context stream (0) the pack launch and the `packed` event, on the
 * communication stream (1) the wait for it, the group with each send / receive (peer, offset, bytes), the `moved`
 * event, then on the context stream the interior launch, the wait for `moved`, the unpack and the border launches
 * -- and otherwise runs the pass with a zeroed receive buffer (the border strips then read zero reservoirs: not a
 * valid image).  restir_halo_log copies the log out in issue order and clears it; *count: in = capacity, out =
 * entries (RESTIR_ERR_INVALID, nothing cleared, when the capacity is short: *count = entries needed).  Attaching a
 * communicator (restir_halo_attach_rccl / _attach_comm) ends record-only mode. */
#define RESTIR_HALO_EV_PACK         0u
#define RESTIR_HALO_EV_RECORD       1u   /* peer: 0 = `packed`, 1 = `moved` */
#define RESTIR_HALO_EV_WAIT         2u   /* peer: the event waited for, as above */
#define RESTIR_HALO_EV_GROUP_START  3u
#define RESTIR_HALO_EV_SEND         4u
#define RESTIR_HALO_EV_RECV         5u
#define RESTIR_HALO_EV_GROUP_END    6u
#define RESTIR_HALO_EV_INTERIOR     7u
#define RESTIR_HALO_EV_UNPACK       8u
#define RESTIR_HALO_EV_BORDER       9u
typedef struct restir_halo_event {
    uint32_t what, stream, peer, pass;
    uint64_t offset, bytes;
} restir_halo_event;
restir_status restir_halo_record(restir_ctx* ctx, int on);
restir_status restir_halo_log(restir_ctx* ctx, restir_halo_event* out, uint32_t* count);

/* ---- frame output (pure host, no device needed) --------------------------------------------------------
 * restir_rgb_to_rgba8: Screen::writeBitmapToFile's conversion (screen.cpp:45-51): glm::clamp(c, 0, 1), then
 * glm::u8vec4(vec4(c, 1) * 255) (truncation toward zero), for `pixels` float RGB triples -> RGBA bytes.
 * restir_encode_bmp / restir_write_bmp: that conversion of a width x height float RGB image (row 0 = top, the
 * layout restir_render returns) written as stbi_write_bmp(path, w, h, 4, data) writes it (screen.cpp:55):
 * BITMAPV4 header, 32 bpp BGRA rows bottom-up.  encode: out == NULL queries *length.
 * restir_features_json: the configuration record renderRayTraced saves per render (render.cpp:281-287,
 * cereal::JSONOutputArchive of struct Features, common.h:138-147), byte for byte; `extra` carries the Features
 * fields the ReSTIR path does not read (NULL: the struct's defaults).  out == NULL queries *length (without the
 * terminating NUL, which is written).  Non-finite gamma / exposure: RESTIR_ERR_INVALID (cereal throws). */
typedef struct restir_features_record_extra {
    uint8_t  enable_recursive;         /* false */
    uint8_t  enable_hard_shadow;       /* true  */
    uint8_t  enable_soft_shadow;       /* true  */
    uint8_t  enable_normal_interp;     /* true  */
    uint8_t  enable_accel_structure;   /* true  */
    uint8_t  reserved[3];
    uint32_t max_reflection_recursion; /* 5 */
} restir_features_record_extra;
restir_status restir_rgb_to_rgba8(const float* rgb, size_t pixels, uint8_t* rgba);
restir_status restir_encode_bmp(const float* rgb, uint32_t width, uint32_t height, uint8_t* out, size_t capacity,
                                size_t* length);
restir_status restir_write_bmp(const char* path, const float* rgb, uint32_t width, uint32_t height);
restir_status restir_features_json(const restir_features* features, const restir_features_record_extra* extra,
                                   char* out, size_t capacity, size_t* length);

/* Measured HBM read bandwidth of this device (the roofline's practical ceiling next to the 8 TB/s spec): a
 * streaming-read kernel over `bytes` (rounded down to 16 B; pass >= 1 GiB to defeat the 256 MB Infinity
 * Cache), timed with HIP events over `iters` launches.  *out_gbps = bytes * iters / time / 1e9. */
restir_status restir_measure_read_bandwidth(restir_ctx* ctx, uint64_t bytes, uint32_t iters, double* out_gbps);

/* Background pixels of the last restir_render frame (the compulsory-byte roofline, bench.py roofline.frac_compulsory):
 * the pixels of the RIS tiles (32 x 8 over the frame's computed region) whose every pixel missed the scene with the RIS
 * result known -- the MissTiles flags from which the spatial passes and final shading write those tiles without reading
 * them.  *computed = the region's pixels; *background = 0 when the frame kept no flags (temporal reuse, N > 2, knob
 * "miss.tiles" off).  Synchronises the context's stream. */
restir_status restir_background_pixels(restir_ctx* ctx, uint64_t* background, uint64_t* computed);

/* ---- timing ----------------------------------------------------------------------------------------- */
/* When enabled, every kernel of restir_render / restir_stage_* is bracketed by HIP events on the
 * context's stream; restir_timings returns the accumulated milliseconds and launch counts per kernel. */
typedef enum restir_kernel {
    RESTIR_K_PRIMARY = 0, RESTIR_K_RIS = 1, RESTIR_K_TEMPORAL = 2, RESTIR_K_SPATIAL = 3, RESTIR_K_FINAL = 4,
    RESTIR_K_PRIMARY_RIS = 5,   /* primary rays + initial RIS fused (restir_render, tuning "fuse.primary_ris") */
    RESTIR_K_MIS = 6,           /* R-MIS / R-OMIS neighbour selection, per-iteration combination, finish */
    RESTIR_K_COUNT = 7
} restir_kernel;
restir_status restir_enable_timing(restir_ctx* ctx, int enable);
/* Launch-shape knobs (never change results): "primary.lds", "ris.lds", "final.lds" (stage the BVH / light table in
 * LDS when it fits), "fuse.primary_ris" (restir_render runs primary rays + RIS as one kernel), "fuse.temporal" (with a predecessor
 * grid, temporal reuse runs inside that kernel: N = 1 / 2, point lights, the light table in LDS; default 1), "spatial.lean" (the
 * lean N = 1 / 2 passes; 0: the general kernels), "timing.mask": the kernels (bit 1 << RESTIR_K_*) restir_enable_timing
 * brackets with HIP events (default all).  "bvh.max_leaf": triangles per BVH leaf for the next restir_set_scene
 * (default 2).  "layout.records": restir_render's buffers as per-pixel records [n_t, res_a, res_b] (1) or SoA planes
 * (0, default).  "ris.compact": initial RIS (N = 1, 2) reads a compact light table when the scene allows one -- point
 * lights only, a light grid, one-colour parallelograms -- instead of the 7-float4 records (default 1; restir_set_scene
 * detects the form bit for bit).  "spatial.xcd_rows|xcd_cols" (the spatial pass's XCD chunk shape; 255 = automatic),
 * "spatial.th" (0: auto, 1: 32x8, 2: 32x16 tiles), "spatial.handles" (N = 1 biased passes over a point-light scene read
 * sample handles, k_spatial1h; with temporal reuse when the predecessor frame carries the handles its last pass wrote
 * -- N = 1 point lights, no ghost ring, the same scene upload -- else its reservoir planes are read; default 1),
 * "spatial.gather" (the point-light handle pass on 32x16 tiles gathers the accepted neighbours' handles instead of
 * staging the handle windows in LDS, k_spatial1hg_t2; default 1), "spatial.n2h" (N = 2 biased passes over a point-light
 * scene without temporal reuse read 16-byte handle records, k_spatial2hg; default 1), "final.qbvh" (final shading's
 * shadow rays walk 16-byte quantized BVH nodes: 0 never, 1 always, 2 = at N = 2, the default), "primary.tl" (the fused
 * primary + RIS kernel's primary rays test their 32x8 tile's candidate triangles -- those not wholly outside the tile's
 * ray pyramid -- instead of walking the BVH; default 1), "ris.late" (stage the light table after the primary rays, only
 * for tiles that need it), "final.sort" (bin each tile's shadow rays by target), "final.miss" (final shading reads only p_mat and
 * (pos, W) for a primary-ray miss), "miss.tiles" (background-tile flags from RIS to the spatial passes and final
 * shading, N <= 2 without temporal reuse), "miss.gbuf" (0 / 1 / 2 = auto: RIS also skips background tiles' G-buffer
 * stores), "timing.every" / "timing.fence" (event sampling), "mis.chunk" (R-OMIS samples per launch pair).  All default
 * on where measured faster.  Round 5 removed the knobs measured slower in two rounds (persistent *.blocks grids, the
 * RIS work queue, the gather-only spatial pass, non-XCD / row-wave tile orders, 1-D primary / final maps, frames in
 * flight): unknown keys are RESTIR_ERR_INVALID. */
restir_status restir_set_tuning(restir_ctx* ctx, const char* key, int value);
restir_status restir_timings(restir_ctx* ctx, double* ms /*[RESTIR_K_COUNT]*/, uint64_t* launches /*[RESTIR_K_COUNT]*/);
restir_status restir_reset_timings(restir_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* RESTIR_C_H */

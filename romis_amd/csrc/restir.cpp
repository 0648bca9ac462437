// restir.cpp -- implementation of the C ABI in include/restir_c.h (host side of libromis_amd.so).
//
// Drop-in for renderReSTIR / renderRayTraced (src/rendering/render.cpp:28-62, :268-290): a context owns one
// HIP device + stream, the uploaded scene (materials, lights, flattened BVH) and the per-frame device
// buffers; every pass is one hand-written gfx950 kernel (kernels.hip) enqueued on the context's stream.
#include "restir_c.h"

#include <rccl/rccl.h>

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <dlfcn.h>
#include <filesystem>
#include <memory>
#include <mutex>
#include <string>
#include <system_error>
#include <vector>

#include "bvh.h"
#include "device_math.h"
#include "launch.h"
#include "restir_types.h"

namespace romis {
bool write_bmp_words(const char* path, uint32_t width, uint32_t height, const uint32_t* words);   // screen.cpp
}
using namespace romis;

// ---------------------------------------------------------------------------------------------------------
// errors
namespace {
thread_local std::string g_err;

restir_status fail(restir_status s, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return s;
}

#define HIP_TRY(expr)                                                                                   \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess) return fail(RESTIR_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

#define ST_TRY(expr)                            \
    do {                                        \
        restir_status s_ = (expr);              \
        if (s_ != RESTIR_OK) return s_;         \
    } while (0)

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    restir_status ensure(size_t n) {
        if (n <= bytes && p) return RESTIR_OK;
        release();
        if (n == 0) n = 16;
        hipError_t e = hipMalloc(&p, n);
        if (e != hipSuccess) { p = nullptr; bytes = 0; return fail(RESTIR_ERR_HIP, "hipMalloc(%zu): %s", n, hipGetErrorString(e)); }
        bytes = n;
        return RESTIR_OK;
    }
    restir_status upload(const void* h, size_t n, hipStream_t s) {
        ST_TRY(ensure(n));
        HIP_TRY(hipMemcpyAsync(p, h, n, hipMemcpyHostToDevice, s));
        return RESTIR_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

uint32_t f2u(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
float u2f(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
// the exponent classes material_pow branches on (ROMIS_PWC_*): glibc's checkint(y) and zeroinfnan(y) cases
uint32_t pw_class(float y) {
    uint32_t iy; std::memcpy(&iy, &y, 4);
    if (std::isnan(y)) return ROMIS_PWC_NAN;
    if (y == 0.0f) return ROMIS_PWC_ZERO;
    if (std::isinf(y)) return y > 0.0f ? ROMIS_PWC_PINF : ROMIS_PWC_NINF;
    uint32_t c = y < 0.0f ? ROMIS_PWC_NEG : 0u;
    const int e = (int)(iy >> 23 & 0xff);
    if (e < 0x7f) return c;
    if (e > 0x7f + 23) return c | ROMIS_PWC_INT;
    if (iy & ((1u << (0x7f + 23 - e)) - 1)) return c;
    return c | ((iy & (1u << (0x7f + 23 - e))) ? ROMIS_PWC_INT | ROMIS_PWC_ODD : ROMIS_PWC_INT);
}

struct Pending {
    int kernel;
    hipEvent_t start, stop;
};

}  // namespace

// Record buffers that temporal frames hand back (restir_frame_release): each comes with the events of the work
// that last touched it (the producing frame's kernels, every render that read it as a predecessor), so a context
// re-uses it by making its stream wait on those events -- no hipMalloc / hipFree / device-wide sync per frame.
struct FramePool {
    struct Entry {
        DevBuf buf;
        std::vector<hipEvent_t> busy;
    };
    std::mutex mu;
    std::vector<Entry> free;
    bool closed = false;   // the owning context is gone: returned buffers are freed
    int device = 0;
    // the owning context's stream (null once closed): its own later frames read a predecessor's records on it without
    // recording read events (used_prev), so a drain waits for that stream before the records are freed
    hipStream_t owner = nullptr;
    static void drain(Entry& e) {
        for (hipEvent_t ev : e.busy) { (void)hipEventSynchronize(ev); (void)hipEventDestroy(ev); }
        e.busy.clear();
        e.buf.release();
    }
    // a buffer of at least `bytes` whose past users `stream` now waits for; false: none pooled
    bool take(size_t bytes, hipStream_t stream, DevBuf& out) {
        std::lock_guard<std::mutex> lk(mu);
        for (size_t i = 0; i < free.size(); i++) {
            if (free[i].buf.bytes < bytes) continue;
            for (hipEvent_t ev : free[i].busy) {
                (void)hipStreamWaitEvent(stream, ev, 0);
                (void)hipEventDestroy(ev);   // released when the recorded work completes
            }
            out = free[i].buf;
            free.erase(free.begin() + (long)i);
            return true;
        }
        return false;
    }
    // own: an event recorded on the owning context's own stream (the frame's `ready`): the next taker, on that stream,
    // is ordered after it already -- no wait packet (a 5-10 us gap between kernels); only a drain needs it
    void give(DevBuf buf, std::vector<hipEvent_t> busy, hipEvent_t own = nullptr) {
        Entry e{buf, std::move(busy)};
        std::lock_guard<std::mutex> lk(mu);
        if (closed || free.size() >= 4) {
            if (own) e.busy.push_back(own);
            // a later frame of the owner may still be reading the buffer on its stream (no read event): wait for it
            // rather than rely on hipFree's implicit synchronisation
            if (!closed && owner) (void)hipStreamSynchronize(owner);
            drain(e);
            return;
        }
        if (own) (void)hipEventDestroy(own);   // released when the recorded work completes
        free.push_back(std::move(e));
    }
    void close() {
        std::lock_guard<std::mutex> lk(mu);
        closed = true;
        owner = nullptr;   // the context synchronised its stream before closing the pool
        for (Entry& e : free) drain(e);
        free.clear();
    }
};

struct restir_frame {
    std::atomic<int> refs{1};
    int device = 0;
    DevBuf rec;   // the frame's reservoirs over its view: per-pixel records [n_t, a_0, b_0, ...] or [a planes | b planes]
    bool records = true;
    uint32_t W = 0, H = 0, vx0 = 0, vy0 = 0, vw = 0, vh = 0, N = 0;
    // frame handles: the scene upload (restir_ctx::scene_gen) whose light table the sample handles at rec's tail
    // (W, M | light index << 24, after the reservoir planes) index; 0 = none written
    uint64_t hgen = 0;
    std::shared_ptr<FramePool> pool;   // where rec goes back on release (the producing context's)
    std::mutex mu;
    hipEvent_t ready = nullptr;        // recorded on the producer's stream after its last kernel touching rec
    std::vector<hipEvent_t> reads;     // recorded after each render that read this frame as its predecessor
};

namespace {
hipEvent_t record_event(hipStream_t s) {
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return nullptr;
    if (hipEventRecord(ev, s) != hipSuccess) { (void)hipEventDestroy(ev); return nullptr; }
    return ev;
}
// a frame's records leave the producing context: remember where they go back to and when they are written
restir_frame* make_frame(const std::shared_ptr<FramePool>& pool, int device, hipStream_t s) {
    restir_frame* fr = new restir_frame();
    fr->device = device;
    fr->pool = pool;
    fr->ready = record_event(s);
    return fr;
}
// the consumer of a predecessor frame: its stream waits for the producer's kernels (another context / stream; a frame
// of this context -- own, its pool, which the frame keeps alive -- was produced on this stream: ordered already)
restir_status use_prev(const restir_frame* prev, int device, hipStream_t s, const FramePool* own) {
    if (prev->device != device)
        return fail(RESTIR_ERR_INVALID, "temporal predecessor lives on device %d, this context on %d", prev->device, device);
    if (prev->ready && prev->pool.get() != own) HIP_TRY(hipStreamWaitEvent(s, prev->ready, 0));
    return RESTIR_OK;
}
// ... and records that it read it, so the records are not recycled under the read (the pool's taker is its own
// context, on this stream when the reader is that context: ordered already)
void used_prev(const restir_frame* prev, hipStream_t s, const FramePool* own) {
    if (prev->pool.get() == own) return;
    restir_frame* fr = const_cast<restir_frame*>(prev);
    hipEvent_t ev = record_event(s);
    if (!ev) { (void)hipStreamSynchronize(s); return; }
    std::lock_guard<std::mutex> lk(fr->mu);
    fr->reads.push_back(ev);
}
}  // namespace

struct restir_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;

    // scene
    DevBuf nodes, tri_v0, tri_e1, tri_e2, tri_n0, tri_n1, tri_n2, materials, lights, light_c2, light_c4, light_col, tex_texels,
        tex_dims, tri_uv, nodes_q;
    SceneDev sdev{};
    bool has_scene = false;
    uint64_t scene_gen = 0;   // unique per scene upload (frame handles name the light table they index)

    // work buffers for one view
    uint32_t vw = 0, vh = 0, N = 0;
    DevBuf n_t, p_mat, ra[2], rb[2], dbg[2], rgb;   // stage API: SoA planes
    DevBuf uv;                                      // the G-buffer texCoord plane (textured scenes)
    DevBuf rec[2];                                  // restir_render / halo frames: per-pixel records
    std::shared_ptr<FramePool> pool = std::make_shared<FramePool>();
    DevBuf rp[2];                                   // their target-pdf cache planes (N = 1, planes layout)
    DevBuf vis;                                     // unbiased + visibility pass -> final shading: own-pixel ray
    DevBuf tmiss;                                   // RIS -> spatial passes / final shading: background tiles (MissTiles)
    uint32_t tmiss_w = 0, tmiss_h = 0;              // the last frame's computed region when it kept the flags (else 0)
    uint64_t last_px = 0;                           // the last frame's computed pixels
    DevBuf hnd[2];                                  // sample handles of rec[i] (N = 1 point lights, k_spatial1h)
    int cur = 0;
    uint32_t rgb_w = 0, rgb_h = 0;

    // launch-shape knobs (restir_set_tuning)
    Tuning tuning{};

    // RNG
    uint32_t seed = RESTIR_DEFAULT_SEED;
    uint32_t frame_index = 0;

    // halo-mode frame in flight (restir_halo_begin .. restir_halo_end)
    struct {
        bool active = false;
        uint32_t W = 0, H = 0, frame = 0, pass = 0, passes = 0;
        Region view{}, owned{};
        FeaturesDev f{};
        CameraDev camd{};
        HaloSegs send{}, recv{};
        uint64_t send_bytes = 0, recv_bytes = 0;
        uint32_t send_rank[RESTIR_MAX_HALO_SEGS] = {}, recv_rank[RESTIR_MAX_HALO_SEGS] = {};
        restir_halo_op ops[2 * RESTIR_MAX_HALO_SEGS] = {};   // what restir_halo_pass posts (restir_halo_ops)
        uint32_t nops = 0;
        uint32_t rank = 0, nranks = 0;   // this frame's tile (rank) of tiles_x * tiles_y
        int cur = 0;
        bool fb_records = true;
        bool rp_ok = false;          // the current grid's target-pdf cache is valid (restir_render's rp_ok)
        bool interior_done = false;  // the current pass's interior launch is issued (restir_halo_spatial_interior)
        bool part_rp = false;        // every launch of the current pass wrote the pdf cache
        uint8_t* tmiss = nullptr;    // the view's background-tile flags (fused RIS over the view, no temporal reuse)
    } halo;
    DevBuf halo_scratch;
    // record-only restir_halo_pass (restir_halo_record): the steps it issues, no RCCL call
    bool halo_record = false;
    std::vector<restir_halo_event> halo_log;
    // native RCCL halo transport (restir_halo_attach_rccl / _comm, restir_halo_pass)
    struct {
        void* comm = nullptr;            // ncclComm_t
        bool owned = false;              // created by restir_halo_attach_rccl (destroyed with the context)
        hipStream_t stream = nullptr;    // communication stream
        hipEvent_t packed = nullptr, moved = nullptr;
        int nranks = 0, rank = -1;       // the communicator's size and this context's rank in it
        DevBuf send, recv;
    } rccl;

    // stage API region
    Region stage_rg{};
    bool stage_ok = false;

    // R-MIS / R-OMIS: neighbourhoods [1 + cap][pixels] and accumulators [rows][pixels] (RESTIR_BUF_MIS_*)
    DevBuf mis_nbr, mis_acc, mis_smp;
    uint32_t mis_cap = 0, mis_rows = 0, mis_smp_samples = 0;
    // file side outputs (restir_set_renders_dir): R-OMIS alpha visualisation words [3T][pixels]
    std::string renders_dir;
    DevBuf mis_vis;
    std::vector<uint32_t> mis_vis_host;

    // timing
    bool timing = false;
    std::vector<Pending> pending;
    std::vector<hipEvent_t> free_events;
    double ms[RESTIR_K_COUNT] = {0};
    uint64_t launches[RESTIR_K_COUNT] = {0};
    uint64_t timing_seq[RESTIR_K_COUNT] = {0};   // launches seen per kernel (timing.every sampling)
};

// ---------------------------------------------------------------------------------------------------------
// pure host helpers
extern "C" {

const char* restir_last_error(void) { return g_err.c_str(); }
int restir_abi_version(void) { return RESTIR_ABI_VERSION; }

void restir_features_default(restir_features* out) {
    if (!out) return;
    std::memset(out, 0, sizeof(*out));
    out->ray_trace_mode = RESTIR_MODE_RESTIR;
    out->initial_light_samples = 32;
    out->num_samples_in_reservoir = 2;
    out->num_neighbours_to_sample = 5;
    out->spatial_resample_radius = 10;
    out->spatial_resampling_passes = 2;
    out->temporal_clamp_m = 20;
    out->initial_samples_visibility_check = 0;
    out->unbiased_combination = 0;
    out->spatial_reuse = 1;
    out->spatial_reuse_visibility_check = 0;
    out->temporal_reuse = 1;
    out->enable_shading = 1;
    out->enable_texture_mapping = 1;
    out->enable_tone_mapping = 1;
    out->gamma = 1.0f;
    out->exposure = 1.5f;
    out->neighbour_same_geometry = 1;
    out->use_progressive_romis = 0;
    out->save_alphas_visualisation = 1;
    out->neighbour_max_depth_difference_fraction = 0.10f;
    out->neighbour_max_normal_angle_difference_radians = 0.436332f;
    out->max_iterations_mis = 5;
    out->neighbour_selection_strategy = RESTIR_NEIGHBOURS_SIMILAR;
    out->mis_weight_rmis = RESTIR_MIS_EQUAL;
    out->progressive_update_mod = 1;
}

uint32_t restir_rng_key(uint32_t seed, uint32_t frame, uint32_t stage, uint32_t pass) {
    return mix32(mix32(mix32(seed ^ 0x9E3779B9u) + frame) ^ (stage * 0x01000193u + pass * 0x27D4EB2Fu));
}

uint32_t restir_rng_draw(uint32_t key, uint32_t global_pixel, uint32_t slot) {
    return draw(pix_state(key, global_pixel), slot);
}

// Trackball (trackball.cpp:20-29, 75-78, 105-114) with glm::quat(euler) (type_quat.inl:208-217) and
// quat * vec3 (type_quat.inl:347-354); plain float arithmetic, no contraction.
void restir_camera_derive(const restir_camera* cam, restir_camera_frame* out) {
    if (!cam || !out) return;
    float hh = std::tan(cam->fovy / 2.0f);
    float hw = cam->aspect * hh;
    float hx = cam->rotation[0] * 0.5f, hy = cam->rotation[1] * 0.5f, hz = cam->rotation[2] * 0.5f;
    float cx = std::cos(hx), cy = std::cos(hy), cz = std::cos(hz);
    float sx = std::sin(hx), sy = std::sin(hy), sz = std::sin(hz);
    float q[4];
    q[3] = cx * cy * cz + sx * sy * sz;
    q[0] = sx * cy * cz - cx * sy * sz;
    q[1] = cx * sy * cz + sx * cy * sz;
    q[2] = cx * cy * sz - sx * sy * cz;
    // v = (0, 0, -distance): uv = cross(q.xyz, v), uuv = cross(q.xyz, uv), v + ((uv * w) + uuv) * 2
    const float v[3] = {0.0f, 0.0f, -cam->distance};
    float uv[3] = {q[1] * v[2] - v[1] * q[2], q[2] * v[0] - v[2] * q[0], q[0] * v[1] - v[0] * q[1]};
    float uuv[3] = {q[1] * uv[2] - uv[1] * q[2], q[2] * uv[0] - uv[2] * q[0], q[0] * uv[1] - uv[0] * q[1]};
    for (int a = 0; a < 3; a++) {
        float r = v[a] + ((uv[a] * q[3]) + uuv[a]) * 2.0f;
        out->origin[a] = cam->look_at[a] + r;
    }
    std::memcpy(out->quat, q, sizeof(q));
    out->half_w = hw;
    out->half_h = hh;
}

}  // extern "C"

namespace {
// a layout's cuts are well formed: every column and every row of a column at least one pixel, the ends at the image
restir_status layout_check(const restir_tile_layout* L) {
    if (!L) return fail(RESTIR_ERR_INVALID, "tile layout is NULL");
    const uint32_t tx = L->tiles_x, ty = L->tiles_y;
    if (L->global_width == 0 || L->global_height == 0 || tx == 0 || ty == 0 || tx > RESTIR_MAX_TILES_X ||
        ty > RESTIR_MAX_TILES_Y)
        return fail(RESTIR_ERR_INVALID, "tile layout: bad size (W=%u H=%u tiles=%ux%u, at most %ux%u)", L->global_width,
                    L->global_height, tx, ty, RESTIR_MAX_TILES_X, RESTIR_MAX_TILES_Y);
    if (L->x_cuts[0] != 0 || L->x_cuts[tx] != L->global_width)
        return fail(RESTIR_ERR_INVALID, "tile layout: x cuts must run from 0 to the width");
    for (uint32_t c = 0; c < tx; c++) {
        if (L->x_cuts[c + 1] <= L->x_cuts[c]) return fail(RESTIR_ERR_INVALID, "tile layout: x cuts not increasing at %u", c);
        if (L->y_cuts[c][0] != 0 || L->y_cuts[c][ty] != L->global_height)
            return fail(RESTIR_ERR_INVALID, "tile layout: column %u's y cuts must run from 0 to the height", c);
        for (uint32_t r = 0; r < ty; r++)
            if (L->y_cuts[c][r + 1] <= L->y_cuts[c][r])
                return fail(RESTIR_ERR_INVALID, "tile layout: column %u's y cuts not increasing at %u", c, r);
    }
    return RESTIR_OK;
}
// pixels of cost cell i along an axis of n pixels split into m cells: x belongs to cell floor(x m / n)
inline uint32_t cell_of(uint32_t x, uint32_t m, uint32_t n) { return (uint32_t)((uint64_t)x * m / n); }
inline uint32_t cell_begin(uint32_t i, uint32_t m, uint32_t n) { return (uint32_t)(((uint64_t)i * n + m - 1) / m); }
// pixels of [a, b) in cell i
inline uint32_t cell_overlap(uint32_t i, uint32_t m, uint32_t n, uint32_t a, uint32_t b) {
    const uint32_t c0 = std::max(cell_begin(i, m, n), a), c1 = std::min(cell_begin(i + 1, m, n), b);
    return c1 > c0 ? c1 - c0 : 0u;
}
// the cost the grid puts on the rectangle [xa, xb) x [ya, yb) (each cell's cost spread evenly over its pixels)
double rect_cost(const float* cost, uint32_t cw, uint32_t ch, uint32_t W, uint32_t H, uint32_t xa, uint32_t xb,
                 uint32_t ya, uint32_t yb) {
    double sum = 0.0;
    const uint32_t j0 = cell_of(ya, ch, H), j1 = cell_of(yb - 1, ch, H), i0 = cell_of(xa, cw, W), i1 = cell_of(xb - 1, cw, W);
    for (uint32_t j = j0; j <= j1; j++) {
        const double fy = (double)cell_overlap(j, ch, H, ya, yb) / (cell_begin(j + 1, ch, H) - cell_begin(j, ch, H));
        for (uint32_t i = i0; i <= i1; i++) {
            const double fx = (double)cell_overlap(i, cw, W, xa, xb) / (cell_begin(i + 1, cw, W) - cell_begin(i, cw, W));
            sum += (double)cost[(size_t)j * cw + i] * fx * fy;
        }
    }
    return sum;
}
// cuts c[1..parts-1] of [0, n) at the equal-share points of the per-pixel prefix cost P (P[x] = cost of [0, x)),
// rounded to multiples of `align`, every part at least `align` wide (the last takes the remainder)
void share_cuts(const std::vector<double>& P, uint32_t n, uint32_t parts, uint32_t align, uint32_t* c) {
    c[0] = 0;
    c[parts] = n;
    const double total = P[n];
    for (uint32_t k = 1; k < parts; k++) {
        const double target = total * k / parts;
        const uint32_t x = (uint32_t)(std::lower_bound(P.begin(), P.begin() + n + 1, target) - P.begin());
        uint64_t q = ((uint64_t)x + align / 2) / align * align;
        const uint64_t lo = (uint64_t)c[k - 1] + align, hi = (uint64_t)n - (uint64_t)(parts - k) * align;
        q = std::min(std::max(q, lo), hi);
        c[k] = (uint32_t)q;
    }
}
void layout_rect(const restir_tile_layout& L, uint32_t rank, uint32_t& x0, uint32_t& y0, uint32_t& w, uint32_t& h) {
    const uint32_t tx = rank % L.tiles_x, ty = rank / L.tiles_x;
    x0 = L.x_cuts[tx]; w = L.x_cuts[tx + 1] - x0;
    y0 = L.y_cuts[tx][ty]; h = L.y_cuts[tx][ty + 1] - y0;
}
}  // namespace

extern "C" {

restir_status restir_layout_even(uint32_t W, uint32_t H, uint32_t tiles_x, uint32_t tiles_y, restir_tile_layout* out) {
    if (!out || W == 0 || H == 0 || tiles_x == 0 || tiles_y == 0 || tiles_x > W || tiles_y > H ||
        tiles_x > RESTIR_MAX_TILES_X || tiles_y > RESTIR_MAX_TILES_Y)
        return fail(RESTIR_ERR_INVALID, "restir_tile_plan: bad arguments (W=%u H=%u tiles=%ux%u)", W, H, tiles_x, tiles_y);
    restir_tile_layout L{};
    L.global_width = W; L.global_height = H; L.tiles_x = tiles_x; L.tiles_y = tiles_y;
    // even split, remainder to the first tiles (deterministic, every pixel owned exactly once)
    auto start = [](uint32_t n, uint32_t parts, uint32_t i) { return i * (n / parts) + std::min(i, n % parts); };
    for (uint32_t c = 0; c <= tiles_x; c++) L.x_cuts[c] = start(W, tiles_x, c);
    for (uint32_t c = 0; c < tiles_x; c++)
        for (uint32_t r = 0; r <= tiles_y; r++) L.y_cuts[c][r] = start(H, tiles_y, r);
    *out = L;
    return RESTIR_OK;
}

restir_status restir_layout_balanced(uint32_t W, uint32_t H, uint32_t tiles_x, uint32_t tiles_y, const float* cost,
                                     uint32_t cw, uint32_t ch, uint32_t align_x, uint32_t align_y, restir_tile_layout* out,
                                     double* efficiency) {
    if (!out || !cost || cw == 0 || ch == 0 || cw > W || ch > H)
        return fail(RESTIR_ERR_INVALID, "restir_layout_balanced: bad cost grid (%ux%u over %ux%u)", cw, ch, W, H);
    restir_tile_layout L{};
    ST_TRY(restir_layout_even(W, H, tiles_x, tiles_y, &L));
    align_x = std::max(align_x, 1u);
    align_y = std::max(align_y, 1u);
    if ((uint64_t)tiles_x * align_x > W || (uint64_t)tiles_y * align_y > H)
        return fail(RESTIR_ERR_INVALID, "restir_layout_balanced: %ux%u tiles of at least %ux%u px do not fit %ux%u", tiles_x,
                    tiles_y, align_x, align_y, W, H);
    for (size_t i = 0; i < (size_t)cw * ch; i++)
        if (!(cost[i] >= 0.0f) || !std::isfinite(cost[i]))
            return fail(RESTIR_ERR_INVALID, "restir_layout_balanced: cost cell %zu is negative or not finite", i);
    // columns: the per-pixel-column cost (each cell's column total spread over its pixel columns), prefix-summed
    std::vector<double> colsum(cw, 0.0);
    for (uint32_t j = 0; j < ch; j++)
        for (uint32_t i = 0; i < cw; i++) colsum[i] += cost[(size_t)j * cw + i];
    std::vector<double> P(W + 1, 0.0);
    for (uint32_t x = 0; x < W; x++) {
        const uint32_t i = cell_of(x, cw, W);
        P[x + 1] = P[x] + colsum[i] / (cell_begin(i + 1, cw, W) - cell_begin(i, cw, W));
    }
    share_cuts(P, W, tiles_x, align_x, L.x_cuts);
    // each column: its own rows' cost, prefix-summed over pixel rows
    std::vector<double> Q(H + 1, 0.0), rowsum(ch);
    for (uint32_t c = 0; c < tiles_x; c++) {
        const uint32_t xa = L.x_cuts[c], xb = L.x_cuts[c + 1];
        for (uint32_t j = 0; j < ch; j++) {
            double s = 0.0;
            for (uint32_t i = cell_of(xa, cw, W); i <= cell_of(xb - 1, cw, W); i++)
                s += (double)cost[(size_t)j * cw + i] * cell_overlap(i, cw, W, xa, xb) /
                     (cell_begin(i + 1, cw, W) - cell_begin(i, cw, W));
            rowsum[j] = s;
        }
        for (uint32_t y = 0; y < H; y++) {
            const uint32_t j = cell_of(y, ch, H);
            Q[y + 1] = Q[y] + rowsum[j] / (cell_begin(j + 1, ch, H) - cell_begin(j, ch, H));
        }
        share_cuts(Q, H, tiles_y, align_y, L.y_cuts[c]);
    }
    ST_TRY(layout_check(&L));
    if (efficiency) {
        std::vector<double> sh(tiles_x * tiles_y);
        ST_TRY(restir_layout_shares(&L, cost, cw, ch, sh.data()));
        double mx = 0.0, mean = 0.0;
        for (double v : sh) { mx = std::max(mx, v); mean += v / sh.size(); }
        *efficiency = mx > 0.0 ? mean / mx : 1.0;
    }
    *out = L;
    return RESTIR_OK;
}

restir_status restir_layout_shares(const restir_tile_layout* L, const float* cost, uint32_t cw, uint32_t ch, double* out) {
    ST_TRY(layout_check(L));
    if (!cost || !out || cw == 0 || ch == 0 || cw > L->global_width || ch > L->global_height)
        return fail(RESTIR_ERR_INVALID, "restir_layout_shares: bad cost grid");
    const uint32_t n = L->tiles_x * L->tiles_y;
    double total = 0.0;
    for (uint32_t q = 0; q < n; q++) {
        uint32_t x0, y0, w, h;
        layout_rect(*L, q, x0, y0, w, h);
        out[q] = rect_cost(cost, cw, ch, L->global_width, L->global_height, x0, x0 + w, y0, y0 + h);
        total += out[q];
    }
    for (uint32_t q = 0; q < n; q++) out[q] = total > 0.0 ? out[q] / total : 1.0 / n;
    return RESTIR_OK;
}

restir_status restir_layout_tile(const restir_tile_layout* L, uint32_t rank, uint32_t ghost, restir_tile* out) {
    ST_TRY(layout_check(L));
    if (!out || rank >= L->tiles_x * L->tiles_y)
        return fail(RESTIR_ERR_INVALID, "restir_tile_plan: bad arguments (rank %u of %ux%u tiles)", rank, L->tiles_x,
                    L->tiles_y);
    const uint32_t W = L->global_width, H = L->global_height;
    restir_tile t{};
    t.global_width = W;
    t.global_height = H;
    layout_rect(*L, rank, t.x0, t.y0, t.width, t.height);
    const uint32_t gx0 = t.x0 > ghost ? t.x0 - ghost : 0u;
    const uint32_t gy0 = t.y0 > ghost ? t.y0 - ghost : 0u;
    const uint32_t gx1 = std::min<uint64_t>((uint64_t)t.x0 + t.width + ghost, W);
    const uint32_t gy1 = std::min<uint64_t>((uint64_t)t.y0 + t.height + ghost, H);
    t.gx0 = gx0; t.gy0 = gy0; t.gwidth = gx1 - gx0; t.gheight = gy1 - gy0;
    *out = t;
    return RESTIR_OK;
}

restir_status restir_tile_plan(uint32_t W, uint32_t H, uint32_t tiles_x, uint32_t tiles_y, uint32_t rank, uint32_t ghost,
                               restir_tile* out) {
    restir_tile_layout L;
    if (!out || rank >= tiles_x * tiles_y)
        return fail(RESTIR_ERR_INVALID, "restir_tile_plan: bad arguments (W=%u H=%u tiles=%ux%u rank=%u)", W, H, tiles_x,
                    tiles_y, rank);
    ST_TRY(restir_layout_even(W, H, tiles_x, tiles_y, &L));
    return restir_layout_tile(&L, rank, ghost, out);
}

restir_status restir_layout_halo_plan(const restir_tile_layout* L, uint32_t rank, uint32_t radius, uint32_t N,
                                      restir_halo_segment* send, restir_halo_segment* recv, uint32_t* count) {
    if (!count || !send || !recv || N == 0) return fail(RESTIR_ERR_INVALID, "restir_halo_plan: null argument / N = 0");
    const uint32_t W = L ? L->global_width : 0u, H = L ? L->global_height : 0u;
    restir_tile me{};
    ST_TRY(restir_layout_tile(L, rank, 0, &me));
    struct R { uint64_t x0, y0, x1, y1; };
    auto grow = [&](const restir_tile& t) {
        return R{t.x0 > radius ? t.x0 - radius : 0u, t.y0 > radius ? t.y0 - radius : 0u,
                 std::min<uint64_t>((uint64_t)t.x0 + t.width + radius, W), std::min<uint64_t>((uint64_t)t.y0 + t.height + radius, H)};
    };
    auto owned = [](const restir_tile& t) { return R{t.x0, t.y0, (uint64_t)t.x0 + t.width, (uint64_t)t.y0 + t.height}; };
    auto meet = [](R a, R b) {
        R r{std::max(a.x0, b.x0), std::max(a.y0, b.y0), std::min(a.x1, b.x1), std::min(a.y1, b.y1)};
        if (r.x1 <= r.x0 || r.y1 <= r.y0) r = R{0, 0, 0, 0};
        return r;
    };
    const uint32_t cap = *count;
    uint32_t n = 0;
    uint64_t so = 0, ro = 0;
    for (uint32_t q = 0; q < L->tiles_x * L->tiles_y; q++) {
        if (q == rank) continue;
        restir_tile tq{};
        ST_TRY(restir_layout_tile(L, q, 0, &tq));
        const R s_ = meet(owned(me), grow(tq)), r_ = meet(owned(tq), grow(me));
        if (s_.x1 == 0 || r_.x1 == 0) continue;
        if (n >= cap) return fail(RESTIR_ERR_INVALID, "restir_halo_plan: more than %u segments", cap);
        auto fill = [&](restir_halo_segment& g, R r, uint64_t& off) {
            g.rank = q;
            g.x0 = (uint32_t)r.x0; g.y0 = (uint32_t)r.y0;
            g.width = (uint32_t)(r.x1 - r.x0); g.height = (uint32_t)(r.y1 - r.y0);
            g.offset = off;
            g.bytes = (uint64_t)g.width * g.height * N * 32u;
            off += g.bytes;
        };
        fill(send[n], s_, so);
        fill(recv[n], r_, ro);
        n++;
    }
    *count = n;
    return RESTIR_OK;
}

restir_status restir_halo_plan(uint32_t W, uint32_t H, uint32_t tiles_x, uint32_t tiles_y, uint32_t rank, uint32_t radius,
                               uint32_t N, restir_halo_segment* send, restir_halo_segment* recv, uint32_t* count) {
    restir_tile_layout L;
    ST_TRY(restir_layout_even(W, H, tiles_x, tiles_y, &L));
    return restir_layout_halo_plan(&L, rank, radius, N, send, recv, count);
}

}  // extern "C"

namespace {
// The operations restir_halo_pass posts, from a plan: send i then recv i per segment (restir_halo_ops)
void halo_ops_from(const restir_halo_segment* send, const restir_halo_segment* recv, uint32_t n, restir_halo_op* ops) {
    auto op = [](uint32_t kind, const restir_halo_segment& g) {
        restir_halo_op o{};
        o.kind = kind; o.peer = g.rank; o.offset = g.offset; o.bytes = g.bytes;
        o.x0 = g.x0; o.y0 = g.y0; o.width = g.width; o.height = g.height;
        return o;
    };
    for (uint32_t i = 0; i < n; i++) {
        ops[2 * i] = op(RESTIR_HALO_OP_SEND, send[i]);
        ops[2 * i + 1] = op(RESTIR_HALO_OP_RECV, recv[i]);
    }
}
}  // namespace

extern "C" {

restir_status restir_halo_ops(uint32_t W, uint32_t H, uint32_t tiles_x, uint32_t tiles_y, uint32_t rank, uint32_t radius,
                              uint32_t N, restir_halo_op* ops, uint32_t* count) {
    restir_tile_layout L;
    ST_TRY(restir_layout_even(W, H, tiles_x, tiles_y, &L));
    return restir_layout_halo_ops(&L, rank, radius, N, ops, count);
}

restir_status restir_layout_halo_ops(const restir_tile_layout* L, uint32_t rank, uint32_t radius, uint32_t N,
                                     restir_halo_op* ops, uint32_t* count) {
    if (!count || !ops) return fail(RESTIR_ERR_INVALID, "restir_halo_ops: null argument");
    restir_halo_segment sg[RESTIR_MAX_HALO_SEGS], rg_[RESTIR_MAX_HALO_SEGS];
    uint32_t n = RESTIR_MAX_HALO_SEGS;
    ST_TRY(restir_layout_halo_plan(L, rank, radius, N, sg, rg_, &n));
    if (*count < 2 * n) {
        const uint32_t need = 2 * n;
        *count = need;
        return fail(RESTIR_ERR_INVALID, "restir_halo_ops: capacity for %u operations needed", need);
    }
    halo_ops_from(sg, rg_, n, ops);
    *count = 2 * n;
    return RESTIR_OK;
}

restir_status restir_device_count(int* out) {
    if (!out) return fail(RESTIR_ERR_INVALID, "restir_device_count: null");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) { *out = 0; return fail(RESTIR_ERR_NO_DEVICE, "hipGetDeviceCount: %s", hipGetErrorString(e)); }
    *out = n;
    return RESTIR_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------------------
// context helpers
namespace {

restir_status check_features(const restir_features* f) {
    if (!f) return fail(RESTIR_ERR_INVALID, "features is NULL");
    if (f->ray_trace_mode > RESTIR_MODE_ROMIS)
        return fail(RESTIR_ERR_INVALID, "Unsupported ray-tracing render mode %u requested from entry point", f->ray_trace_mode);
    if (f->ray_trace_mode != RESTIR_MODE_RESTIR) {
        if (f->neighbour_selection_strategy > RESTIR_NEIGHBOURS_EQUAL_SIMILAR_DISSIMILAR)
            return fail(RESTIR_ERR_INVALID, "neighbourSelectionStrategy %u", f->neighbour_selection_strategy);
        if (f->ray_trace_mode == RESTIR_MODE_RMIS && f->mis_weight_rmis > RESTIR_MIS_BALANCE)   // render.cpp:94
            return fail(RESTIR_ERR_INVALID, "Unhandled MIS weight type: %u", f->mis_weight_rmis);
        if (f->ray_trace_mode == RESTIR_MODE_ROMIS && f->num_neighbours_to_sample + 1u > RESTIR_ROMIS_MAX_TECHNIQUES)
            return fail(RESTIR_ERR_UNSUPPORTED, "R-OMIS with %u neighbours: at most %u techniques per pixel",
                        f->num_neighbours_to_sample, RESTIR_ROMIS_MAX_TECHNIQUES);
        if (f->ray_trace_mode == RESTIR_MODE_ROMIS && f->use_progressive_romis && f->progressive_update_mod == 0)
            return fail(RESTIR_ERR_INVALID, "progressiveUpdateMod 0 (iteration %% 0)");
    }
    if (f->num_samples_in_reservoir < 1 || f->num_samples_in_reservoir > RESTIR_MAX_N)
        return fail(RESTIR_ERR_INVALID, "numSamplesInReservoir %u outside 1..%u", f->num_samples_in_reservoir, RESTIR_MAX_N);
    if (f->spatial_resample_radius > 4096) return fail(RESTIR_ERR_INVALID, "spatialResampleRadius too large");
    if (f->num_neighbours_to_sample > 4096) return fail(RESTIR_ERR_INVALID, "numNeighboursToSample too large");
    if (f->gamma == 0.0f && f->enable_tone_mapping) { /* 1/gamma = inf, as in the reference */ }
    return RESTIR_OK;
}

FeaturesDev to_dev(const restir_features* f) {
    FeaturesDev d{};
    d.M = f->initial_light_samples;
    d.N = f->num_samples_in_reservoir;
    d.K = f->num_neighbours_to_sample;
    d.R = f->spatial_resample_radius;
    d.clamp_m = f->temporal_clamp_m;
    d.initial_vis = f->initial_samples_visibility_check;
    d.unbiased = f->unbiased_combination;
    d.spatial_vis = f->spatial_reuse_visibility_check;
    d.shading = f->enable_shading;
    d.tone_map = f->enable_tone_mapping;
    d.texture = f->enable_texture_mapping;
    d.gamma = f->gamma;
    d.exposure = f->exposure;
    d.mode = f->ray_trace_mode;
    d.strategy = f->neighbour_selection_strategy;
    d.same_geom = f->neighbour_same_geometry;
    d.depth_frac = f->neighbour_max_depth_difference_fraction;
    d.normal_rad = f->neighbour_max_normal_angle_difference_radians;
    d.mis_weight = f->mis_weight_rmis;
    d.progressive = f->use_progressive_romis;
    d.prog_mod = f->progressive_update_mod;
    d.iterations = f->max_iterations_mis;
    return d;
}

}  // namespace

// The scene as one launch over a view of npx pixels sees it: the G-buffer texCoord plane (allocated for textured
// scenes; k_primary writes it, every target pdf reads it) and whether diffuseAlbedo reads the textures.
static restir_status scene_for(restir_ctx* c, const FeaturesDev& f, size_t npx, SceneDev& out, DevBuf* uv = nullptr);

namespace {

// neighbourhood capacity of generateResampleIndicesGrid's output (neighbour_selection.cpp:45-105): k + 1, or the
// whole window for the strategies whose size arithmetic can take every member of a class
uint32_t mis_capacity(const restir_features* f, uint32_t W, uint32_t H) {
    const uint32_t k1 = f->num_neighbours_to_sample + 1u;
    if (f->neighbour_selection_strategy == RESTIR_NEIGHBOURS_RANDOM || f->neighbour_selection_strategy == RESTIR_NEIGHBOURS_SIMILAR)
        return k1;
    const uint64_t side = 2ull * f->spatial_resample_radius + 1ull;
    const uint64_t win = std::min<uint64_t>(side, W) * std::min<uint64_t>(side, H);
    return win > k1 ? (uint32_t)win : k1;
}
uint32_t mis_acc_rows(const restir_features* f) {
    const uint32_t T = f->num_neighbours_to_sample + 1u;
    return f->ray_trace_mode == RESTIR_MODE_ROMIS ? T * T + 6u * T + 3u : 3u;
}
constexpr uint64_t kMisSampleBudget = 4ull << 30;   // bytes of R-OMIS per-sample scratch
restir_status ensure_mis(restir_ctx* c, const restir_features* f, uint32_t W, uint32_t H) {
    if (f->ray_trace_mode == RESTIR_MODE_RESTIR) return fail(RESTIR_ERR_INVALID, "the MIS stages need rayTraceMode RMIS or ROMIS");
    const size_t npx = (size_t)W * H;
    c->mis_cap = mis_capacity(f, W, H);
    c->mis_rows = mis_acc_rows(f);
    ST_TRY(c->mis_nbr.ensure((size_t)(1u + c->mis_cap) * npx * 4));
    ST_TRY(c->mis_acc.ensure((size_t)c->mis_rows * npx * 4));
    c->mis_smp_samples = 0;
    if (f->ray_trace_mode == RESTIR_MODE_ROMIS) {
        // R-OMIS per-sample scratch (k_romis_samples -> k_romis_accum): T + 3 rows per sample, as many of the T x N
        // samples as fit kMisSampleBudget (or the mis.chunk knob) and keep one launch's items below 2^31
        const uint64_t T = f->num_neighbours_to_sample + 1ull, S = T * f->num_samples_in_reservoir;
        const uint64_t per = (T + 3ull) * npx * 4ull;
        uint64_t n = std::max<uint64_t>(1, std::min<uint64_t>(S, kMisSampleBudget / per));
        if (c->tuning.mis_chunk) n = std::min<uint64_t>(n, c->tuning.mis_chunk);
        n = std::min<uint64_t>(n, std::max<uint64_t>(1, ((1ull << 31) - 1ull) / std::max<uint64_t>(npx, 1)));
        c->mis_smp_samples = (uint32_t)n;
        ST_TRY(c->mis_smp.ensure((size_t)(n * per)));
    }
    return RESTIR_OK;
}
// renderROMIS reads neighborhood[0..k] (render.cpp:155-181): every pixel's window must hold k candidates
restir_status check_romis_window(const restir_features* f, uint32_t W, uint32_t H) {
    if (f->ray_trace_mode != RESTIR_MODE_ROMIS || f->neighbour_selection_strategy == RESTIR_NEIGHBOURS_RANDOM) return RESTIR_OK;
    const uint64_t corner = std::min<uint64_t>((uint64_t)f->spatial_resample_radius + 1u, W) *
                            std::min<uint64_t>((uint64_t)f->spatial_resample_radius + 1u, H);
    if (corner - 1u < f->num_neighbours_to_sample)
        return fail(RESTIR_ERR_INVALID, "R-OMIS: a %ux%u image with radius %u leaves fewer than k = %u candidates in a corner window "
                                        "(the reference indexes past the neighbourhood)", W, H, f->spatial_resample_radius,
                    f->num_neighbours_to_sample);
    return RESTIR_OK;
}

restir_status ensure_work(restir_ctx* c, uint32_t vw, uint32_t vh, uint32_t N, bool debug) {
    const size_t npx = (size_t)vw * vh;
    ST_TRY(c->n_t.ensure(npx * 16));
    ST_TRY(c->p_mat.ensure(npx * 16));
    for (int i = 0; i < 2; i++) {
        ST_TRY(c->ra[i].ensure(npx * N * 16));
        ST_TRY(c->rb[i].ensure(npx * N * 16));
        if (debug) ST_TRY(c->dbg[i].ensure(npx * N * 8));
    }
    c->vw = vw; c->vh = vh; c->N = N;
    return RESTIR_OK;
}

// A timing event: read only by hipEventElapsedTime after hipStreamSynchronize (collect_timings), so it needs no
// system-scope release of its own -- with one, the timed kernel's completion waits for a cache writeback that
// showed as 6.7 us before and 4.6 us after the C2 spatial pass (profiles/r4/gap).
hipError_t timing_event_create(const restir_ctx* c, hipEvent_t* e) {
    return c->tuning.timing_fence ? hipEventCreate(e) : hipEventCreateWithFlags(e, hipEventDisableSystemFence);
}

restir_status timed_begin(restir_ctx* c, int kernel, Pending& p) {
    p.kernel = kernel;
    p.start = p.stop = nullptr;
    set_launch_events(nullptr, nullptr);
    if (!c->timing || !((c->tuning.timing_mask >> kernel) & 1u)) return RESTIR_OK;
    if (c->tuning.timing_every > 1u && (c->timing_seq[kernel]++ % c->tuning.timing_every) != 0u) return RESTIR_OK;
    for (hipEvent_t* e : {&p.start, &p.stop}) {
        if (!c->free_events.empty()) { *e = c->free_events.back(); c->free_events.pop_back(); }
        else HIP_TRY(timing_event_create(c, e));
    }
    set_launch_events(p.start, p.stop);   // recorded by the launch itself (hipExtLaunchKernelGGL)
    return RESTIR_OK;
}

restir_status timed_end(restir_ctx* c, Pending& p, hipError_t launch_err) {
    const bool used = launch_events_used();
    set_launch_events(nullptr, nullptr);
    if (launch_err != hipSuccess) return fail(RESTIR_ERR_HIP, "kernel launch: %s", hipGetErrorString(launch_err));
    if (!p.start) return RESTIR_OK;
    if (!used) {   // nothing launched (empty region): the events were never recorded
        c->free_events.push_back(p.start);
        c->free_events.push_back(p.stop);
        return RESTIR_OK;
    }
    c->pending.push_back(p);
    return RESTIR_OK;
}

restir_status collect_timings(restir_ctx* c) {
    if (c->pending.empty()) return RESTIR_OK;
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (Pending& p : c->pending) {
        float ms = 0.0f;
        HIP_TRY(hipEventElapsedTime(&ms, p.start, p.stop));
        c->ms[p.kernel] += ms;
        c->launches[p.kernel] += 1;
        c->free_events.push_back(p.start);
        c->free_events.push_back(p.stop);
    }
    c->pending.clear();
    return RESTIR_OK;
}

#define TIMED(ctx, kid, call)                                   \
    do {                                                        \
        Pending p_;                                             \
        ST_TRY(timed_begin((ctx), (kid), p_));                  \
        ST_TRY(timed_end((ctx), p_, (call)));                   \
    } while (0)

CameraDev camera_dev(const restir_camera* cam) {
    restir_camera_frame cf;
    restir_camera_derive(cam, &cf);
    CameraDev d{};
    d.quat = make_float4(cf.quat[0], cf.quat[1], cf.quat[2], cf.quat[3]);
    for (int a = 0; a < 3; a++) d.origin[a] = cf.origin[a];
    d.half_w = cf.half_w;
    d.half_h = cf.half_h;
    return d;
}

Region make_region(uint32_t W, uint32_t H, uint32_t vx0, uint32_t vy0, uint32_t vw, uint32_t vh, uint32_t rx0,
                   uint32_t ry0, uint32_t rw, uint32_t rh) {
    Region r{};
    r.W = W; r.H = H;
    r.vx0 = vx0; r.vy0 = vy0; r.vw = vw; r.vh = vh;
    r.rx0 = rx0; r.ry0 = ry0; r.rw = rw; r.rh = rh;
    r.ps = 1; r.js = vw * vh;   // SoA planes (the stage API's buffers)
    return r;
}

// The frame path keeps one record per pixel, [n_t, res_a_0, res_b_0, res_a_1, ...]: a neighbour's depth /
// normal test and its reservoir come from the same cache lines (the spatial pass's gathers touch one record
// instead of three planes).
Region with_records(Region r, uint32_t N) {
    r.ps = 1u + 2u * N;
    r.js = 2u;
    return r;
}

// Frame-path buffers in either layout (tuning "layout.records"): records = rec[i] holds [n_t, a_j, b_j] per
// pixel; planes = rec[i] holds N res_a planes then N res_b planes, n_t is the separate plane n_t.
struct FrameBufs {
    restir_ctx* c;
    bool records;
    size_t npx;
    uint32_t N;
    DevBuf* rec_() const { return c->rec; }
    DevBuf& n_t_() const { return c->n_t; }
    DevBuf* rp_() const { return c->rp; }
    float4* pm() const { return c->p_mat.as<float4>(); }
    DevBuf& rgb() const { return c->rgb; }
    DevBuf& uv() const { return c->uv; }
    DevBuf& vis() const { return c->vis; }
    DevBuf& tmiss() const { return c->tmiss; }
    DevBuf* hnd_() const { return c->hnd; }
    // the sample-handle planes of rec[i]: W then M | index << 24, one 4-byte plane each (ensure_handles)
    Handles h(int i) const {
        float* w = hnd_()[i].as<float>();
        return w ? Handles{w, reinterpret_cast<uint32_t*>(w + npx), 0u} : Handles{nullptr, nullptr, 0u};
    }
    // frame handles: the same planes at the tail of rec[i] (planes layout, ensure_records), handed on with the records to
    // the frame restir_render returns -- the next frame's fused temporal reuse reads them: N = 1 the W and M | index
    // planes (8 B / px, not 32), N = 2 the 16-byte handle records (not 64 B)
    Handles fh(int i) const {
        if (records || (N != 1 && N != 2)) return Handles{nullptr, nullptr, 0u};
        float* w = reinterpret_cast<float*>(rec_()[i].as<float4>() + 2 * N * npx);
        return Handles{w, N == 1 ? reinterpret_cast<uint32_t*>(w + npx) : nullptr, 0u};
    }
    const float* fhw(const restir_frame* f) const { return reinterpret_cast<const float*>(f->rec.as<float4>() + 2 * N * npx); }
    const uint32_t* fhm(const restir_frame* f) const {
        return N == 1 ? reinterpret_cast<const uint32_t*>(fhw(f) + npx) : nullptr;
    }
    float4* nt(int i) const { return records ? rec_()[i].as<float4>() : n_t_().as<float4>(); }
    float4* ra(int i) const { return rec_()[i].as<float4>() + (records ? 1 : 0); }
    float4* rb(int i) const { return rec_()[i].as<float4>() + (records ? 2 : npx * N); }
    float4* nt2() const { return records ? rec_()[1].as<float4>() : nullptr; }
    // the target-pdf cache planes (N = 1 planes layout only)
    float* rp(int i) const { return (!records && N == 1) ? rp_()[i].as<float>() : nullptr; }
    const float4* pa(const restir_frame* f) const { return f->rec.as<float4>() + (records ? 1 : 0); }
    const float4* pb(const restir_frame* f) const { return f->rec.as<float4>() + (records ? 2 : npx * N); }
    Region region(Region r) const { return records ? with_records(r, N) : r; }
};

restir_status ensure_records(restir_ctx* c, uint32_t vw, uint32_t vh, uint32_t N, FrameBufs& fb) {
    const size_t npx = (size_t)vw * vh;
    fb = FrameBufs{c, c->tuning.records != 0, npx, N};
    const hipStream_t st = c->stream;
    ST_TRY(c->p_mat.ensure(npx * 16));
    if (!fb.records) ST_TRY(fb.n_t_().ensure(npx * 16));
    // (planes, N = 1: + the frame handles' two 4-byte planes and 16 B of slack; N = 2: + the 16-byte handle records and
    // 16 B; FrameBufs::fh)
    const size_t rec_bytes = npx * (fb.records ? 1u + 2u * N : 2u * N) * 16 +
                             (fb.records ? 0 : N == 1 ? npx * 8 + 16 : N == 2 ? npx * 16 + 16 : 0);
    DevBuf* rec = fb.rec_();
    for (int i = 0; i < 2; i++) {
        // a buffer handed to a frame comes back through the pool (stream-ordered against its past users)
        if (!rec[i].p && c->pool->take(rec_bytes, st, rec[i])) continue;
        ST_TRY(rec[i].ensure(rec_bytes));
    }
    if (!fb.records && N == 1)
        for (int i = 0; i < 2; i++) ST_TRY(fb.rp_()[i].ensure(npx * 4));
    c->vw = vw; c->vh = vh; c->N = N;
    return RESTIR_OK;
}

// rect grown by g, clipped to the view
Region grow_rect(const Region& base, uint32_t g) {
    Region r = base;
    uint32_t x0 = base.rx0 > base.vx0 + g ? base.rx0 - g : base.vx0;
    uint32_t y0 = base.ry0 > base.vy0 + g ? base.ry0 - g : base.vy0;
    uint64_t x1 = std::min<uint64_t>((uint64_t)base.rx0 + base.rw + g, (uint64_t)base.vx0 + base.vw);
    uint64_t y1 = std::min<uint64_t>((uint64_t)base.ry0 + base.rh + g, (uint64_t)base.vy0 + base.vh);
    r.rx0 = x0; r.ry0 = y0; r.rw = (uint32_t)(x1 - x0); r.rh = (uint32_t)(y1 - y0);
    return r;
}

}  // namespace

// ---------------------------------------------------------------------------------------------------------
static restir_status scene_for(restir_ctx* c, const FeaturesDev& f, size_t npx, SceneDev& out, DevBuf* uv) {
    out = c->sdev;
    if (c->sdev.num_textures) {
        DevBuf& u = uv ? *uv : c->uv;
        ST_TRY(u.ensure(std::max<size_t>(npx, 1) * 8));
        out.gbuf_uv = u.as<float2>();
        out.tex_on = f.texture ? 1u : 0u;
    }
    return RESTIR_OK;
}

extern "C" {

restir_status restir_create(int device, restir_ctx** out) {
    if (!out) return fail(RESTIR_ERR_INVALID, "restir_create: out is NULL");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) return fail(RESTIR_ERR_NO_DEVICE, "no HIP device (%s)", hipGetErrorString(e));
    if (device < 0) device = 0;
    if (device >= n) return fail(RESTIR_ERR_NO_DEVICE, "device %d >= device count %d", device, n);
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(RESTIR_ERR_NO_DEVICE, "device %d is %s; libromis_amd is built for gfx950 only", device, prop.gcnArchName);
    HIP_TRY(hipSetDevice(device));
    restir_ctx* c = new restir_ctx();
    c->device = device;
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) { delete c; return fail(RESTIR_ERR_HIP, "hipStreamCreate: %s", hipGetErrorString(e)); }
    c->pool->owner = c->stream;
    *out = c;
    return RESTIR_OK;
}

static void release_rccl(restir_ctx* c);   // (halo section)

void restir_destroy(restir_ctx* c) {
    if (!c) return;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
        for (DevBuf* b : {&c->vis, &c->tmiss, &c->hnd[0], &c->hnd[1]}) b->release();
        for (DevBuf* b : {&c->nodes, &c->nodes_q, &c->tri_v0, &c->tri_e1, &c->tri_e2, &c->tri_n0, &c->tri_n1, &c->tri_n2,
                          &c->materials, &c->lights, &c->light_c2, &c->light_c4, &c->light_col, &c->tex_texels, &c->tex_dims, &c->tri_uv, &c->uv, &c->n_t, &c->p_mat, &c->ra[0], &c->ra[1], &c->rb[0], &c->rb[1],
                          &c->dbg[0], &c->dbg[1], &c->rgb, &c->halo_scratch, &c->rec[0], &c->rec[1], &c->rp[0], &c->rp[1]})
            b->release();
        for (Pending& p : c->pending) { (void)hipEventDestroy(p.start); (void)hipEventDestroy(p.stop); }
        for (hipEvent_t ev : c->free_events) (void)hipEventDestroy(ev);
        c->pool->close();   // frames still alive free their records themselves on release
        release_rccl(c);
        (void)hipStreamDestroy(c->stream);
    }
    delete c;
}

restir_status restir_set_seed(restir_ctx* c, uint32_t seed, uint32_t frame_index) {
    if (!c) return fail(RESTIR_ERR_INVALID, "ctx is NULL");
    std::lock_guard<std::mutex> lk(c->mu);
    c->seed = seed;
    c->frame_index = frame_index;
    return RESTIR_OK;
}

restir_status restir_set_renders_dir(restir_ctx* c, const char* dir) {
    if (!c) return fail(RESTIR_ERR_INVALID, "ctx is NULL");
    std::lock_guard<std::mutex> lk(c->mu);
    c->renders_dir = dir ? dir : "";
    return RESTIR_OK;
}

restir_status restir_set_scene(restir_ctx* c, const restir_mesh* meshes, uint32_t num_meshes, const restir_light* lights,
                               uint32_t num_lights) {
    return restir_set_scene_textured(c, meshes, num_meshes, lights, num_lights, nullptr, 0);
}

// regularLightGrid's layout (scene.cpp:5-28) recovered from a light grid's corners: light i = x * ny + y has its corner
// at (start + s01 * float(x)) + s02 * float(y), computed in float as the reference does.  start = light 0's corner;
// s01 / s02 per component from the corners of lights ny and 1 (their difference, then the nearest floats around it)
// and accepted only when they reproduce every light's corner bit for bit; ny = the first power-of-two divisor of
// the light count that works.  The RIS kernels' kLtRegular form then evaluates the same expression instead of
// reading the corner from the table.
struct RegularGrid {
    bool ok = false;
    uint32_t ny_log2 = 0;
    float start[3] = {0, 0, 0}, s01[3] = {0, 0, 0}, s02[3] = {0, 0, 0};
};
static float grid_corner(float start, float s01, float s02, uint32_t x, uint32_t y) {
    volatile float a = s01 * (float)x;   // float products and sums, no contraction (the reference's order)
    volatile float b = start + a;
    volatile float c = s02 * (float)y;
    return b + c;
}
static RegularGrid find_regular_grid(const std::vector<float>& lt, uint32_t L) {
    RegularGrid g;
    if (L < 2) return g;
    auto near_floats = [](float t, float* out) {   // t and its 64 float neighbours on either side
        int n = 0;
        out[n++] = t;
        float up = t, dn = t;
        for (int k = 0; k < 64; k++) {
            up = std::nextafter(up, INFINITY);
            dn = std::nextafter(dn, -INFINITY);
            out[n++] = up;
            out[n++] = dn;
        }
        return n;
    };
    for (uint32_t lg = 0; (1u << lg) <= L; lg++) {
        const uint32_t ny = 1u << lg, nx = L / ny;
        if (nx * ny != L) break;
        if (ny < 2) continue;
        bool all = true;
        float st[3], a01[3], a02[3];
        for (int cpt = 0; cpt < 3 && all; cpt++) {
            const float start = lt[cpt];
            float c01[129], c02[129];
            const int n01 = nx > 1 ? near_floats(lt[28 * ny + cpt] - start, c01) : (c01[0] = 0.0f, 1);
            const int n02 = near_floats(lt[28 * 1 + cpt] - start, c02);
            bool found = false;
            for (int i01 = 0; i01 < n01 && !found; i01++)
                for (int i02 = 0; i02 < n02 && !found; i02++) {
                    bool match = true;
                    for (uint32_t i = 0; i < L && match; i++) {
                        const float v = grid_corner(start, c01[i01], c02[i02], i >> lg, i & (ny - 1u));
                        match = std::memcmp(&v, &lt[28 * i + cpt], 4) == 0;
                    }
                    if (match) { found = true; st[cpt] = start; a01[cpt] = c01[i01]; a02[cpt] = c02[i02]; }
                }
            all = found;
        }
        if (all) {
            g.ok = true;
            g.ny_log2 = lg;
            for (int cpt = 0; cpt < 3; cpt++) {
                g.start[cpt] = st[cpt]; g.s01[cpt] = a01[cpt]; g.s02[cpt] = a02[cpt];
            }
            return g;
        }
    }
    return g;
}

restir_status restir_set_scene_textured(restir_ctx* c, const restir_mesh* meshes, uint32_t num_meshes,
                                        const restir_light* lights, uint32_t num_lights, const restir_texture* textures,
                                        uint32_t num_textures) {
    if (!c) return fail(RESTIR_ERR_INVALID, "ctx is NULL");
    if (num_meshes && !meshes) return fail(RESTIR_ERR_INVALID, "meshes is NULL");
    if (num_lights && !lights) return fail(RESTIR_ERR_INVALID, "lights is NULL");
    if (num_textures && !textures) return fail(RESTIR_ERR_INVALID, "textures is NULL");
    for (uint32_t i = 0; i < num_textures; i++)
        if (!textures[i].width || !textures[i].height || !textures[i].rgb)
            return fail(RESTIR_ERR_INVALID, "texture %u: empty image", i);
    for (uint32_t m = 0; m < num_meshes; m++)
        if (meshes[m].material.kd_texture > num_textures)
            return fail(RESTIR_ERR_INVALID, "mesh %u: kd_texture %u of %u textures", m, meshes[m].material.kd_texture,
                        num_textures);
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));

    // flatten triangles (mesh order = original index order, like the oracle)
    std::vector<BvhTriangle> tris;
    std::vector<float> n0, n1, n2;   // float4 records
    std::vector<float> tuv;          // 2 float4 per triangle: (t0.xy, t1.xy), (t2.xy, 0, 0)
    for (uint32_t m = 0; m < num_meshes; m++) {
        const restir_mesh& mesh = meshes[m];
        if (mesh.num_triangles && (!mesh.positions || !mesh.normals || !mesh.triangles))
            return fail(RESTIR_ERR_INVALID, "mesh %u: null arrays", m);
        for (uint32_t i = 0; i < mesh.num_triangles; i++) {
            const uint32_t* t = &mesh.triangles[3 * i];
            if (t[0] >= mesh.num_vertices || t[1] >= mesh.num_vertices || t[2] >= mesh.num_vertices)
                return fail(RESTIR_ERR_INVALID, "mesh %u triangle %u: vertex index out of range", m, i);
            BvhTriangle bt;
            std::memcpy(bt.v0, &mesh.positions[3 * t[0]], 12);
            std::memcpy(bt.v1, &mesh.positions[3 * t[1]], 12);
            std::memcpy(bt.v2, &mesh.positions[3 * t[2]], 12);
            tris.push_back(bt);
            for (int k = 0; k < 3; k++) {
                std::vector<float>& dst = k == 0 ? n0 : (k == 1 ? n1 : n2);
                dst.insert(dst.end(), &mesh.normals[3 * t[k]], &mesh.normals[3 * t[k]] + 3);
                dst.push_back(k == 0 ? u2f(m) : 0.0f);
            }
            for (int k = 0; k < 3; k++) {
                tuv.push_back(mesh.texcoords ? mesh.texcoords[2 * t[k]] : 0.0f);
                tuv.push_back(mesh.texcoords ? mesh.texcoords[2 * t[k] + 1] : 0.0f);
            }
            tuv.push_back(0.0f);
            tuv.push_back(0.0f);
        }
    }
    if (tris.size() >= (1u << 24)) return fail(RESTIR_ERR_INVALID, "too many triangles (%zu)", tris.size());
    FlatBvh bvh = build_bvh(tris, c->tuning.bvh_max_leaf);
    const size_t T = tris.size();
    std::vector<float> v0(4 * std::max<size_t>(T, 1)), e1(v0.size()), e2(v0.size());
    for (size_t k = 0; k < T; k++) {
        const BvhTriangle& t = tris[bvh.tri_order[k]];
        for (int a = 0; a < 3; a++) {
            v0[4 * k + a] = t.v0[a];
            e1[4 * k + a] = t.v1[a] - t.v0[a];
            e2[4 * k + a] = t.v2[a] - t.v0[a];
        }
        v0[4 * k + 3] = u2f(bvh.tri_order[k]);
    }
    // materials: one per mesh + the miss material (value-initialised HitInfo: kd 0, ks 0, shininess 1)
    // 3 float4 per material: (kd, shininess), (ks, pow mode), (underflow threshold, exponent, transparency, 0)
    std::vector<float> mats(12 * (num_meshes + 1), 0.0f);
    auto put_material = [&](uint32_t m, const restir_material& mt) {
        float* o = &mats[12 * m];
        o[0] = mt.kd[0]; o[1] = mt.kd[1]; o[2] = mt.kd[2]; o[3] = mt.shininess;
        o[4] = mt.ks[0]; o[5] = mt.ks[1]; o[6] = mt.ks[2];
        uint32_t mode = ROMIS_POW_GLIBC;
        float thr = 0.0f;
        const double y = (double)mt.shininess;
        if (mt.ks[0] == 0.0f && mt.ks[1] == 0.0f && mt.ks[2] == 0.0f) {
            mode = ROMIS_POW_SKIP;
        } else if (std::isfinite(y) && y > 0.0) {
            // |x| < thr  =>  y * log2|x| < -150 (1 + 2^-20): glibc's powf takes its underflow exit
            // (ylogx <= -150, returns +-0, the sign for a negative base and an odd integer y); the margin
            // dwarfs the 2^-32 relative error of its log2 and the rounding of y * log2|x|
            thr = (float)std::exp2(-150.0 * (1.0 + 0x1p-20) / y);
            if ((double)thr > std::exp2(-150.0 * (1.0 + 0x1p-20) / y)) thr = std::nextafter(thr, 0.0f);
        }
        const uint32_t cls = pw_class(mt.shininess);
        if (mode == ROMIS_POW_GLIBC && !(cls & (ROMIS_PWC_SPECIAL | ROMIS_PWC_NEG)) && thr >= FLT_MIN) mode = ROMIS_POW_SIMPLE;
        o[7] = u2f(mode);
        o[8] = thr; o[9] = u2f(cls); o[10] = mt.transparency; o[11] = u2f(mt.kd_texture);
    };
    for (uint32_t m = 0; m < num_meshes; m++) put_material(m, meshes[m].material);
    {
        restir_material miss{};   // value-initialised HitInfo material: kd 0, ks 0, shininess 1, transparency 1
        miss.shininess = 1.0f;
        miss.transparency = 1.0f;
        put_material(num_meshes, miss);
    }
    // lights: 7 float4 records
    std::vector<float> lt(28 * std::max<uint32_t>(num_lights, 1), 0.0f);
    uint32_t types = 0;
    for (uint32_t i = 0; i < num_lights; i++) {
        const restir_light& l = lights[i];
        if (l.type > RESTIR_LIGHT_PARALLELOGRAM) return fail(RESTIR_ERR_INVALID, "light %u: bad type %u", i, l.type);
        types |= 1u << l.type;
        float* o = &lt[28 * i];
        const float* src[7] = {l.p0, l.p1, l.p2, l.c0, l.c1, l.c2, l.c3};
        for (int r = 0; r < 7; r++) { std::memcpy(&o[4 * r], src[r], 12); o[4 * r + 3] = 0.0f; }
        o[3] = u2f(l.type);
    }
    if (n0.empty()) { n0.assign(4, 0.0f); n1.assign(4, 0.0f); n2.assign(4, 0.0f); }
    std::vector<float> nodes = bvh.nodes;
    if (nodes.empty()) nodes.assign(8, 0.0f);
    // The shadow rays' 16-byte nodes (SceneDev::nodes_q, kernels_common.h occluded_q): each padded box snapped outward to
    // a 16-bit grid over the root box, so the quantized box contains the float one -- a test against it accepts every
    // box the float test accepts (and a few more), and any-hit decides by the exact triangle tests alone, in any order.
    std::vector<uint32_t> nq;
    float q_lo[3] = {0.0f, 0.0f, 0.0f}, q_s[3] = {1.0f, 1.0f, 1.0f};
    bool q_ok = bvh.num_nodes > 0 && bvh.num_nodes < 65536u;
    for (uint32_t i = 0; q_ok && i < bvh.num_nodes; i++) {
        const uint32_t leaf = f2u(nodes[8 * i + 7]);
        q_ok = leaf == 0u || ((leaf >> 24) < 16u && (leaf & 0xFFFFFFu) + (leaf >> 24) <= 4096u);
    }
    if (q_ok) {
        for (int a = 0; a < 3; a++) {
            const double lo = nodes[a], hi = nodes[4 + a];   // the root's padded box
            q_lo[a] = (float)lo;
            if ((double)q_lo[a] > lo) q_lo[a] = std::nextafter(q_lo[a], -INFINITY);
            q_s[a] = (float)std::max((hi - (double)q_lo[a]) / 65532.0, 1e-30);
            q_ok = q_ok && std::isfinite(q_lo[a]) && std::isfinite(q_s[a]);
        }
    }
    if (q_ok) {
        nq.assign(4 * (size_t)bvh.num_nodes, 0u);
        for (uint32_t i = 0; i < bvh.num_nodes && q_ok; i++) {
            uint32_t q[6];
            for (int a = 0; a < 3; a++) {
                const double lo = nodes[8 * i + a], hi = nodes[8 * i + 4 + a];
                const double ql = std::floor((lo - (double)q_lo[a]) / (double)q_s[a]);
                const double qh = std::ceil((hi - (double)q_lo[a]) / (double)q_s[a]);
                q_ok = q_ok && ql >= -1.0 && qh <= 65535.0;
                q[a] = (uint32_t)std::max(ql, 0.0);
                q[3 + a] = (uint32_t)std::min(std::max(qh, 0.0), 65535.0);
            }
            const uint32_t miss = f2u(nodes[8 * i + 3]), leaf = f2u(nodes[8 * i + 7]);
            nq[4 * i + 0] = q[0] | (q[1] << 16);
            nq[4 * i + 1] = q[2] | (q[3] << 16);
            nq[4 * i + 2] = q[4] | (q[5] << 16);
            // miss link (16 bits: bvh.num_nodes < 65536), first triangle (12 bits), count (4 bits; 0 = inner node)
            nq[4 * i + 3] = std::min(miss, 65535u) | ((leaf & 0xFFFu) << 16) | ((leaf >> 24) << 28);
        }
    }
    if (!q_ok) nq.assign(4, 0u);

    HIP_TRY(hipStreamSynchronize(c->stream));   // previous frames (either slot) may still read the old scene
    ST_TRY(c->nodes.upload(nodes.data(), nodes.size() * 4, c->stream));
    ST_TRY(c->nodes_q.upload(nq.data(), nq.size() * 4, c->stream));
    ST_TRY(c->tri_v0.upload(v0.data(), v0.size() * 4, c->stream));
    ST_TRY(c->tri_e1.upload(e1.data(), e1.size() * 4, c->stream));
    ST_TRY(c->tri_e2.upload(e2.data(), e2.size() * 4, c->stream));
    ST_TRY(c->tri_n0.upload(n0.data(), n0.size() * 4, c->stream));
    ST_TRY(c->tri_n1.upload(n1.data(), n1.size() * 4, c->stream));
    ST_TRY(c->tri_n2.upload(n2.data(), n2.size() * 4, c->stream));
    ST_TRY(c->materials.upload(mats.data(), mats.size() * 4, c->stream));
    ST_TRY(c->lights.upload(lt.data(), lt.size() * 4, c->stream));
    // the compact light table of the RIS kernels' point and grid forms (kernels.hip kLtPoint / kLtGrid): rows 0 and 3
    // of every record.  A light grid (the reference's regularLightGrid, scene.cpp:5-28): every light a parallelogram
    // with light 0's edges and one colour at all four of its corners, bit for bit.
    // Parallelograms with one colour at all four corners (kLtPgram: rows 0..3 of every record) are the
    // reference's default nightclub set (scene.cpp:30-66); a grid also shares light 0's edges.
    bool pgram = num_lights > 0 && types == (1u << RESTIR_LIGHT_PARALLELOGRAM);
    for (uint32_t i = 0; pgram && i < num_lights; i++) {
        const float* o = &lt[28 * i];
        pgram = std::memcmp(o + 16, o + 12, 3 * sizeof(float)) == 0 && std::memcmp(o + 20, o + 12, 3 * sizeof(float)) == 0 &&
                std::memcmp(o + 24, o + 12, 3 * sizeof(float)) == 0;
    }
    bool grid = pgram;
    for (uint32_t i = 0; grid && i < num_lights; i++) grid = std::memcmp(&lt[28 * i + 4], &lt[4], 8 * sizeof(float)) == 0;
    const RegularGrid reg = grid ? find_regular_grid(lt, num_lights) : RegularGrid{};
    std::vector<float> lc4(16 * std::max<uint32_t>(pgram ? num_lights : 1u, 1u), 0.0f);
    for (uint32_t i = 0; pgram && i < num_lights; i++) std::memcpy(&lc4[16 * i], &lt[28 * i], 64);
    ST_TRY(c->light_c4.upload(lc4.data(), lc4.size() * 4, c->stream));
    // two planes (SceneDev::light_c2): rows 0 of every light, then rows 3 -- a random light's 16-byte read from an LDS
    // copy then lands on one of 16 bank groups instead of 8 (32-byte records)
    std::vector<float> lc2(8 * std::max<uint32_t>(num_lights, 1), 0.0f);
    for (uint32_t i = 0; i < num_lights; i++) {
        std::memcpy(&lc2[4 * i], &lt[28 * i], 16);
        std::memcpy(&lc2[4 * (num_lights + i)], &lt[28 * i + 12], 16);
    }
    ST_TRY(c->light_c2.upload(lc2.data(), lc2.size() * 4, c->stream));
    std::vector<float> lcol(4 * std::max<uint32_t>(num_lights, 1), 0.0f);   // c0 of every light (kLtRegular)
    for (uint32_t i = 0; i < num_lights; i++) std::memcpy(&lcol[4 * i], &lt[28 * i + 12], 12);
    ST_TRY(c->light_col.upload(lcol.data(), lcol.size() * 4, c->stream));
    // textures: texels as float4, images back to back; (width, height, first texel, 0) per image
    std::vector<float> texels;
    std::vector<uint32_t> dims;
    double tmax = 0.0;
    bool tfinite = true;
    for (uint32_t i = 0; i < num_textures; i++) {
        const restir_texture& tx = textures[i];
        dims.insert(dims.end(), {tx.width, tx.height, (uint32_t)(texels.size() / 4), 0u});
        for (size_t k = 0; k < (size_t)tx.width * tx.height; k++) {
            for (int a = 0; a < 3; a++) {
                const float v = tx.rgb[3 * k + a];
                texels.push_back(v);
                tfinite = tfinite && std::isfinite(v);
                tmax = std::max(tmax, (double)std::fabs(v));
            }
            texels.push_back(0.0f);
        }
    }
    if (texels.size() / 4 >= 0xFFFFFFFFull) return fail(RESTIR_ERR_INVALID, "textures too large");
    if (texels.empty()) texels.assign(4, 0.0f);
    if (dims.empty()) dims.assign(4, 0u);
    if (tuv.empty()) tuv.assign(8, 0.0f);
    ST_TRY(c->tex_texels.upload(texels.data(), texels.size() * 4, c->stream));
    ST_TRY(c->tex_dims.upload(dims.data(), dims.size() * 4, c->stream));
    ST_TRY(c->tri_uv.upload(tuv.data(), tuv.size() * 4, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));   // host vectors go out of scope

    SceneDev& s = c->sdev;
    s.nodes = c->nodes.as<float4>();
    s.num_nodes = bvh.num_nodes;
    s.nodes_q = c->nodes_q.as<uint4>();
    s.nodes_q_ok = q_ok ? 1u : 0u;
    s.q_lo = make_float4(q_lo[0], q_lo[1], q_lo[2], 0.0f);
    s.q_s = make_float4(q_s[0], q_s[1], q_s[2], 0.0f);
    s.tri_v0 = c->tri_v0.as<float4>();
    s.tri_e1 = c->tri_e1.as<float4>();
    s.tri_e2 = c->tri_e2.as<float4>();
    s.tri_n0 = c->tri_n0.as<float4>();
    s.tri_n1 = c->tri_n1.as<float4>();
    s.tri_n2 = c->tri_n2.as<float4>();
    s.num_tris = (uint32_t)T;
    s.materials = c->materials.as<float4>();
    s.num_materials = num_meshes + 1;
    s.tex_texels = c->tex_texels.as<float4>();
    s.tex_dims = c->tex_dims.as<uint4>();
    s.tri_uv = c->tri_uv.as<float4>();
    s.num_textures = num_textures;
    s.gbuf_uv = nullptr;   // per launch (scene_for)
    s.tex_on = 0u;
    s.lights = c->lights.as<float4>();
    s.num_lights = num_lights;
    s.light_types = types;
    s.light_c2 = c->light_c2.as<float4>();
    s.lights_grid = grid ? 1u : 0u;
    s.light_c4 = c->light_c4.as<float4>();
    s.lights_pgram = pgram ? 1u : 0u;
    s.lights_regular = reg.ok ? 1u : 0u;
    s.grid_ny_log2 = reg.ny_log2;
    s.grid_start = make_float4(reg.start[0], reg.start[1], reg.start[2], 0.0f);
    s.grid_s01 = make_float4(reg.s01[0], reg.s01[1], reg.s01[2], 0.0f);
    s.grid_s02 = make_float4(reg.s02[0], reg.s02[1], reg.s02[2], 0.0f);
    s.light_col = c->light_col.as<float4>();
    // w = p / (1/L) (light.cpp:80) equals p * L exactly when 1/L is a power of two
    s.light_scale = (num_lights && (num_lights & (num_lights - 1)) == 0) ? (float)num_lights : 0.0f;
    s.lights_finite = 1u;
    for (uint32_t i = 0; i < 28 * num_lights; i++)
        if (!std::isfinite(lt[i]) && (i % 4) != 3) s.lights_finite = 0u;
    // every product colour x kd / colour x ks stays finite (with a margin for the mix() rounding of segment /
    // parallelogram colours): shade() may then skip its per-component NaN tests for finite dotNL and pow
    {
        double cmax = 0.0, kmax = 0.0;
        bool finite = true;
        for (uint32_t i = 0; i < num_lights; i++)
            for (int r = 3; r < 7; r++)
                for (int a = 0; a < 3; a++) {
                    const float v = lt[28 * i + 4 * r + a];
                    finite = finite && std::isfinite(v);
                    cmax = std::max(cmax, (double)std::fabs(v));
                }
        for (uint32_t m = 0; m <= num_meshes; m++)
            for (int a : {0, 1, 2, 4, 5, 6}) {
                const float v = mats[12 * m + a];
                finite = finite && std::isfinite(v);
                kmax = std::max(kmax, (double)std::fabs(v));
            }
        finite = finite && tfinite;   // texels are diffuse colours too
        kmax = std::max(kmax, tmax);
        s.shade_finite = (finite && cmax * kmax <= 0x1p120) ? 1u : 0u;
        bool miss_zero = s.lights_finite && cmax <= 0x1p126;
        for (int a : {0, 1, 2, 4, 5, 6}) miss_zero = miss_zero && mats[12 * num_meshes + a] == 0.0f;
        s.miss_shade_zero = miss_zero ? 1u : 0u;
    }
    s.normals_bounded = 1u;
    for (const std::vector<float>* nv : {&n0, &n1, &n2})
        for (size_t i = 0; i < nv->size(); i++)
            if ((i % 4) != 3 && !(std::fabs((*nv)[i]) <= 0x1p125f)) s.normals_bounded = 0u;
    static std::atomic<uint64_t> scene_gens{0};
    c->scene_gen = ++scene_gens;
    c->has_scene = true;
    return RESTIR_OK;
}

// visualiseAlphas (render_utils.cpp:189-243) of the accumulators so far: k_romis_vis_t{T} solves and colours the
// 3T images on the device, the host writes them to <renders dir>/<currentTime()>/ (utils.cpp:16-22's format).
static restir_status save_alphas_visualisation(restir_ctx* c, uint32_t W, uint32_t H, uint32_t T) {
    const size_t npx = (size_t)W * H, words = (size_t)3 * T * npx;
    ST_TRY(c->mis_vis.ensure(words * 4));
    HIP_TRY(launch_romis_vis(W, H, T, c->mis_acc.as<float>(), c->mis_vis.as<uint32_t>(), c->stream));
    c->mis_vis_host.resize(words);
    HIP_TRY(hipMemcpyAsync(c->mis_vis_host.data(), c->mis_vis.p, words * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    const std::time_t now = std::time(nullptr);
    std::tm tm_local{};
    localtime_r(&now, &tm_local);
    char stamp[64];
    std::strftime(stamp, sizeof(stamp), "%d-%m-%Y %H-%M-%S", &tm_local);
    const std::filesystem::path dir = std::filesystem::path(c->renders_dir) / stamp;
    std::error_code ec;
    std::filesystem::create_directories(dir, ec);
    if (ec) return fail(RESTIR_ERR_INVALID, "alpha visualisation: cannot create %s: %s", dir.c_str(), ec.message().c_str());
    static const char* const kColour[3] = {"Red", "Green", "Blue"};   // enum Color (render_utils.cpp:238)
    for (uint32_t i = 0; i < T; i++)
        for (uint32_t ch = 0; ch < 3; ch++) {
            const std::filesystem::path file =
                dir / ("Distribution " + std::to_string(i) + " - " + kColour[ch] + ".bmp");
            if (!write_bmp_words(file.c_str(), W, H, c->mis_vis_host.data() + (size_t)(3 * i + ch) * npx))
                return fail(RESTIR_ERR_INVALID, "alpha visualisation: cannot write %s", file.c_str());
        }
    return RESTIR_OK;
}

// renderRMIS / renderROMIS (render.cpp:64-265) over the whole image; the caller holds c->mu.
static restir_status render_mis(restir_ctx* c, const restir_camera* cam, const restir_features* features, uint32_t W,
                                uint32_t H, float* out_rgb) {
    if (W == 0 || H == 0) return fail(RESTIR_ERR_INVALID, "empty image %ux%u", W, H);
    ST_TRY(check_romis_window(features, W, H));
    const FeaturesDev f = to_dev(features);
    ST_TRY(ensure_work(c, W, H, f.N, true));
    ST_TRY(ensure_mis(c, features, W, H));
    ST_TRY(c->rgb.ensure((size_t)W * H * 12));
    c->rgb_w = W; c->rgb_h = H;
    c->stage_ok = false;   // the stage buffers now hold this render's state
    const CameraDev camd = camera_dev(cam);
    const Region view = make_region(W, H, 0, 0, W, H, 0, 0, W, H);
    const uint32_t frame = c->frame_index++;
    SceneDev s;
    ST_TRY(scene_for(c, f, (size_t)W * H, s));
    float4* nt = c->n_t.as<float4>();
    float4* pm = c->p_mat.as<float4>();
    TIMED(c, RESTIR_K_PRIMARY, launch_primary(s, view, camd, nt, pm, nullptr, c->tuning, c->stream));
    TIMED(c, RESTIR_K_MIS, launch_mis_neighbours(s, W, H, f, restir_rng_key(c->seed, frame, RESTIR_STAGE_NEIGHBOURS, 0),
                                                 restir_rng_key(c->seed, frame, RESTIR_STAGE_NEIGHBOURS, 1), nt, pm,
                                                 c->mis_nbr.as<uint32_t>(), c->stream));
    HIP_TRY(hipMemsetAsync(c->mis_acc.p, 0, (size_t)c->mis_rows * W * H * 4, c->stream));
    for (uint32_t it = 0; it < features->max_iterations_mis; it++) {
        TIMED(c, RESTIR_K_RIS, launch_ris(s, view, f, restir_rng_key(c->seed, frame, RESTIR_STAGE_RIS, it), camd.origin, nt, pm,
                                          c->ra[0].as<float4>(), c->rb[0].as<float4>(), c->dbg[0].as<float2>(), nullptr,
                                          c->tuning, c->stream));
        TIMED(c, RESTIR_K_MIS, launch_mis_accumulate(s, W, H, f, camd.origin, nt, pm, c->mis_nbr.as<uint32_t>(),
                                                     c->ra[0].as<float4>(), c->rb[0].as<float4>(), c->dbg[0].as<float2>(), it,
                                                     c->mis_acc.as<float>(), c->mis_smp.as<float>(), c->mis_smp_samples,
                                                     c->tuning, c->stream));
        if (f.mode == RESTIR_MODE_ROMIS && features->save_alphas_visualisation && !c->renders_dir.empty())
            ST_TRY(save_alphas_visualisation(c, W, H, f.K + 1u));   // render.cpp:227-229
    }
    TIMED(c, RESTIR_K_MIS, launch_mis_finish(W, H, f, c->mis_acc.as<float>(), c->rgb.as<float>(), c->stream));
    if (out_rgb) {
        HIP_TRY(hipMemcpyAsync(out_rgb, c->rgb.p, (size_t)W * H * 12, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    return RESTIR_OK;
}

// renderReSTIR (render.cpp:28-62)
restir_status restir_render(restir_ctx* c, const restir_camera* cam, const restir_features* features, uint32_t width,
                            uint32_t height, const restir_tile* tile, const restir_frame* prev, restir_frame** out_next,
                            float* out_rgb) {
    if (!c) return fail(RESTIR_ERR_INVALID, "ctx is NULL");
    if (!cam) return fail(RESTIR_ERR_INVALID, "camera is NULL");
    ST_TRY(check_features(features));
    if (out_next) *out_next = nullptr;
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->has_scene) return fail(RESTIR_ERR_STATE, "restir_render before restir_set_scene");
    HIP_TRY(hipSetDevice(c->device));
    if (features->ray_trace_mode != RESTIR_MODE_RESTIR) {   // renderRayTraced's switch (render.cpp:274-279)
        if (tile && (tile->global_width != width || tile->global_height != height || tile->x0 || tile->y0 ||
                     tile->width != width || tile->height != height))
            return fail(RESTIR_ERR_UNSUPPORTED, "R-MIS / R-OMIS render whole images only (no screen tiles)");
            return render_mis(c, cam, features, width, height, out_rgb);
    }

    restir_tile t{};
    if (tile) {
        t = *tile;
        if (t.global_width != width || t.global_height != height)
            return fail(RESTIR_ERR_INVALID, "tile global size %ux%u != %ux%u", t.global_width, t.global_height, width, height);
        if (t.width == 0 || t.height == 0 || t.x0 + t.width > width || t.y0 + t.height > height || t.gx0 > t.x0 ||
            t.gy0 > t.y0 || t.gx0 + t.gwidth < t.x0 + t.width || t.gy0 + t.gheight < t.y0 + t.height ||
            t.gx0 + t.gwidth > width || t.gy0 + t.gheight > height)
            return fail(RESTIR_ERR_INVALID, "inconsistent tile");
    } else {
        if (width == 0 || height == 0) return fail(RESTIR_ERR_INVALID, "empty image %ux%u", width, height);
        t.global_width = width; t.global_height = height;
        t.x0 = 0; t.y0 = 0; t.width = width; t.height = height;
        t.gx0 = 0; t.gy0 = 0; t.gwidth = width; t.gheight = height;
    }
    const FeaturesDev f = to_dev(features);
    const uint32_t N = f.N;
    const uint32_t passes = features->spatial_reuse ? features->spatial_resampling_passes : 0u;
    // the computed region must hold the ghost zone the spatial passes read (clipped at the image border)
    {
        restir_tile need{};
        const uint64_t g = (uint64_t)passes * f.R;
        uint32_t gx0 = t.x0 > g ? (uint32_t)(t.x0 - g) : 0u, gy0 = t.y0 > g ? (uint32_t)(t.y0 - g) : 0u;
        uint64_t gx1 = std::min<uint64_t>((uint64_t)t.x0 + t.width + g, width);
        uint64_t gy1 = std::min<uint64_t>((uint64_t)t.y0 + t.height + g, height);
        if (t.gx0 > gx0 || t.gy0 > gy0 || (uint64_t)t.gx0 + t.gwidth < gx1 || (uint64_t)t.gy0 + t.gheight < gy1)
            return fail(RESTIR_ERR_INVALID, "tile ghost zone narrower than passes * radius = %llu", (unsigned long long)g);
        (void)need;
    }
    const bool temporal = features->temporal_reuse && prev != nullptr;
    if (temporal) {
        if (prev->N != N || prev->vw != t.gwidth || prev->vh != t.gheight || prev->vx0 != t.gx0 || prev->vy0 != t.gy0 ||
            prev->W != width || prev->H != height)
            return fail(RESTIR_ERR_INVALID, "temporal predecessor grid does not match this frame's region / N");
        const bool has_ghost = t.gwidth != t.width || t.gheight != t.height;
        if (has_ghost && passes > 0)
            return fail(RESTIR_ERR_UNSUPPORTED, "temporal reuse on a ghost-zoned tile needs the predecessor's ghost zone: "
                                                "render such tiles with the halo-exchange stages (restir_halo_begin)");
        if (prev->records != (c->tuning.records != 0))
            return fail(RESTIR_ERR_INVALID, "temporal predecessor grid was rendered with the other buffer layout");
    }

    const hipStream_t st = c->stream;
    FrameBufs fb;
    ST_TRY(ensure_records(c, t.gwidth, t.gheight, N, fb));
    c->stage_ok = false;   // ensure_records re-sized the shared view state: the stage API must be reconfigured
    ST_TRY(fb.rgb().ensure((size_t)t.width * t.height * 12));
    c->rgb_w = t.width; c->rgb_h = t.height;

    const CameraDev camd = camera_dev(cam);
    const Region view = fb.region(make_region(width, height, t.gx0, t.gy0, t.gwidth, t.gheight, t.gx0, t.gy0, t.gwidth, t.gheight));
    const Region owned = fb.region(make_region(width, height, t.gx0, t.gy0, t.gwidth, t.gheight, t.x0, t.y0, t.width, t.height));
    const uint32_t frame = c->frame_index++;
    SceneDev s;
    ST_TRY(scene_for(c, f, (size_t)t.gwidth * t.gheight, s, &fb.uv()));
    float4* pm = fb.pm();
    int cur = 0;

    const uint32_t ris_key = restir_rng_key(c->seed, frame, RESTIR_STAGE_RIS, 0);
    // background tiles (MissTiles): N <= 2, no temporal reuse (its output is not the RIS result), the fused kernel with
    // one 32 x 8 tile per block; the spatial shortcuts also need bounded normals (their miss tests)
    uint8_t* tmiss = nullptr;
    const bool fused = c->tuning.fuse_primary_ris && primary_ris_fits(s);
    if (c->tuning.miss_tiles && fused && N <= 2 && !temporal &&
        s.normals_bounded && !fb.records) {
        const size_t tiles = (size_t)((t.gwidth + 31u) / 32u) * ((t.gheight + 7u) / 8u);
        ST_TRY(fb.tmiss().ensure((tiles + 3u) & ~(size_t)3u));   // whole words: the spatial pass reads its flag's word
        tmiss = fb.tmiss().as<uint8_t>();
    }
    // the first spatial pass substitutes a background tile's known reservoirs (k_spatial1_ntl / _t2, k_spatial1u); the
    // later passes and final shading read the passes' outputs, and with no ghost ring the last pass overwrites the
    // whole returned grid: RIS need not store those reservoirs
    const bool skip_res = tmiss && passes > 0 && t.gwidth == t.width && t.gheight == t.height &&
                          spatial_reads_flags(s, f, c->tuning) &&
                          (size_t)t.gwidth * t.gheight * 16u <= 0xFFFFFFFFull;
    // a single unbiased pass (k_spatial1u) also substitutes a background pixel's G-buffer records (own and the Z loop's
    // neighbours); final shading reads none of them (its tiles are the RIS tiles here): nor are those stored
    // Biased passes (every pass reads the flags) fix their window up instead (MissTiles::gbuf); knob miss.gbuf.
    const uint32_t mg = c->tuning.miss_gbuf;
    const bool gbuf_ok = mg && final_reads_flags(s, f, c->tuning) &&
                         (f.unbiased ? passes == 1u : (mg == 1u || t.gwidth >= 2048u));
    uint32_t skip_mode = skip_res ? (1u | (gbuf_ok ? 2u : 0u)) : 0u;
    // sample handles (k_spatial1h): N = 1 biased passes over a point-light scene, written by the fused RIS kernel and by
    // every pass but the last; 4 + 4 B per pixel and 16 B of slack (the planes are read a word at a time)
    // (point lights: two 4-byte planes; a regular light grid: one float4 plane, k_spatial1g)
    // With temporal reuse the passes read handles when the fused temporal kernel can rebuild the predecessor from its
    // frame handles (point lights, the same scene upload): every M then bounded by RIS's plus the clamp's
    const bool no_ghost = t.gwidth == t.width && t.gheight == t.height;
    const bool temporal_handles = temporal && fused && !fb.records && (N == 1 || N == 2) && no_ghost && prev->hgen != 0 &&
                                  prev->hgen == c->scene_gen && primary_ris_temporal_fits(s, f, c->tuning);
    // the M every sub-reservoir can hold entering the passes after temporal reuse: the current M plus each of the N
    // predecessor sub-reservoirs clamped to clampM M + 1 (kernels.hip ris_pixel TEMP)
    const uint64_t m_temporal = (uint64_t)f.M + (uint64_t)N * ((uint64_t)f.clamp_m * f.M + 1u);
    const uint64_t m_in = temporal ? m_temporal : 0u;
    const int hkind = (temporal && !temporal_handles) ? -1 : spatial_handle_kind(s, f, c->tuning, passes, m_in);
    const bool handles = fused && !fb.records && hkind >= 0 && (!temporal || hkind == 0 || hkind == 2) &&
                         (size_t)t.gwidth * t.gheight * 16u <= 0xFFFFFFFFull;
    // the last pass also writes the returned grid's handles (point lights, no ghost ring) for the next frame, bounded as
    // if that frame's temporal reuse had run (its M bound)
    const bool frame_handles = handles && (hkind == 0 || hkind == 2) && out_next && no_ghost &&
                               spatial_handle_kind(s, f, c->tuning, passes, m_temporal) == hkind;
    if (handles)
        for (int i = 0; i < 2; i++) ST_TRY(fb.hnd_()[i].ensure((size_t)t.gwidth * t.gheight * (hkind ? 16u : 8u) + 16u));
    // the handle passes read RIS's samples through the handles alone, and a pass's output is read by the next pass's
    // handles alone: their reservoir planes are dead (the last pass writes the returned grid's owned rect; a tile's
    // ghost ring holds intermediate values, include/restir_c.h)
    Handles ris_handles = fb.h(cur);
    ris_handles.res_dead = 1u;
    // temporal reuse inside the fused kernel (k_primary_ris_n{1,2}_lds_pt_temporal): the predecessor's reservoirs are
    // combined while the RIS reservoirs are still in registers (no store / reload, no G-buffer re-read, one launch less)
    const bool temporal_fused = temporal && fused && primary_ris_temporal_fits(s, f, c->tuning);
    if (temporal_fused) {
        ST_TRY(use_prev(prev, c->device, st, c->pool.get()));   // the predecessor's records are complete (its producer's stream)
        TIMED(c, RESTIR_K_PRIMARY_RIS,
              launch_primary_ris_temporal(s, view, camd, f, ris_key, fb.nt(0), pm, fb.nt2(), fb.ra(cur), fb.rb(cur), nullptr,
                                          fb.rp(cur), c->tuning, st,
                                          TemporalIn{fb.pa(prev), fb.pb(prev),
                                                     restir_rng_key(c->seed, frame, RESTIR_STAGE_TEMPORAL, 0),
                                                     handles ? fb.fhw(prev) : nullptr, handles ? fb.fhm(prev) : nullptr},
                                          handles ? ris_handles : Handles{nullptr, nullptr, 0u}));
        used_prev(prev, st, c->pool.get());
    } else if (fused) {   // same region: one kernel (kernels.hip k_primary_ris)
        bool written = false;
        TIMED(c, RESTIR_K_PRIMARY_RIS, launch_primary_ris(s, view, camd, f, ris_key, fb.nt(0), pm, fb.nt2(), fb.ra(cur),
                                                          fb.rb(cur), nullptr, fb.rp(cur), c->tuning, st, tmiss, skip_mode,
                                                          &written, handles ? ris_handles : Handles{nullptr, nullptr, 0u}));
        if (!written) {   // (then RIS skipped nothing either: its skips need the flags)
            tmiss = nullptr;
            skip_mode = 0u;
        }
    } else {
        TIMED(c, RESTIR_K_PRIMARY, launch_primary(s, view, camd, fb.nt(0), pm, fb.nt2(), c->tuning, st));
        TIMED(c, RESTIR_K_RIS, launch_ris(s, view, f, ris_key, camd.origin, fb.nt(cur), pm, fb.ra(cur), fb.rb(cur), nullptr,
                                          fb.rp(cur), c->tuning, st));
    }
    c->last_px = (uint64_t)t.gwidth * t.gheight;   // restir_background_pixels
    c->tmiss_w = tmiss ? t.gwidth : 0u;
    c->tmiss_h = tmiss ? t.gheight : 0u;
    if (temporal && !temporal_fused) {
        ST_TRY(use_prev(prev, c->device, st, c->pool.get()));   // the predecessor's records are complete (its producer's stream)
        TIMED(c, RESTIR_K_TEMPORAL,
              launch_temporal(s, view, f, restir_rng_key(c->seed, frame, RESTIR_STAGE_TEMPORAL, 0), camd.origin, fb.nt(cur), pm,
                              fb.ra(cur), fb.rb(cur), fb.pa(prev), fb.pb(prev), fb.ra(cur), fb.rb(cur), nullptr,
                              fb.rp(cur), fb.rp(cur), c->tuning, st));
        used_prev(prev, st, c->pool.get());
    }
    bool rp_ok = fb.rp(cur) != nullptr;   // the current grid's target-pdf cache holds its samples' pdfs
    // the last pass's own-pixel shadow rays (unbiased + visibility reuse, N = 1) go on to final shading
    uint8_t* vis = nullptr;
    bool vis_ok = false;
    if (passes && features->unbiased_combination && features->spatial_reuse_visibility_check && N == 1) {
        ST_TRY(fb.vis().ensure((size_t)t.gwidth * t.gheight));
        vis = fb.vis().as<uint8_t>();
    }
    for (uint32_t pass = 0; pass < passes; pass++) {
        const Region pr = grow_rect(owned, (passes - 1u - pass) * f.R);
        const int nxt = cur ^ 1;
        TIMED(c, RESTIR_K_SPATIAL,
              launch_spatial(s, pr, f, restir_rng_key(c->seed, frame, RESTIR_STAGE_SPATIAL, pass), camd.origin, fb.nt(cur), pm,
                             fb.ra(cur), fb.rb(cur), fb.ra(nxt), fb.rb(nxt), nullptr, rp_ok ? fb.rp(cur) : nullptr,
                             // every neighbour of this pass lies in the region the cache's producer covered (RIS /
                             // temporal: the whole view; pass p - 1: the owned rect grown by (P - p) R)
                             rp_ok ? fb.rp(cur) : nullptr,
                             // the last pass's pdf cache has no reader (final shading re-shades; the next frame's
                             // temporal pass evaluates its own): not written
                             pass + 1 < passes ? fb.rp(nxt) : nullptr, &rp_ok, c->tuning, st,
                             pass + 1 == passes ? vis : nullptr, &vis_ok,
                             // a background pixel holds M = f.M after RIS and after every biased pass; an unbiased pass
                             // sums its neighbours' M, which only pass 0 knows
                             MissTiles{tmiss, (!f.unbiased || pass == 0) ? f.M : 0u, (skip_mode & 2u) ? 1u : 0u},
                             handles ? fb.h(cur) : Handles{nullptr, nullptr, 0u},
                             // a pass before the last is read by the next one's handles alone: no reservoir planes
                             handles && pass + 1 < passes ? Handles{fb.h(nxt).w, fb.h(nxt).m, 1u}
                             : frame_handles              ? fb.fh(nxt)
                                                          : Handles{nullptr, nullptr, 0u}));
        cur = nxt;
    }
    TIMED(c, RESTIR_K_FINAL, launch_final(s, owned, f, camd.origin, fb.nt(cur), pm, fb.ra(cur), fb.rb(cur), fb.rgb().as<float>(),
                                          c->tuning, st, vis_ok ? vis : nullptr, MissTiles{tmiss, 0u, 0u}));
    c->cur = cur;

    if (out_next) {
        restir_frame* fr = make_frame(c->pool, c->device, st);   // after the final kernel, the records' last reader
        fr->W = width; fr->H = height; fr->vx0 = t.gx0; fr->vy0 = t.gy0; fr->vw = t.gwidth; fr->vh = t.gheight; fr->N = N;
        // hand the final grid's records to the frame (no copy); the context re-allocates lazily
        std::swap(fr->rec, fb.rec_()[cur]);
        fr->records = fb.records;
        fr->hgen = frame_handles ? c->scene_gen : 0u;
        *out_next = fr;
    }
    if (out_rgb) {
        HIP_TRY(hipMemcpyAsync(out_rgb, fb.rgb().p, (size_t)t.width * t.height * 12, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    return RESTIR_OK;
}

restir_status restir_frame_retain(restir_frame* fr) {
    if (!fr) return fail(RESTIR_ERR_INVALID, "frame is NULL");
    fr->refs.fetch_add(1);
    return RESTIR_OK;
}

void restir_frame_release(restir_frame* fr) {
    if (!fr) return;
    if (fr->refs.fetch_sub(1) == 1) {
        // stream-ordered: the records go back to the producing context's pool with the events of the work that
        // touched them (the next user waits on those on its own stream); no device-wide synchronisation
        (void)hipSetDevice(fr->device);
        std::vector<hipEvent_t> busy = std::move(fr->reads);
        if (fr->pool) {
            fr->pool->give(fr->rec, std::move(busy), fr->ready);   // ready: on the pool owner's stream
        } else {
            if (fr->ready) busy.push_back(fr->ready);
            FramePool::Entry e{fr->rec, std::move(busy)};
            FramePool::drain(e);
        }
        fr->rec = DevBuf{};
        delete fr;
    }
}

restir_status restir_frame_info(const restir_frame* fr, uint32_t* width, uint32_t* height, uint32_t* vx0, uint32_t* vy0,
                                uint32_t* vw, uint32_t* vh, uint32_t* n) {
    if (!fr) return fail(RESTIR_ERR_INVALID, "frame is NULL");
    if (width) *width = fr->W;
    if (height) *height = fr->H;
    if (vx0) *vx0 = fr->vx0;
    if (vy0) *vy0 = fr->vy0;
    if (vw) *vw = fr->vw;
    if (vh) *vh = fr->vh;
    if (n) *n = fr->N;
    return RESTIR_OK;
}

restir_status restir_frame_download(const restir_frame* fr, float* pos, float* color, float* w, uint32_t* m) {
    if (!fr) return fail(RESTIR_ERR_INVALID, "frame is NULL");
    HIP_TRY(hipSetDevice(fr->device));
    if (fr->ready) HIP_TRY(hipEventSynchronize(fr->ready));
    const size_t npx = (size_t)fr->vw * fr->vh, N = fr->N;
    // the records as stored: per pixel [n_t, a_0, b_0, a_1, b_1, ...] or planes [a_0 .. a_N-1 | b_0 .. b_N-1]
    const size_t f4 = fr->records ? npx * (1 + 2 * N) : npx * 2 * N;
    std::vector<float> host(4 * f4);
    HIP_TRY(hipMemcpy(host.data(), fr->rec.p, host.size() * 4, hipMemcpyDeviceToHost));
    for (size_t j = 0; j < N; j++)
        for (size_t p = 0; p < npx; p++) {
            const float* a = fr->records ? &host[4 * (p * (1 + 2 * N) + 1 + 2 * j)] : &host[4 * (j * npx + p)];
            const float* b = fr->records ? &host[4 * (p * (1 + 2 * N) + 2 + 2 * j)] : &host[4 * ((N + j) * npx + p)];
            const size_t i = j * npx + p;
            if (pos) { pos[3 * i] = a[0]; pos[3 * i + 1] = a[1]; pos[3 * i + 2] = a[2]; }
            if (w) w[i] = a[3];
            if (color) { color[3 * i] = b[0]; color[3 * i + 1] = b[1]; color[3 * i + 2] = b[2]; }
            if (m) std::memcpy(&m[i], &b[3], 4);
        }
    return RESTIR_OK;
}

restir_status restir_synchronize(restir_ctx* c) {
    if (!c) return fail(RESTIR_ERR_INVALID, "ctx is NULL");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return RESTIR_OK;
}

restir_status restir_download_rgb(restir_ctx* c, float* out_rgb, size_t count) {
    if (!c || !out_rgb) return fail(RESTIR_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(c->mu);
    const size_t need = (size_t)c->rgb_w * c->rgb_h * 3;
    if (need == 0) return fail(RESTIR_ERR_STATE, "nothing rendered yet");
    if (count < need) return fail(RESTIR_ERR_INVALID, "buffer holds %zu floats, need %zu", count, need);
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpyAsync(out_rgb, c->rgb.p, need * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return RESTIR_OK;
}

// ---------------------------------------------------------------------------------------------------------
// stage API (parity tests): a whole width x height image, reservoir slot 0 = "current", slot 1 = "prev"
restir_status restir_stage_configure(restir_ctx* c, uint32_t width, uint32_t height, uint32_t n) {
    if (!c || width == 0 || height == 0 || n < 1 || n > RESTIR_MAX_N) return fail(RESTIR_ERR_INVALID, "bad stage size");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    ST_TRY(ensure_work(c, width, height, n, true));
    ST_TRY(c->rgb.ensure((size_t)width * height * 12));
    c->rgb_w = width; c->rgb_h = height;
    c->stage_rg = make_region(width, height, 0, 0, width, height, 0, 0, width, height);
    c->stage_ok = true;
    c->cur = 0;
    return RESTIR_OK;
}

static restir_status stage_buffer(restir_ctx* c, restir_buffer which, DevBuf** out, size_t* bytes) {
    const size_t npx = (size_t)c->vw * c->vh;
    const int cur = c->cur, prv = c->cur ^ 1;
    switch (which) {
        case RESTIR_BUF_GBUF_N_T: *out = &c->n_t; *bytes = npx * 16; break;
        case RESTIR_BUF_GBUF_P_MAT: *out = &c->p_mat; *bytes = npx * 16; break;
        case RESTIR_BUF_RES_A: *out = &c->ra[cur]; *bytes = npx * c->N * 16; break;
        case RESTIR_BUF_RES_B: *out = &c->rb[cur]; *bytes = npx * c->N * 16; break;
        case RESTIR_BUF_RES_DBG: *out = &c->dbg[cur]; *bytes = npx * c->N * 8; break;
        case RESTIR_BUF_PREV_A: *out = &c->ra[prv]; *bytes = npx * c->N * 16; break;
        case RESTIR_BUF_PREV_B: *out = &c->rb[prv]; *bytes = npx * c->N * 16; break;
        case RESTIR_BUF_PREV_DBG: *out = &c->dbg[prv]; *bytes = npx * c->N * 8; break;
        case RESTIR_BUF_RGB: *out = &c->rgb; *bytes = (size_t)c->rgb_w * c->rgb_h * 12; break;
        case RESTIR_BUF_GBUF_UV:
            if (!c->sdev.num_textures) return fail(RESTIR_ERR_INVALID, "gbuf_uv: the scene has no textures");
            ST_TRY(c->uv.ensure(npx * 8));
            *out = &c->uv; *bytes = npx * 8; break;
        case RESTIR_BUF_MIS_NBR:
            if (!c->mis_cap) return fail(RESTIR_ERR_STATE, "MIS buffers: call restir_stage_mis_capacity first");
            *out = &c->mis_nbr; *bytes = (size_t)(1u + c->mis_cap) * npx * 4; break;
        case RESTIR_BUF_MIS_ACC:
            if (!c->mis_cap) return fail(RESTIR_ERR_STATE, "MIS buffers: call restir_stage_mis_capacity first");
            *out = &c->mis_acc; *bytes = (size_t)c->mis_rows * npx * 4; break;
        default: return fail(RESTIR_ERR_INVALID, "unknown buffer %d", (int)which);
    }
    return RESTIR_OK;
}

restir_status restir_stage_upload(restir_ctx* c, restir_buffer which, const void* host, size_t bytes) {
    if (!c || !host) return fail(RESTIR_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->stage_ok) return fail(RESTIR_ERR_STATE, "restir_stage_configure first");
    DevBuf* b;
    size_t need;
    ST_TRY(stage_buffer(c, which, &b, &need));
    if (bytes != need) return fail(RESTIR_ERR_INVALID, "buffer %d: %zu bytes given, %zu expected", (int)which, bytes, need);
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpyAsync(b->p, host, bytes, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return RESTIR_OK;
}

restir_status restir_stage_download(restir_ctx* c, restir_buffer which, void* host, size_t bytes) {
    if (!c || !host) return fail(RESTIR_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->stage_ok) return fail(RESTIR_ERR_STATE, "restir_stage_configure first");
    DevBuf* b;
    size_t need;
    ST_TRY(stage_buffer(c, which, &b, &need));
    if (bytes != need) return fail(RESTIR_ERR_INVALID, "buffer %d: %zu bytes given, %zu expected", (int)which, bytes, need);
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpyAsync(host, b->p, bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return RESTIR_OK;
}

#define STAGE_PRELUDE()                                                             \
    if (!c) return fail(RESTIR_ERR_INVALID, "ctx is NULL");                         \
    std::lock_guard<std::mutex> lk(c->mu);                                          \
    if (!c->stage_ok) return fail(RESTIR_ERR_STATE, "restir_stage_configure first"); \
    if (!c->has_scene) return fail(RESTIR_ERR_STATE, "restir_set_scene first");      \
    HIP_TRY(hipSetDevice(c->device));                                               \

restir_status restir_stage_primary(restir_ctx* c, const restir_camera* cam) {
    if (!cam) return fail(RESTIR_ERR_INVALID, "camera is NULL");
    STAGE_PRELUDE();
    const CameraDev camd = camera_dev(cam);
    FeaturesDev d{};
    d.texture = 1u;
    SceneDev sd;
    ST_TRY(scene_for(c, d, (size_t)c->vw * c->vh, sd));
    TIMED(c, RESTIR_K_PRIMARY, launch_primary(sd, c->stage_rg, camd, c->n_t.as<float4>(), c->p_mat.as<float4>(), nullptr,
                                              c->tuning, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return RESTIR_OK;
}

static restir_status stage_features(restir_ctx* c, const restir_features* f, FeaturesDev& d) {
    ST_TRY(check_features(f));
    if (f->num_samples_in_reservoir != c->N)
        return fail(RESTIR_ERR_INVALID, "N=%u but stage configured for N=%u", f->num_samples_in_reservoir, c->N);
    d = to_dev(f);
    return RESTIR_OK;
}

restir_status restir_stage_ris(restir_ctx* c, const restir_camera* cam, const restir_features* f, uint32_t key, int debug) {
    if (!cam) return fail(RESTIR_ERR_INVALID, "camera is NULL");
    STAGE_PRELUDE();
    FeaturesDev d;
    ST_TRY(stage_features(c, f, d));
    SceneDev sd;
    ST_TRY(scene_for(c, d, (size_t)c->vw * c->vh, sd));
    const CameraDev camd = camera_dev(cam);
    const int cur = c->cur;
    TIMED(c, RESTIR_K_RIS, launch_ris(sd, c->stage_rg, d, key, camd.origin, c->n_t.as<float4>(), c->p_mat.as<float4>(),
                                      c->ra[cur].as<float4>(), c->rb[cur].as<float4>(),
                                      debug ? c->dbg[cur].as<float2>() : nullptr, nullptr, c->tuning, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return RESTIR_OK;
}

restir_status restir_stage_temporal(restir_ctx* c, const restir_camera* cam, const restir_features* f, uint32_t key,
                                    int debug) {
    if (!cam) return fail(RESTIR_ERR_INVALID, "camera is NULL");
    STAGE_PRELUDE();
    FeaturesDev d;
    ST_TRY(stage_features(c, f, d));
    SceneDev sd;
    ST_TRY(scene_for(c, d, (size_t)c->vw * c->vh, sd));
    const CameraDev camd = camera_dev(cam);
    const int cur = c->cur, prv = cur ^ 1;
    TIMED(c, RESTIR_K_TEMPORAL,
          launch_temporal(sd, c->stage_rg, d, key, camd.origin, c->n_t.as<float4>(), c->p_mat.as<float4>(),
                          c->ra[cur].as<float4>(), c->rb[cur].as<float4>(), c->ra[prv].as<float4>(), c->rb[prv].as<float4>(),
                          c->ra[cur].as<float4>(), c->rb[cur].as<float4>(), debug ? c->dbg[cur].as<float2>() : nullptr,
                          nullptr, nullptr, c->tuning, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return RESTIR_OK;
}

restir_status restir_stage_spatial(restir_ctx* c, const restir_camera* cam, const restir_features* f, uint32_t key,
                                   int debug) {
    if (!cam) return fail(RESTIR_ERR_INVALID, "camera is NULL");
    STAGE_PRELUDE();
    FeaturesDev d;
    ST_TRY(stage_features(c, f, d));
    SceneDev sd;
    ST_TRY(scene_for(c, d, (size_t)c->vw * c->vh, sd));
    const CameraDev camd = camera_dev(cam);
    const int cur = c->cur, nxt = cur ^ 1;
    TIMED(c, RESTIR_K_SPATIAL,
          launch_spatial(sd, c->stage_rg, d, key, camd.origin, c->n_t.as<float4>(), c->p_mat.as<float4>(),
                         c->ra[cur].as<float4>(), c->rb[cur].as<float4>(), c->ra[nxt].as<float4>(), c->rb[nxt].as<float4>(),
                         debug ? c->dbg[nxt].as<float2>() : nullptr, nullptr, nullptr, nullptr, nullptr, c->tuning,
                         c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->cur = nxt;   // the pass output becomes "current" (RES_*), its input "prev" (PREV_*)
    return RESTIR_OK;
}

restir_status restir_stage_final(restir_ctx* c, const restir_camera* cam, const restir_features* f) {
    if (!cam) return fail(RESTIR_ERR_INVALID, "camera is NULL");
    STAGE_PRELUDE();
    FeaturesDev d;
    ST_TRY(stage_features(c, f, d));
    SceneDev sd;
    ST_TRY(scene_for(c, d, (size_t)c->vw * c->vh, sd));
    const CameraDev camd = camera_dev(cam);
    const int cur = c->cur;
    TIMED(c, RESTIR_K_FINAL, launch_final(sd, c->stage_rg, d, camd.origin, c->n_t.as<float4>(), c->p_mat.as<float4>(),
                                          c->ra[cur].as<float4>(), c->rb[cur].as<float4>(), c->rgb.as<float>(), c->tuning, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return RESTIR_OK;
}

restir_status restir_stage_mis_capacity(restir_ctx* c, const restir_features* f, uint32_t* out_cap) {
    if (!out_cap) return fail(RESTIR_ERR_INVALID, "out_cap is NULL");
    STAGE_PRELUDE();
    FeaturesDev d;
    ST_TRY(stage_features(c, f, d));
    SceneDev sd;
    ST_TRY(scene_for(c, d, (size_t)c->vw * c->vh, sd));
    ST_TRY(ensure_mis(c, f, c->vw, c->vh));
    *out_cap = c->mis_cap;
    return RESTIR_OK;
}

restir_status restir_stage_neighbours(restir_ctx* c, const restir_features* f, uint32_t key_similar, uint32_t key_dissimilar) {
    STAGE_PRELUDE();
    FeaturesDev d;
    ST_TRY(stage_features(c, f, d));
    SceneDev sd;
    ST_TRY(scene_for(c, d, (size_t)c->vw * c->vh, sd));
    ST_TRY(ensure_mis(c, f, c->vw, c->vh));
    TIMED(c, RESTIR_K_MIS, launch_mis_neighbours(sd, c->vw, c->vh, d, key_similar, key_dissimilar, c->n_t.as<float4>(),
                                                 c->p_mat.as<float4>(), c->mis_nbr.as<uint32_t>(), c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return RESTIR_OK;
}

restir_status restir_stage_mis_accumulate(restir_ctx* c, const restir_camera* cam, const restir_features* f, uint32_t iteration) {
    if (!cam) return fail(RESTIR_ERR_INVALID, "camera is NULL");
    STAGE_PRELUDE();
    FeaturesDev d;
    ST_TRY(stage_features(c, f, d));
    SceneDev sd;
    ST_TRY(scene_for(c, d, (size_t)c->vw * c->vh, sd));
    ST_TRY(check_romis_window(f, c->vw, c->vh));
    ST_TRY(ensure_mis(c, f, c->vw, c->vh));
    const CameraDev camd = camera_dev(cam);
    const int cur = c->cur;
    if (iteration == 0) HIP_TRY(hipMemsetAsync(c->mis_acc.p, 0, (size_t)c->mis_rows * c->vw * c->vh * 4, c->stream));
    TIMED(c, RESTIR_K_MIS, launch_mis_accumulate(sd, c->vw, c->vh, d, camd.origin, c->n_t.as<float4>(), c->p_mat.as<float4>(),
                                                 c->mis_nbr.as<uint32_t>(), c->ra[cur].as<float4>(), c->rb[cur].as<float4>(),
                                                 c->dbg[cur].as<float2>(), iteration, c->mis_acc.as<float>(),
                                                 c->mis_smp.as<float>(), c->mis_smp_samples, c->tuning, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return RESTIR_OK;
}

restir_status restir_stage_mis_finish(restir_ctx* c, const restir_features* f) {
    STAGE_PRELUDE();
    FeaturesDev d;
    ST_TRY(stage_features(c, f, d));
    SceneDev sd;
    ST_TRY(scene_for(c, d, (size_t)c->vw * c->vh, sd));
    if (!c->mis_cap) return fail(RESTIR_ERR_STATE, "MIS buffers: run restir_stage_mis_accumulate first");
    TIMED(c, RESTIR_K_MIS, launch_mis_finish(c->vw, c->vh, d, c->mis_acc.as<float>(), c->rgb.as<float>(), c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return RESTIR_OK;
}

restir_status restir_debug_cod_solve(restir_ctx* c, uint32_t n, const float* A, const float* b, float* x, size_t count) {
    if (!c || (count && (!A || !b || !x))) return fail(RESTIR_ERR_INVALID, "null argument");
    if (n < 1 || n > RESTIR_ROMIS_MAX_TECHNIQUES) return fail(RESTIR_ERR_INVALID, "n = %u outside 1..%u", n, RESTIR_ROMIS_MAX_TECHNIQUES);
    if (count > 0xFFFFFFFFull) return fail(RESTIR_ERR_INVALID, "count too large");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    DevBuf bA, bb, bx;
    ST_TRY(bA.upload(A, count * n * n * 4, c->stream));
    ST_TRY(bb.upload(b, count * n * 4, c->stream));
    ST_TRY(bx.ensure(count * n * 4));
    hipError_t e = launch_debug_cod(n, bA.as<float>(), bb.as<float>(), bx.as<float>(), (uint32_t)count, c->stream);
    if (e != hipSuccess) return fail(RESTIR_ERR_HIP, "debug cod launch: %s", hipGetErrorString(e));
    HIP_TRY(hipMemcpyAsync(x, bx.p, count * n * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    bA.release(); bb.release(); bx.release();
    return RESTIR_OK;
}

restir_status restir_debug_math(restir_ctx* c, const float* x, const float* y, float* out_pow, float* out_exp, size_t n) {
    if (!c || (n && (!x || !y || !out_pow || !out_exp))) return fail(RESTIR_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    DevBuf bx, by, bp, be;
    ST_TRY(bx.upload(x, n * 4, c->stream));
    ST_TRY(by.upload(y, n * 4, c->stream));
    ST_TRY(bp.ensure(n * 4));
    ST_TRY(be.ensure(n * 4));
    hipError_t e = launch_debug_math(bx.as<float>(), by.as<float>(), bp.as<float>(), be.as<float>(), (uint32_t)n, c->stream);
    if (e != hipSuccess) return fail(RESTIR_ERR_HIP, "debug math launch: %s", hipGetErrorString(e));
    HIP_TRY(hipMemcpyAsync(out_pow, bp.p, n * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(out_exp, be.p, n * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    bx.release(); by.release(); bp.release(); be.release();
    return RESTIR_OK;
}

restir_status restir_background_pixels(restir_ctx* c, uint64_t* background, uint64_t* computed) {
    if (!c || !background || !computed) return fail(RESTIR_ERR_INVALID, "bad argument");
    std::lock_guard<std::mutex> lk(c->mu);
    *background = 0;
    *computed = c->last_px;
    if (!c->tmiss_w || !c->tmiss.p) return RESTIR_OK;
    HIP_TRY(hipSetDevice(c->device));
    const uint32_t ntx = (c->tmiss_w + 31u) / 32u, nty = (c->tmiss_h + 7u) / 8u;
    std::vector<uint8_t> flags((size_t)ntx * nty);
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipMemcpy(flags.data(), c->tmiss.p, flags.size(), hipMemcpyDeviceToHost));
    uint64_t bg = 0;
    for (uint32_t ty = 0; ty < nty; ty++)
        for (uint32_t tx = 0; tx < ntx; tx++)
            if (flags[(size_t)ty * ntx + tx] == 0u)   // flag 0: a background tile (kernels.hip primary_ris_body)
                bg += (uint64_t)std::min(32u, c->tmiss_w - 32u * tx) * std::min(8u, c->tmiss_h - 8u * ty);
    *background = bg;
    return RESTIR_OK;
}

restir_status restir_measure_read_bandwidth(restir_ctx* c, uint64_t bytes, uint32_t iters, double* out_gbps) {
    if (!c || !out_gbps || iters == 0 || bytes < (1u << 20)) return fail(RESTIR_ERR_INVALID, "bad argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    const size_t n4 = (size_t)(bytes / 16);
    DevBuf buf, sink;
    ST_TRY(buf.ensure(n4 * 16));
    ST_TRY(sink.ensure(1 << 20));
    HIP_TRY(hipMemsetAsync(buf.p, 0, n4 * 16, c->stream));
    hipEvent_t e0, e1;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    hipError_t e = launch_read_stream(buf.as<float4>(), n4, sink.as<float>(), c->stream);   // warm
    if (e == hipSuccess) e = hipEventRecord(e0, c->stream);
    for (uint32_t i = 0; i < iters && e == hipSuccess; i++) e = launch_read_stream(buf.as<float4>(), n4, sink.as<float>(), c->stream);
    if (e == hipSuccess) e = hipEventRecord(e1, c->stream);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float ms = 0.0f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    buf.release();
    sink.release();
    if (e != hipSuccess) return fail(RESTIR_ERR_HIP, "read-bandwidth kernel: %s", hipGetErrorString(e));
    *out_gbps = (double)n4 * 16.0 * iters / (ms * 1e-3) / 1e9;
    return RESTIR_OK;
}

// ---------------------------------------------------------------------------------------------------------
// halo-mode frames (include/restir_c.h "Reservoir halo exchange"): the stages of restir_render with the
// ghost-zone recomputation replaced by an exchange of the owned border strips before each spatial pass
namespace {
restir_status to_segs(const restir_halo_segment* g, uint32_t n, HaloSegs& hs, uint64_t& bytes) {
    if (n > RESTIR_MAX_HALO_SEGS) return fail(RESTIR_ERR_INVALID, "halo: %u segments", n);
    hs = HaloSegs{};
    hs.n = n;
    uint64_t px = 0;
    bytes = 0;
    for (uint32_t i = 0; i < n; i++) {
        hs.x0[i] = g[i].x0; hs.y0[i] = g[i].y0; hs.w[i] = g[i].width; hs.h[i] = g[i].height;
        hs.px0[i] = (uint32_t)px;
        px += (uint64_t)g[i].width * g[i].height;
        bytes += g[i].bytes;
    }
    if (px >= (1ull << 31)) return fail(RESTIR_ERR_INVALID, "halo: %llu pixels", (unsigned long long)px);
    hs.px0[n] = (uint32_t)px;
    return RESTIR_OK;
}
}  // namespace

restir_status restir_halo_begin(restir_ctx* c, const restir_camera* cam, const restir_features* features, uint32_t width,
                                uint32_t height, uint32_t tiles_x, uint32_t tiles_y, uint32_t rank, const restir_frame* prev,
                                uint64_t* send_bytes, uint64_t* recv_bytes) {
    restir_tile_layout L;
    ST_TRY(restir_layout_even(width, height, tiles_x, tiles_y, &L));
    return restir_halo_begin_layout(c, cam, features, &L, rank, prev, send_bytes, recv_bytes);
}

restir_status restir_halo_begin_layout(restir_ctx* c, const restir_camera* cam, const restir_features* features,
                                       const restir_tile_layout* layout, uint32_t rank, const restir_frame* prev,
                                       uint64_t* send_bytes, uint64_t* recv_bytes) {
    if (!c || !cam) return fail(RESTIR_ERR_INVALID, "null argument");
    ST_TRY(check_features(features));
    ST_TRY(layout_check(layout));
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->has_scene) return fail(RESTIR_ERR_STATE, "restir_halo_begin before restir_set_scene");
    HIP_TRY(hipSetDevice(c->device));
    const FeaturesDev f = to_dev(features);
    const uint32_t passes = features->spatial_reuse ? features->spatial_resampling_passes : 0u;
    const uint32_t width = layout->global_width, height = layout->global_height;
    const uint32_t tiles_x = layout->tiles_x, tiles_y = layout->tiles_y;
    restir_tile t{};
    ST_TRY(restir_layout_tile(layout, rank, passes ? f.R : 0u, &t));
    // plan into locals, validate everything, then commit to c->halo (a failure leaves no half-updated plan)
    restir_halo_segment sg[RESTIR_MAX_HALO_SEGS], rg_[RESTIR_MAX_HALO_SEGS];
    uint32_t n = 0;
    HaloSegs send{}, recv{};
    uint64_t send_b = 0, recv_b = 0;
    if (passes) {   // no spatial pass, no exchange: skip the plan (and its segment cap)
        n = RESTIR_MAX_HALO_SEGS;
        ST_TRY(restir_layout_halo_plan(layout, rank, f.R, f.N, sg, rg_, &n));
        ST_TRY(to_segs(sg, n, send, send_b));
        ST_TRY(to_segs(rg_, n, recv, recv_b));
    }
    const bool temporal = features->temporal_reuse && prev != nullptr;
    if (temporal) {
        if (prev->N != f.N || prev->vw != t.gwidth || prev->vh != t.gheight || prev->vx0 != t.gx0 ||
            prev->vy0 != t.gy0 || prev->W != width || prev->H != height)
            return fail(RESTIR_ERR_INVALID, "temporal predecessor grid does not match this tile's view / N");
        if (prev->records != (c->tuning.records != 0))
            return fail(RESTIR_ERR_INVALID, "temporal predecessor grid was rendered with the other buffer layout");
        ST_TRY(use_prev(prev, c->device, c->stream, c->pool.get()));
    }
    auto& h = c->halo;
    h.active = false;
    FrameBufs fb;
    ST_TRY(ensure_records(c, t.gwidth, t.gheight, f.N, fb));
    c->stage_ok = false;
    h.send = send; h.recv = recv; h.send_bytes = send_b; h.recv_bytes = recv_b;
    for (uint32_t i = 0; i < n; i++) { h.send_rank[i] = sg[i].rank; h.recv_rank[i] = rg_[i].rank; }
    halo_ops_from(sg, rg_, n, h.ops);
    h.nops = 2 * n;
    h.rank = rank;
    h.nranks = tiles_x * tiles_y;
    h.interior_done = false;
    ST_TRY(c->rgb.ensure((size_t)t.width * t.height * 12));
    c->rgb_w = t.width; c->rgb_h = t.height;
    h.W = width; h.H = height;
    h.view = fb.region(make_region(width, height, t.gx0, t.gy0, t.gwidth, t.gheight, t.gx0, t.gy0, t.gwidth, t.gheight));
    h.owned = fb.region(make_region(width, height, t.gx0, t.gy0, t.gwidth, t.gheight, t.x0, t.y0, t.width, t.height));
    h.fb_records = fb.records;
    h.f = f;
    h.camd = camera_dev(cam);
    h.frame = c->frame_index++;
    h.pass = 0;
    h.passes = passes;
    h.cur = 0;
    SceneDev s;
    ST_TRY(scene_for(c, f, (size_t)t.gwidth * t.gheight, s));
    float4* pm = c->p_mat.as<float4>();
    // G-buffer on the whole view (the spatial passes read the neighbours' depth / normal / position).  Without temporal
    // reuse: restir_render's fused primary + RIS kernel over the whole view, with its background-tile flags (the ring's
    // RIS results are the ones its owner computes -- same G-buffer, same global-pixel keys -- and the exchange before
    // the first pass overwrites them with those same values), so the passes and final shading write background tiles
    // without reading them; the ring's RIS costs (ring / tile) of the RIS time.  Otherwise primary rays on the view
    // and RIS / temporal reuse on the owned rectangle.
    const bool fused = !temporal && c->tuning.fuse_primary_ris && primary_ris_fits(s);
    h.tmiss = nullptr;
    if (fused) {
        uint8_t* tm = nullptr;
        if (c->tuning.miss_tiles && f.N <= 2 && s.normals_bounded && !fb.records) {
            const size_t tiles = (size_t)((t.gwidth + 31u) / 32u) * ((t.gheight + 7u) / 8u);
            ST_TRY(c->tmiss.ensure((tiles + 3u) & ~(size_t)3u));   // whole words (the spatial pass reads its flag's word)
            tm = c->tmiss.as<uint8_t>();
        }
        bool written = false;
        TIMED(c, RESTIR_K_PRIMARY_RIS,
              launch_primary_ris(s, h.view, h.camd, f, restir_rng_key(c->seed, h.frame, RESTIR_STAGE_RIS, 0), fb.nt(0), pm,
                                 fb.nt2(), fb.ra(0), fb.rb(0), nullptr, fb.rp(0), c->tuning, c->stream, tm, 0u, &written));
        if (written) h.tmiss = tm;
    } else {
        TIMED(c, RESTIR_K_PRIMARY, launch_primary(s, h.view, h.camd, fb.nt(0), pm, fb.nt2(), c->tuning, c->stream));
        TIMED(c, RESTIR_K_RIS, launch_ris(s, h.owned, f, restir_rng_key(c->seed, h.frame, RESTIR_STAGE_RIS, 0),
                                          h.camd.origin, fb.nt(0), pm, fb.ra(0), fb.rb(0), nullptr, fb.rp(0), c->tuning,
                                          c->stream));
    }
    if (temporal)
        TIMED(c, RESTIR_K_TEMPORAL,
              launch_temporal(s, h.owned, f, restir_rng_key(c->seed, h.frame, RESTIR_STAGE_TEMPORAL, 0), h.camd.origin, fb.nt(0),
                              pm, fb.ra(0), fb.rb(0), fb.pa(prev), fb.pb(prev), fb.ra(0), fb.rb(0), nullptr, fb.rp(0),
                              fb.rp(0), c->tuning, c->stream));
    if (temporal) used_prev(prev, c->stream, c->pool.get());
    h.rp_ok = fb.rp(0) != nullptr;
    h.active = true;
    if (send_bytes) *send_bytes = h.send_bytes;
    if (recv_bytes) *recv_bytes = h.recv_bytes;
    return RESTIR_OK;
}

restir_status restir_halo_pack(restir_ctx* c, void* buf, uint64_t bytes, int host_memory) {
    if (!c || (bytes && !buf)) return fail(RESTIR_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(c->mu);
    auto& h = c->halo;
    if (!h.active || h.pass >= h.passes) return fail(RESTIR_ERR_STATE, "restir_halo_pack outside a halo frame's passes");
    if (bytes != h.send_bytes) return fail(RESTIR_ERR_INVALID, "halo send buffer is %llu bytes, plan needs %llu",
                                           (unsigned long long)bytes, (unsigned long long)h.send_bytes);
    HIP_TRY(hipSetDevice(c->device));
    float4* dst = static_cast<float4*>(buf);
    if (host_memory) { ST_TRY(c->halo_scratch.ensure(bytes)); dst = c->halo_scratch.as<float4>(); }
    const FrameBufs fb{c, h.fb_records, (size_t)h.view.vw * h.view.vh, h.f.N};
    HIP_TRY(launch_halo_pack(h.view, h.send, h.f.N, fb.ra(h.cur), fb.rb(h.cur), dst, c->stream));
    if (host_memory && bytes) HIP_TRY(hipMemcpyAsync(buf, dst, bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));   // the caller's transport reads the buffer next
    return RESTIR_OK;
}

restir_status restir_halo_unpack(restir_ctx* c, const void* buf, uint64_t bytes, int host_memory) {
    if (!c || (bytes && !buf)) return fail(RESTIR_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(c->mu);
    auto& h = c->halo;
    if (!h.active || h.pass >= h.passes) return fail(RESTIR_ERR_STATE, "restir_halo_unpack outside a halo frame's passes");
    if (bytes != h.recv_bytes) return fail(RESTIR_ERR_INVALID, "halo recv buffer is %llu bytes, plan needs %llu",
                                           (unsigned long long)bytes, (unsigned long long)h.recv_bytes);
    HIP_TRY(hipSetDevice(c->device));
    const float4* src = static_cast<const float4*>(buf);
    if (host_memory && bytes) {
        ST_TRY(c->halo_scratch.ensure(bytes));
        HIP_TRY(hipMemcpyAsync(c->halo_scratch.p, buf, bytes, hipMemcpyHostToDevice, c->stream));
        src = c->halo_scratch.as<float4>();
    }
    const FrameBufs fb{c, h.fb_records, (size_t)h.view.vw * h.view.vh, h.f.N};
    HIP_TRY(launch_halo_unpack(h.view, h.recv, h.f.N, src, fb.ra(h.cur), fb.rb(h.cur), c->stream));
    if (host_memory) HIP_TRY(hipStreamSynchronize(c->stream));   // the host buffer may be reused on return
    return RESTIR_OK;
}

// The owned rectangle of a halo pass split into the interior -- pixels at least R from every side that faces
// another tile, whose neighbourhoods (+-R, clamped to the image) stay inside the owned rectangle -- and up to
// four border strips (bottom / top full width, left / right between them) that read the exchanged ring.
// Per-pixel results do not depend on how the rectangle is split into launches (keyed RNG by global pixel id).
struct HaloSplit {
    Region part[5];   // part[0] = interior (may be empty), part[1..nb] = border strips
    uint32_t nb;
};
static HaloSplit halo_split(const Region& owned, uint32_t R) {
    const uint32_t x0 = owned.rx0, y0 = owned.ry0, x1 = x0 + owned.rw, y1 = y0 + owned.rh;
    const uint32_t l = x0 > 0 ? R : 0u, r = x1 < owned.W ? R : 0u, b = y0 > 0 ? R : 0u, t = y1 < owned.H ? R : 0u;
    const uint32_t ix0 = x0 + std::min(l, owned.rw), ix1 = std::max(ix0, x1 - std::min(r, owned.rw));
    const uint32_t iy0 = y0 + std::min(b, owned.rh), iy1 = std::max(iy0, y1 - std::min(t, owned.rh));
    auto rect = [&](uint32_t ax0, uint32_t ay0, uint32_t ax1, uint32_t ay1) {
        Region q = owned;
        q.rx0 = ax0; q.ry0 = ay0; q.rw = ax1 - ax0; q.rh = ay1 - ay0;
        return q;
    };
    HaloSplit hs{};
    hs.part[0] = rect(ix0, iy0, ix1, iy1);
    hs.nb = 0;
    if (iy0 > y0) hs.part[1 + hs.nb++] = rect(x0, y0, x1, iy0);
    if (y1 > iy1) hs.part[1 + hs.nb++] = rect(x0, iy1, x1, y1);
    if (iy1 > iy0 && ix0 > x0) hs.part[1 + hs.nb++] = rect(x0, iy0, ix0, iy1);
    if (iy1 > iy0 && x1 > ix1) hs.part[1 + hs.nb++] = rect(ix1, iy0, x1, iy1);
    return hs;
}

// one launch of the current pass over `rg` (a part of the owned rectangle); the pdf cache stays valid only if
// every part wrote it.  The cache covers the owned rectangle only (the exchange moves reservoirs, not their
// pdfs), so only the interior -- whose neighbourhoods stay inside it -- may read it at neighbour pixels.
static restir_status halo_spatial_part(restir_ctx* c, const Region& rg, bool interior, bool& rp_written) {
    auto& h = c->halo;
    const int nxt = h.cur ^ 1;
    const FrameBufs fb{c, h.fb_records, (size_t)h.view.vw * h.view.vh, h.f.N};
    SceneDev sd;
    ST_TRY(scene_for(c, h.f, (size_t)h.view.vw * h.view.vh, sd));
    bool wrote = false;
    TIMED(c, RESTIR_K_SPATIAL,
          launch_spatial(sd, rg, h.f, restir_rng_key(c->seed, h.frame, RESTIR_STAGE_SPATIAL, h.pass), h.camd.origin,
                         fb.nt(h.cur), c->p_mat.as<float4>(), fb.ra(h.cur), fb.rb(h.cur), fb.ra(nxt), fb.rb(nxt), nullptr,
                         h.rp_ok ? fb.rp(h.cur) : nullptr, h.rp_ok && interior ? fb.rp(h.cur) : nullptr, fb.rp(nxt),
                         &wrote, c->tuning, c->stream, nullptr, nullptr,
                         // background tiles (restir_render's MissTiles): every ring pixel holds its owner's value, which
                         // for a background tile is the known one
                         MissTiles{h.tmiss, (!h.f.unbiased || h.pass == 0) ? h.f.M : 0u, 0u}));
    rp_written = rp_written && wrote;
    return RESTIR_OK;
}

static restir_status halo_interior_locked(restir_ctx* c) {
    auto& h = c->halo;
    if (!h.active || h.pass >= h.passes || h.interior_done)
        return fail(RESTIR_ERR_STATE, "restir_halo_spatial_interior: no pass pending");
    HIP_TRY(hipSetDevice(c->device));
    const HaloSplit hs = halo_split(h.owned, h.f.R);
    h.part_rp = true;
    if (hs.part[0].rw && hs.part[0].rh) ST_TRY(halo_spatial_part(c, hs.part[0], true, h.part_rp));
    h.interior_done = true;
    return RESTIR_OK;
}

static restir_status halo_border_locked(restir_ctx* c) {
    auto& h = c->halo;
    if (!h.active || h.pass >= h.passes || !h.interior_done)
        return fail(RESTIR_ERR_STATE, "restir_halo_spatial_border before the pass's interior");
    HIP_TRY(hipSetDevice(c->device));
    const HaloSplit hs = halo_split(h.owned, h.f.R);
    for (uint32_t i = 1; i <= hs.nb; i++) ST_TRY(halo_spatial_part(c, hs.part[i], false, h.part_rp));
    h.rp_ok = h.part_rp;
    h.cur ^= 1;
    h.pass++;
    h.interior_done = false;
    return RESTIR_OK;
}

restir_status restir_halo_spatial_interior(restir_ctx* c) {
    if (!c) return fail(RESTIR_ERR_INVALID, "ctx is NULL");
    std::lock_guard<std::mutex> lk(c->mu);
    return halo_interior_locked(c);
}

restir_status restir_halo_spatial_border(restir_ctx* c) {
    if (!c) return fail(RESTIR_ERR_INVALID, "ctx is NULL");
    std::lock_guard<std::mutex> lk(c->mu);
    return halo_border_locked(c);
}

restir_status restir_halo_spatial(restir_ctx* c) {
    if (!c) return fail(RESTIR_ERR_INVALID, "ctx is NULL");
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->halo.interior_done) ST_TRY(halo_interior_locked(c));
    return halo_border_locked(c);
}

// ---- native RCCL transport ----------------------------------------------------------------------------
}  // extern "C"

namespace {
struct RcclApi {
    bool ok = false;
    std::string why;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    decltype(&ncclCommCount) comm_count = nullptr;
    decltype(&ncclCommUserRank) comm_user_rank = nullptr;
};

const RcclApi& rccl_api() {
    static RcclApi api = [] {
        RcclApi a;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) { a.why = dlerror() ? dlerror() : "librccl.so.1 not found"; return a; }
        bool all = true;
        auto sym = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            all = all && fn != nullptr;
        };
        sym(a.get_unique_id, "ncclGetUniqueId");
        sym(a.comm_init_rank, "ncclCommInitRank");
        sym(a.comm_destroy, "ncclCommDestroy");
        sym(a.send, "ncclSend");
        sym(a.recv, "ncclRecv");
        sym(a.group_start, "ncclGroupStart");
        sym(a.group_end, "ncclGroupEnd");
        sym(a.error_string, "ncclGetErrorString");
        sym(a.comm_count, "ncclCommCount");
        sym(a.comm_user_rank, "ncclCommUserRank");
        a.ok = all;
        if (!all) a.why = "librccl lacks a symbol";
        return a;
    }();
    return api;
}
}  // namespace

extern "C" {

#define RCCL_TRY(expr)                                                                                            \
    do {                                                                                                          \
        const ncclResult_t rc_ = (expr);                                                                          \
        if (rc_ != ncclSuccess)                                                                                   \
            return fail(RESTIR_ERR_COMM, "%s: %s", #expr, rccl_api().error_string(rc_));                           \
    } while (0)

// inside an open ncclGroupStart: close the group before reporting the error, so the thread's RCCL group state
// does not leak into the next call
#define RCCL_GROUP_TRY(expr)                                                                                      \
    do {                                                                                                          \
        const ncclResult_t rc_ = (expr);                                                                          \
        if (rc_ != ncclSuccess) {                                                                                 \
            (void)rccl_api().group_end();                                                                         \
            return fail(RESTIR_ERR_COMM, "%s: %s", #expr, rccl_api().error_string(rc_));                           \
        }                                                                                                         \
    } while (0)

static void release_rccl(restir_ctx* c) {
    auto& q = c->rccl;
    // the context stream may still hold an unpack that waits on the transfer, and the communication stream the
    // transfer itself: drain both before the communicator and the streams go
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (q.stream) (void)hipStreamSynchronize(q.stream);
    if (q.comm && q.owned && rccl_api().ok) (void)rccl_api().comm_destroy(static_cast<ncclComm_t>(q.comm));
    q.comm = nullptr;
    q.owned = false;
    if (q.packed) (void)hipEventDestroy(q.packed);
    if (q.moved) (void)hipEventDestroy(q.moved);
    if (q.stream) (void)hipStreamDestroy(q.stream);
    q.packed = q.moved = nullptr;
    q.stream = nullptr;
    q.nranks = 0;
    q.rank = -1;
    q.send.release();
    q.recv.release();
}

// the communication stream and the pass's two events (a communicator's, or a record-only pass's)
static restir_status comm_stream_locked(restir_ctx* c) {
    auto& q = c->rccl;
    if (!q.stream) HIP_TRY(hipStreamCreateWithFlags(&q.stream, hipStreamNonBlocking));
    if (!q.packed) HIP_TRY(hipEventCreateWithFlags(&q.packed, hipEventDisableTiming));
    if (!q.moved) HIP_TRY(hipEventCreateWithFlags(&q.moved, hipEventDisableTiming));
    return RESTIR_OK;
}

static restir_status attach_comm_locked(restir_ctx* c, void* comm, bool owned) {
    auto& q = c->rccl;
    ST_TRY(comm_stream_locked(c));
    if (q.comm && q.owned) RCCL_TRY(rccl_api().comm_destroy(static_cast<ncclComm_t>(q.comm)));
    q.comm = comm;
    q.owned = owned;
    int n = 0, r = -1;
    RCCL_TRY(rccl_api().comm_count(static_cast<ncclComm_t>(comm), &n));
    RCCL_TRY(rccl_api().comm_user_rank(static_cast<ncclComm_t>(comm), &r));
    q.nranks = n;
    q.rank = r;
    c->halo_record = false;   // a communicator ends record-only mode: its passes move real reservoirs
    c->halo_log.clear();
    return RESTIR_OK;
}

restir_status restir_rccl_unique_id(void* out, size_t bytes) {
    if (!out || bytes < RESTIR_RCCL_ID_BYTES) return fail(RESTIR_ERR_INVALID, "restir_rccl_unique_id: need %u bytes", RESTIR_RCCL_ID_BYTES);
    static_assert(sizeof(ncclUniqueId) == RESTIR_RCCL_ID_BYTES, "ncclUniqueId size");
    const RcclApi& api = rccl_api();
    if (!api.ok) return fail(RESTIR_ERR_UNSUPPORTED, "RCCL unavailable: %s", api.why.c_str());
    ncclUniqueId id;
    RCCL_TRY(api.get_unique_id(&id));
    std::memcpy(out, &id, sizeof(id));
    return RESTIR_OK;
}

restir_status restir_halo_attach_rccl(restir_ctx* c, const void* unique_id, uint32_t nranks, uint32_t rank) {
    if (!c || !unique_id || nranks == 0 || rank >= nranks) return fail(RESTIR_ERR_INVALID, "restir_halo_attach_rccl: bad argument");
    const RcclApi& api = rccl_api();
    if (!api.ok) return fail(RESTIR_ERR_UNSUPPORTED, "RCCL unavailable: %s", api.why.c_str());
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof(id));
    ncclComm_t comm = nullptr;
    RCCL_TRY(api.comm_init_rank(&comm, (int)nranks, id, (int)rank));
    return attach_comm_locked(c, comm, true);
}

restir_status restir_halo_attach_comm(restir_ctx* c, void* nccl_comm) {
    if (!c || !nccl_comm) return fail(RESTIR_ERR_INVALID, "restir_halo_attach_comm: null argument");
    const RcclApi& api = rccl_api();
    if (!api.ok) return fail(RESTIR_ERR_UNSUPPORTED, "RCCL unavailable: %s", api.why.c_str());
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    return attach_comm_locked(c, nccl_comm, false);
}

restir_status restir_halo_pass(restir_ctx* c) {
    if (!c) return fail(RESTIR_ERR_INVALID, "ctx is NULL");
    std::lock_guard<std::mutex> lk(c->mu);
    auto& h = c->halo;
    auto& q = c->rccl;
    const bool rec = c->halo_record;
    if (!q.comm && !rec) return fail(RESTIR_ERR_STATE, "restir_halo_pass before restir_halo_attach_rccl / _comm");
    if (!h.active || h.pass >= h.passes || h.interior_done) return fail(RESTIR_ERR_STATE, "restir_halo_pass: no pass pending");
    // the plan's peers are tile ranks: the communicator must hold exactly the tiles, with this context's tile at
    // its own rank, or the halos would go to the wrong peers
    if (!rec && (q.nranks != (int)h.nranks || q.rank != (int)h.rank))
        return fail(RESTIR_ERR_INVALID, "restir_halo_pass: communicator rank %d of %d, halo frame is tile %u of %u",
                    q.rank, q.nranks, h.rank, h.nranks);
    for (uint32_t i = 0; i < h.nops; i++)
        if (h.ops[i].peer >= h.nranks || h.ops[i].peer == h.rank)
            return fail(RESTIR_ERR_INVALID, "restir_halo_pass: operation %u peer %u outside the %u tiles", i, h.ops[i].peer,
                        h.nranks);
    HIP_TRY(hipSetDevice(c->device));
    ST_TRY(comm_stream_locked(c));
    ST_TRY(q.send.ensure(std::max<uint64_t>(h.send_bytes, 16)));
    ST_TRY(q.recv.ensure(std::max<uint64_t>(h.recv_bytes, 16)));
    const uint32_t pass = h.pass;
    auto log = [&](uint32_t what, uint32_t stream, uint32_t peer = 0, uint64_t off = 0, uint64_t bytes = 0) {
        if (rec) c->halo_log.push_back(restir_halo_event{what, stream, peer, pass, off, bytes});
    };
    const FrameBufs fb{c, h.fb_records, (size_t)h.view.vw * h.view.vh, h.f.N};
    // context stream: pack (after the previous pass's transfer released the send buffer -- stream order:
    // the previous pass waited on q.moved before its unpack)
    HIP_TRY(launch_halo_pack(h.view, h.send, h.f.N, fb.ra(h.cur), fb.rb(h.cur), q.send.as<float4>(), c->stream));
    log(RESTIR_HALO_EV_PACK, 0, 0, 0, h.send_bytes);
    HIP_TRY(hipEventRecord(q.packed, c->stream));
    log(RESTIR_HALO_EV_RECORD, 0, 0);
    // communication stream: the grouped point-to-point transfer of every plan segment (restir_halo_ops' list)
    HIP_TRY(hipStreamWaitEvent(q.stream, q.packed, 0));
    log(RESTIR_HALO_EV_WAIT, 1, 0);
    if (h.nops) {
        if (rec) {   // nothing moves: a zeroed receive buffer stands in for the transfer
            HIP_TRY(hipMemsetAsync(q.recv.p, 0, h.recv_bytes, q.stream));
        } else {
            RCCL_TRY(rccl_api().group_start());
        }
        log(RESTIR_HALO_EV_GROUP_START, 1);
        const ncclComm_t comm = static_cast<ncclComm_t>(q.comm);
        for (uint32_t i = 0; i < h.nops; i++) {
            const restir_halo_op& o = h.ops[i];
            if (o.kind == RESTIR_HALO_OP_SEND) {
                if (!rec) RCCL_GROUP_TRY(rccl_api().send(static_cast<const char*>(q.send.p) + o.offset, o.bytes, ncclUint8,
                                                         (int)o.peer, comm, q.stream));
                log(RESTIR_HALO_EV_SEND, 1, o.peer, o.offset, o.bytes);
            } else {
                if (!rec) RCCL_GROUP_TRY(rccl_api().recv(static_cast<char*>(q.recv.p) + o.offset, o.bytes, ncclUint8,
                                                         (int)o.peer, comm, q.stream));
                log(RESTIR_HALO_EV_RECV, 1, o.peer, o.offset, o.bytes);
            }
        }
        if (!rec) RCCL_TRY(rccl_api().group_end());
        log(RESTIR_HALO_EV_GROUP_END, 1);
    }
    HIP_TRY(hipEventRecord(q.moved, q.stream));
    log(RESTIR_HALO_EV_RECORD, 1, 1);
    // context stream: the interior overlaps the transfer; unpack + border strips after it
    ST_TRY(halo_interior_locked(c));
    log(RESTIR_HALO_EV_INTERIOR, 0);
    HIP_TRY(hipStreamWaitEvent(c->stream, q.moved, 0));
    log(RESTIR_HALO_EV_WAIT, 0, 1);
    HIP_TRY(launch_halo_unpack(h.view, h.recv, h.f.N, q.recv.as<float4>(), fb.ra(h.cur), fb.rb(h.cur), c->stream));
    log(RESTIR_HALO_EV_UNPACK, 0, 0, 0, h.recv_bytes);
    ST_TRY(halo_border_locked(c));
    log(RESTIR_HALO_EV_BORDER, 0);
    return RESTIR_OK;
}

restir_status restir_halo_record(restir_ctx* c, int on) {
    if (!c) return fail(RESTIR_ERR_INVALID, "ctx is NULL");
    std::lock_guard<std::mutex> lk(c->mu);
    c->halo_record = on != 0;
    c->halo_log.clear();
    return RESTIR_OK;
}

restir_status restir_halo_log(restir_ctx* c, restir_halo_event* out, uint32_t* count) {
    if (!c || !count || (*count && !out)) return fail(RESTIR_ERR_INVALID, "restir_halo_log: null argument");
    std::lock_guard<std::mutex> lk(c->mu);
    const size_t n = c->halo_log.size();
    if (*count < n) {
        *count = (uint32_t)n;
        return fail(RESTIR_ERR_INVALID, "restir_halo_log: capacity for %zu entries needed", n);
    }
    std::copy(c->halo_log.begin(), c->halo_log.end(), out);
    *count = (uint32_t)n;
    c->halo_log.clear();
    return RESTIR_OK;
}

restir_status restir_halo_end(restir_ctx* c, restir_frame** out_next, float* out_rgb) {
    if (!c) return fail(RESTIR_ERR_INVALID, "ctx is NULL");
    if (out_next) *out_next = nullptr;
    std::lock_guard<std::mutex> lk(c->mu);
    auto& h = c->halo;
    if (!h.active || h.pass != h.passes)
        return fail(RESTIR_ERR_STATE, "restir_halo_end after %u of %u spatial passes", h.pass, h.passes);
    HIP_TRY(hipSetDevice(c->device));
    const FrameBufs fb{c, h.fb_records, (size_t)h.view.vw * h.view.vh, h.f.N};
    SceneDev sd;
    ST_TRY(scene_for(c, h.f, (size_t)h.view.vw * h.view.vh, sd));
    TIMED(c, RESTIR_K_FINAL, launch_final(sd, h.owned, h.f, h.camd.origin, fb.nt(h.cur), c->p_mat.as<float4>(),
                                          fb.ra(h.cur), fb.rb(h.cur), c->rgb.as<float>(), c->tuning, c->stream, nullptr,
                                          MissTiles{h.tmiss, 0u, 0u}));
    c->cur = h.cur;
    h.active = false;
    if (out_next) {
        restir_frame* fr = make_frame(c->pool, c->device, c->stream);
        fr->W = h.W; fr->H = h.H; fr->vx0 = h.view.vx0; fr->vy0 = h.view.vy0; fr->vw = h.view.vw; fr->vh = h.view.vh;
        fr->N = h.f.N;
        std::swap(fr->rec, c->rec[h.cur]);
        fr->records = h.fb_records;
        *out_next = fr;
    }
    if (out_rgb) {
        HIP_TRY(hipMemcpyAsync(out_rgb, c->rgb.p, (size_t)h.owned.rw * h.owned.rh * 12, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    return RESTIR_OK;
}

// ---------------------------------------------------------------------------------------------------------
// timing
restir_status restir_enable_timing(restir_ctx* c, int enable) {
    if (!c) return fail(RESTIR_ERR_INVALID, "ctx is NULL");
    std::lock_guard<std::mutex> lk(c->mu);
    c->timing = enable != 0;
    if (c->timing) {
        // the events the timed launches take, created here rather than by the launches themselves: a
        // hipEventCreate costs microseconds of host time inside whatever region is being timed
        HIP_TRY(hipSetDevice(c->device));
        const size_t want = 512;   // bench.py's default timed region (200 frames x 2) without growing; more on demand
        while (c->free_events.size() + c->pending.size() * 2 < want) {
            hipEvent_t e = nullptr;
            HIP_TRY(timing_event_create(c, &e));
            c->free_events.push_back(e);
        }
    }
    return RESTIR_OK;
}

restir_status restir_timings(restir_ctx* c, double* ms, uint64_t* launches) {
    if (!c) return fail(RESTIR_ERR_INVALID, "ctx is NULL");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    ST_TRY(collect_timings(c));
    for (int k = 0; k < RESTIR_K_COUNT; k++) {
        if (ms) ms[k] = c->ms[k];
        if (launches) launches[k] = c->launches[k];
    }
    return RESTIR_OK;
}

restir_status restir_set_tuning(restir_ctx* c, const char* key, int value) {
    if (!c || !key) return fail(RESTIR_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(c->mu);
    Tuning& t = c->tuning;
    const uint32_t v = (uint32_t)value;
    if (!std::strcmp(key, "primary.lds")) t.primary_lds = v;
    else if (!std::strcmp(key, "ris.lds")) t.ris_lds = v;
    else if (!std::strcmp(key, "spatial.xcd_rows")) t.spatial_xcd_rows = v;
    else if (!std::strcmp(key, "spatial.xcd_cols")) t.spatial_xcd_cols = v;
    else if (!std::strcmp(key, "ris.late")) t.ris_late = v;
    else if (!std::strcmp(key, "miss.tiles")) t.miss_tiles = v;
    else if (!std::strcmp(key, "miss.gbuf")) t.miss_gbuf = v;
    else if (!std::strcmp(key, "final.miss")) t.final_miss = v;
    else if (!std::strcmp(key, "spatial.lean")) t.spatial_lean = v;
    else if (!std::strcmp(key, "spatial.th")) { if (v > 2) return fail(RESTIR_ERR_INVALID, "spatial.th: 0 (auto), 1 or 2"); t.spatial_th = v; }
    else if (!std::strcmp(key, "spatial.handles")) t.spatial_handles = v;
    else if (!std::strcmp(key, "spatial.gather")) t.spatial_gather = v;
    else if (!std::strcmp(key, "spatial.n2h")) t.spatial_n2h = v;
    else if (!std::strcmp(key, "fuse.primary_ris")) t.fuse_primary_ris = v;
    else if (!std::strcmp(key, "fuse.temporal")) t.fuse_temporal = v;
    else if (!std::strcmp(key, "timing.mask")) t.timing_mask = v;
    else if (!std::strcmp(key, "timing.every")) { t.timing_every = v ? v : 1u; for (auto& q : c->timing_seq) q = 0; }
    else if (!std::strcmp(key, "timing.fence")) {
        // the pooled events carry the old flags: drop the free ones (recreated on demand)
        if (t.timing_fence != v) {
            HIP_TRY(hipSetDevice(c->device));
            ST_TRY(collect_timings(c));   // pending pairs return to the pool first
            for (hipEvent_t e : c->free_events) (void)hipEventDestroy(e);
            c->free_events.clear();
        }
        t.timing_fence = v;
    }
    else if (!std::strcmp(key, "ris.compact")) t.ris_compact = v;
    else if (!std::strcmp(key, "bvh.max_leaf")) t.bvh_max_leaf = v;
    else if (!std::strcmp(key, "final.sort")) t.final_sort = v;
    else if (!std::strcmp(key, "final.qbvh")) t.final_qbvh = v;
    else if (!std::strcmp(key, "primary.tl")) t.primary_tl = v;
    else if (!std::strcmp(key, "mis.chunk")) t.mis_chunk = v;   // applies from the next ensure_mis
    else if (!std::strcmp(key, "layout.records")) t.records = v;   // frame-path buffer layout
    else if (!std::strcmp(key, "final.lds")) t.final_lds = v;
    else return fail(RESTIR_ERR_INVALID, "unknown tuning key '%s'", key);
    return RESTIR_OK;
}

restir_status restir_reset_timings(restir_ctx* c) {
    if (!c) return fail(RESTIR_ERR_INVALID, "ctx is NULL");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    ST_TRY(collect_timings(c));
    for (int k = 0; k < RESTIR_K_COUNT; k++) { c->ms[k] = 0.0; c->launches[k] = 0; }
    return RESTIR_OK;
}

}  // extern "C"

// restir.hpp -- header-only C++ wrapper over the C ABI (include/restir_c.h) that keeps the reference's
// render surface:
//
//   reference  ReservoirGrid renderReSTIR(std::shared_ptr<ReservoirGrid> previousFrameGrid, const Scene&,
//                                         const Trackball&, const EmbreeInterface&, Screen&, const Features&)
//              (src/rendering/render.h:25-28, render.cpp:28-62)
//   here       std::shared_ptr<ReservoirGrid> romis::renderReSTIR(Renderer&, std::shared_ptr<ReservoirGrid> prev,
//                                         const Camera&, Screen&, const Features&)
//
// Errors throw romis::RestirError (a std::runtime_error, as render.cpp:99/278 do).  The grid stays on the GPU
// (a reference-counted device handle, the replacement for the caller's std::shared_ptr<ReservoirGrid>).
// The Scene / EmbreeInterface pair becomes Renderer::setScene (uploads materials, lights and the BVH once).
#pragma once

#include <ctime>
#include <filesystem>
#include <fstream>
#include <iomanip>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../restir_c.h"

namespace romis {

struct RestirError : std::runtime_error {
    explicit RestirError(const std::string& what) : std::runtime_error(what) {}
};

inline void check(restir_status s, const char* what) {
    if (s != RESTIR_OK) throw RestirError(std::string(what) + ": " + restir_last_error());
}

// struct Features (src/utils/common.h:89-136): the fields the ReSTIR path reads.
struct Features : restir_features {
    Features() { restir_features_default(this); }
};

// The reference's own struct Features (src/utils/common.h:89-136) -> Features, field by field by the reference's
// member names (any type with those members works, so the reference's header is not needed here).  The enums
// keep their values: RayTraceMode {ReSTIR, RMIS, ROMIS} (common.h:25-29) = restir_mode,
// NeighbourSelectionStrategy (common.h:36-41) = restir_neighbour_strategy, MISWeightRMIS (common.h:31-34) =
// restir_mis_weight.  Fields off the path (enableRecursive, enableHardShadow, maxReflectionRecursion, ...) are
// not read by renderReSTIR / renderRMIS / renderROMIS and have no counterpart.
template <class RefFeatures>
Features fromReferenceFeatures(const RefFeatures& rf) {
    Features f;
    f.ray_trace_mode = static_cast<uint32_t>(rf.rayTraceMode);
    f.initial_light_samples = rf.initialLightSamples;
    f.num_samples_in_reservoir = rf.numSamplesInReservoir;
    f.num_neighbours_to_sample = rf.numNeighboursToSample;
    f.spatial_resample_radius = rf.spatialResampleRadius;
    f.spatial_resampling_passes = rf.spatialResamplingPasses;
    f.temporal_clamp_m = rf.temporalClampM;
    f.initial_samples_visibility_check = rf.initialSamplesVisibilityCheck ? 1 : 0;
    f.unbiased_combination = rf.unbiasedCombination ? 1 : 0;
    f.spatial_reuse = rf.spatialReuse ? 1 : 0;
    f.spatial_reuse_visibility_check = rf.spatialReuseVisibilityCheck ? 1 : 0;
    f.temporal_reuse = rf.temporalReuse ? 1 : 0;
    f.enable_shading = rf.enableShading ? 1 : 0;
    f.enable_texture_mapping = rf.enableTextureMapping ? 1 : 0;
    f.enable_tone_mapping = rf.enableToneMapping ? 1 : 0;
    f.gamma = rf.gamma;
    f.exposure = rf.exposure;
    f.neighbour_same_geometry = rf.neighbourSameGeometry ? 1 : 0;
    f.use_progressive_romis = rf.useProgressiveROMIS ? 1 : 0;
    f.save_alphas_visualisation = rf.saveAlphasVisualisation ? 1 : 0;
    f.neighbour_max_depth_difference_fraction = rf.neighbourMaxDepthDifferenceFraction;
    f.neighbour_max_normal_angle_difference_radians = rf.neighbourMaxNormalAngleDifferenceRadians;
    f.max_iterations_mis = rf.maxIterationsMIS;
    f.neighbour_selection_strategy = static_cast<uint32_t>(rf.neighbourSelectionStrategy);
    f.mis_weight_rmis = static_cast<uint32_t>(rf.misWeightRMIS);
    f.progressive_update_mod = rf.progressiveUpdateMod;
    return f;
}

// Trackball state after Trackball(window, glm::radians(fov), dist) + setCamera(lookAt, glm::radians(rot), dist)
struct Camera : restir_camera {
    Camera() : restir_camera{} {}
    static Camera fromDegrees(float fovDeg, float aspect, const float lookAt[3], float dist, const float rotDeg[3]) {
        constexpr float rad = 0.01745329251994329576923690768489f;   // glm::radians
        Camera c;
        c.fovy = fovDeg * rad;
        c.aspect = aspect;
        for (int i = 0; i < 3; i++) { c.look_at[i] = lookAt[i]; c.rotation[i] = rotDeg[i] * rad; }
        c.distance = dist;
        return c;
    }
};

// One mesh of the Scene (framework/include/framework/mesh.h:36-43) as flat arrays.
struct Mesh {
    std::vector<float> positions;    // 3 per vertex
    std::vector<float> normals;      // 3 per vertex
    std::vector<uint32_t> triangles; // 3 per triangle
    restir_material material{};
};

struct Scene {
    std::vector<Mesh> meshes;
    std::vector<restir_light> lights;   // Point / Segment / Parallelogram (common.h:72-87)
};

// Screen (src/rendering/screen.h): float RGB, row 0 = top, as Screen::setPixel stores it (screen.cpp:37-43).
struct Screen {
    int width = 0, height = 0;
    std::vector<float> rgb;
    Screen(int w, int h) : width(w), height(h), rgb(size_t(w) * size_t(h) * 3, 0.0f) {}
    float* pixel(int x, int yFromTop) { return &rgb[(size_t(yFromTop) * width + x) * 3]; }
    // Screen::writeBitmapToFile (screen.cpp:45-56): clamp, x255, truncate, stbi_write_bmp byte for byte
    void writeBitmapToFile(const std::filesystem::path& filePath) const {
        check(restir_write_bmp(filePath.string().c_str(), rgb.data(), uint32_t(width), uint32_t(height)),
              "restir_write_bmp");
    }
};

// The configuration record renderRayTraced saves per render (render.cpp:281-287): <dir>/<currentTime()>.json,
// currentTime() = "%d-%m-%Y %H-%M-%S" local time (utils.cpp:16-22), cereal's bytes (restir_features_json).
inline std::filesystem::path saveFeaturesRecord(const restir_features& features, const std::filesystem::path& dir,
                                                const restir_features_record_extra* extra = nullptr) {
    size_t n = 0;
    check(restir_features_json(&features, extra, nullptr, 0, &n), "restir_features_json");
    std::string json(n + 1, '\0');
    check(restir_features_json(&features, extra, json.data(), json.size(), &n), "restir_features_json");
    json.resize(n);
    if (!std::filesystem::exists(dir)) std::filesystem::create_directory(dir);
    const std::time_t t = std::time(nullptr);
    std::ostringstream name;
    name << std::put_time(std::localtime(&t), "%d-%m-%Y %H-%M-%S") << ".json";
    const std::filesystem::path path = dir / name.str();
    std::ofstream out(path, std::ios::binary);
    out << json;
    if (!out) throw RestirError("saveFeaturesRecord: cannot write " + path.string());
    return path;
}

// One sub-reservoir's state as reservoir.h:18-32 keeps it: outputSamples[j] = {position, color, W},
// sampleNums[j] = M.
struct ReservoirSample {
    float position[3], color[3], W;
    uint32_t M;
};

// Device-resident ReservoirGrid (reservoir.h:75).
class ReservoirGrid {
public:
    explicit ReservoirGrid(restir_frame* f) : frame_(f) {}
    ~ReservoirGrid() { restir_frame_release(frame_); }
    ReservoirGrid(const ReservoirGrid&) = delete;
    ReservoirGrid& operator=(const ReservoirGrid&) = delete;
    restir_frame* handle() const { return frame_; }
    // host copy, [N][vh][vw] (rows y = 0 bottom): the per-pixel state renderReSTIR returns (render.cpp:61)
    std::vector<ReservoirSample> download(uint32_t* n = nullptr, uint32_t* vw = nullptr, uint32_t* vh = nullptr) const {
        uint32_t N = 0, w = 0, h = 0;
        check(restir_frame_info(frame_, nullptr, nullptr, nullptr, nullptr, &w, &h, &N), "restir_frame_info");
        const size_t cnt = size_t(N) * w * h;
        std::vector<float> pos(3 * cnt), col(3 * cnt), W(cnt);
        std::vector<uint32_t> M(cnt);
        check(restir_frame_download(frame_, pos.data(), col.data(), W.data(), M.data()), "restir_frame_download");
        std::vector<ReservoirSample> out(cnt);
        for (size_t i = 0; i < cnt; i++) {
            for (int a = 0; a < 3; a++) { out[i].position[a] = pos[3 * i + a]; out[i].color[a] = col[3 * i + a]; }
            out[i].W = W[i];
            out[i].M = M[i];
        }
        if (n) *n = N;
        if (vw) *vw = w;
        if (vh) *vh = h;
        return out;
    }

private:
    restir_frame* frame_;
};

// Owns a HIP device context: the EmbreeInterface + OpenMP loops of the reference become this object.
class Renderer {
public:
    explicit Renderer(int device = 0) { check(restir_create(device, &ctx_), "restir_create"); }
    ~Renderer() { restir_destroy(ctx_); }
    Renderer(const Renderer&) = delete;
    Renderer& operator=(const Renderer&) = delete;

    void setScene(const Scene& scene) {
        std::vector<restir_mesh> m(scene.meshes.size());
        for (size_t i = 0; i < m.size(); i++) {
            const Mesh& src = scene.meshes[i];
            m[i].positions = src.positions.data();
            m[i].normals = src.normals.data();
            m[i].num_vertices = uint32_t(src.positions.size() / 3);
            m[i].triangles = src.triangles.data();
            m[i].num_triangles = uint32_t(src.triangles.size() / 3);
            m[i].material = src.material;
        }
        check(restir_set_scene(ctx_, m.data(), uint32_t(m.size()), scene.lights.data(), uint32_t(scene.lights.size())),
              "restir_set_scene");
    }
    void setSeed(uint32_t seed, uint32_t frameIndex = 0) { check(restir_set_seed(ctx_, seed, frameIndex), "restir_set_seed"); }
    // RENDERS_DIR for the file side outputs the library writes itself (R-OMIS alpha visualisation); empty = none
    void setRendersDir(const std::filesystem::path& dir) {
        check(restir_set_renders_dir(ctx_, dir.empty() ? nullptr : dir.c_str()), "restir_set_renders_dir");
        rendersDir_ = dir;
    }
    const std::filesystem::path& rendersDir() const { return rendersDir_; }
    restir_ctx* handle() const { return ctx_; }

private:
    restir_ctx* ctx_ = nullptr;
    std::filesystem::path rendersDir_;
};

// Contexts for callers that render concurrently: the reference's CLI renders one std::thread per camera through
// renderRayTraced with a shared Scene and EmbreeInterface (main.cpp:213-230).  Each calling thread gets its own
// Renderer -- its own HIP stream, buffers and scene upload -- created on first use, so the threads never
// serialise on one context's mutex, and each camera keeps its own previous-frame grid (the caller's
// std::shared_ptr<ReservoirGrid>, as in the reference).  Thread-safe.
class RendererPool {
public:
    RendererPool(int device, Scene scene, uint32_t seed = RESTIR_DEFAULT_SEED)
        : device_(device), scene_(std::move(scene)), seed_(seed) {}
    RendererPool(const RendererPool&) = delete;
    RendererPool& operator=(const RendererPool&) = delete;
    // this thread's renderer (frame index 0 at creation, advancing by one per render)
    Renderer& local() {
        std::lock_guard<std::mutex> lk(mu_);
        std::unique_ptr<Renderer>& r = per_thread_[std::this_thread::get_id()];
        if (!r) {
            r = std::make_unique<Renderer>(device_);
            r->setScene(scene_);
            r->setSeed(seed_, 0);
        }
        return *r;
    }

private:
    int device_;
    Scene scene_;
    uint32_t seed_;
    std::mutex mu_;
    std::map<std::thread::id, std::unique_ptr<Renderer>> per_thread_;
};

// renderReSTIR (render.cpp:28-62): primary hits, initial RIS, [temporal if prev], [spatial x passes], final
// shading + tone mapping into `screen`; returns the frame's final grid for the next frame's temporal reuse.
inline std::shared_ptr<ReservoirGrid> renderReSTIR(Renderer& r, const std::shared_ptr<ReservoirGrid>& prev,
                                                   const Camera& camera, Screen& screen, const Features& features) {
    restir_frame* next = nullptr;
    check(restir_render(r.handle(), &camera, &features, uint32_t(screen.width), uint32_t(screen.height), nullptr,
                        prev ? prev->handle() : nullptr, &next, screen.rgb.data()),
          "restir_render");
    return std::make_shared<ReservoirGrid>(next);
}

// renderRMIS / renderROMIS (render.cpp:64-265): maxIterationsMIS rounds of initial samples combined over each
// pixel's neighbourhood into `screen` (features.ray_trace_mode selects the estimator).
inline void renderMIS(Renderer& r, const Camera& camera, Screen& screen, const Features& features) {
    check(restir_render(r.handle(), &camera, &features, uint32_t(screen.width), uint32_t(screen.height), nullptr, nullptr,
                        nullptr, screen.rgb.data()),
          "restir_render");
}

// renderRayTraced (render.cpp:268-290): the grid for temporal reuse in ReSTIR mode, nullptr (std::nullopt) for
// R-MIS / R-OMIS.  Like the reference, every render then saves its configuration record to
// <rendersDir>/<currentTime()>.json (render.cpp:281-287, saveFeaturesRecord), and R-OMIS with
// saveAlphasVisualisation writes its alpha bitmaps to <rendersDir>/<currentTime()>/ after every iteration; the
// reference's RENDERS_DIR is a build-time constant, here the caller passes it.  A non-empty rendersDir applies to
// this render only (the Renderer's own setRendersDir is restored afterwards); an empty one writes no record and
// leaves the alpha bitmaps to whatever the Renderer was given with setRendersDir.
inline std::shared_ptr<ReservoirGrid> renderRayTraced(Renderer& r, const std::shared_ptr<ReservoirGrid>& prev,
                                                      const Camera& camera, Screen& screen, const Features& features,
                                                      const std::filesystem::path& rendersDir = {},
                                                      const restir_features_record_extra* extra = nullptr) {
    std::shared_ptr<ReservoirGrid> next;
    // R-OMIS's per-iteration alpha visualisation (render.cpp:227-229) goes to rendersDir for this call
    struct DirScope {
        Renderer& r;
        std::filesystem::path saved;
        bool set;
        DirScope(Renderer& rr, const std::filesystem::path& d) : r(rr), saved(rr.rendersDir()), set(!d.empty()) {
            if (set) r.setRendersDir(d);
        }
        ~DirScope() {
            if (!set) return;
            try { r.setRendersDir(saved); } catch (...) {}   // never throws from a destructor
        }
    } scope(r, rendersDir);
    switch (features.ray_trace_mode) {
        case RESTIR_MODE_RESTIR: next = renderReSTIR(r, prev, camera, screen, features); break;
        case RESTIR_MODE_RMIS:
        case RESTIR_MODE_ROMIS: renderMIS(r, camera, screen, features); break;
        default: throw RestirError("Unsupported ray-tracing render mode requested from entry point");
    }
    if (!rendersDir.empty()) saveFeaturesRecord(features, rendersDir, extra);
    return next;
}
// ... from any thread: the calling thread's context of the pool
inline std::shared_ptr<ReservoirGrid> renderRayTraced(RendererPool& pool, const std::shared_ptr<ReservoirGrid>& prev,
                                                      const Camera& camera, Screen& screen, const Features& features,
                                                      const std::filesystem::path& rendersDir = {},
                                                      const restir_features_record_extra* extra = nullptr) {
    return renderRayTraced(pool.local(), prev, camera, screen, features, rendersDir, extra);
}

}  // namespace romis

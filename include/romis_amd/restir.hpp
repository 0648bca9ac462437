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

#include <memory>
#include <stdexcept>
#include <string>
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
};

// Device-resident ReservoirGrid (reservoir.h:75).
class ReservoirGrid {
public:
    explicit ReservoirGrid(restir_frame* f) : frame_(f) {}
    ~ReservoirGrid() { restir_frame_release(frame_); }
    ReservoirGrid(const ReservoirGrid&) = delete;
    ReservoirGrid& operator=(const ReservoirGrid&) = delete;
    restir_frame* handle() const { return frame_; }

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
    restir_ctx* handle() const { return ctx_; }

private:
    restir_ctx* ctx_ = nullptr;
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
// R-MIS / R-OMIS.
inline std::shared_ptr<ReservoirGrid> renderRayTraced(Renderer& r, const std::shared_ptr<ReservoirGrid>& prev,
                                                      const Camera& camera, Screen& screen, const Features& features) {
    switch (features.ray_trace_mode) {
        case RESTIR_MODE_RESTIR: return renderReSTIR(r, prev, camera, screen, features);
        case RESTIR_MODE_RMIS:
        case RESTIR_MODE_ROMIS: renderMIS(r, camera, screen, features); return nullptr;
        default: throw RestirError("Unsupported ray-tracing render mode requested from entry point");
    }
}

}  // namespace romis

// Drives the C++ wrapper (include/romis_amd/restir.hpp) the way the reference's CLI drives renderRayTraced
// (src/main.cpp:213-230): load a scene, render `frames` frames threading the previous grid, write the last
// frame's RGB.  Used by tests/test_cpp_wrapper.py (compiled on CPU; run on the GPU box).
//
//   render_scene <scene.bin> <out.rgb> <width> <height> <frames> <N> <passes> <temporal> [mode] [renders_dir]
//
// mode: 0 ReSTIR (default), 1 R-MIS, 2 R-OMIS (Features::rayTraceMode, common.h:15).  renders_dir: every render
// saves its Features record there (render.cpp:281-287).
//
// scene.bin (little endian): u32 num_meshes; per mesh: u32 V, u32 T, f32[3V] positions, f32[3V] normals,
// u32[3T] triangles, f32[8] material (kd3 ks3 shininess transparency); u32 num_lights, restir_light[L];
// f32[9] camera (fovy aspect lookAt3 distance rotation3).
#include "scene_io.h"

#include <vector>

int main(int argc, char** argv) {
    if (argc < 9) { std::fprintf(stderr, "usage: %s scene.bin out.rgb W H frames N passes temporal\n", argv[0]); return 2; }
    const int W = std::atoi(argv[3]), H = std::atoi(argv[4]), frames = std::atoi(argv[5]);
    romis::Camera camera;
    romis::Scene scene = read_scene(argv[1], &camera);

    romis::Features features;
    features.num_samples_in_reservoir = uint32_t(std::atoi(argv[6]));
    features.spatial_resampling_passes = uint32_t(std::atoi(argv[7]));
    features.temporal_reuse = uint8_t(std::atoi(argv[8]));
    if (argc > 9) features.ray_trace_mode = uint32_t(std::atoi(argv[9]));
    const std::filesystem::path renders = argc > 10 ? std::filesystem::path(argv[10]) : std::filesystem::path();

    try {
        romis::Renderer renderer(0);
        renderer.setScene(scene);
        renderer.setSeed(RESTIR_DEFAULT_SEED, 0);
        romis::Screen screen(W, H);
        std::shared_ptr<romis::ReservoirGrid> prev;
        for (int i = 0; i < frames; i++) {
            prev = romis::renderRayTraced(renderer, prev, camera, screen, features, renders);
            if (features.ray_trace_mode != RESTIR_MODE_RESTIR && prev) {
                std::fprintf(stderr, "R-MIS / R-OMIS returned a grid\n");
                return 1;
            }
        }
        FILE* o = std::fopen(argv[2], "wb");
        std::fwrite(screen.rgb.data(), sizeof(float), screen.rgb.size(), o);
        std::fclose(o);
        // the reference's error convention: unsupported modes throw (render.cpp:278)
        romis::Features bad = features;
        bad.ray_trace_mode = 7;
        try {
            romis::renderRayTraced(renderer, prev, camera, screen, bad, renders);   // throws before any record
            std::fprintf(stderr, "expected an exception\n");
            return 1;
        } catch (const std::runtime_error&) {
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}

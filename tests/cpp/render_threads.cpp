// The reference CLI's multi-camera layout (src/main.cpp:213-230): one std::thread per camera renders through
// renderRayTraced with a shared scene.  Here each thread renders `frames` temporal frames of its own camera
// through romis::RendererPool (a context per thread) and keeps its own previous-frame grid; the Features come
// from a struct with the reference's member names and defaults (common.h:89-136) via fromReferenceFeatures.
//
//   render_threads <scene.bin> <cameras.bin> <out_prefix> <width> <height> <frames>
//
// cameras.bin: u32 count, then f32[9] per camera (fovy aspect lookAt3 distance rotation3).  Writes
// <out_prefix><i>.rgb (last frame, float RGB, row 0 = top) and <out_prefix><i>.grid (the last frame's grid:
// f32 pos[3n], f32 color[3n], f32 W[n], u32 M[n], n = N * H * W).
#include "scene_io.h"

#include <string>
#include <thread>
#include <vector>

// The reference's Features type as the CLI fills it (test stand-in for src/utils/common.h:89-136: same member
// names and default values; only the members fromReferenceFeatures reads).
namespace ref {
enum class RayTraceMode { ReSTIR = 0, RMIS, ROMIS };
enum class MISWeightRMIS { Equal = 0, Balance };
enum class NeighbourSelectionStrategy { Random = 0, Similar, Dissimilar, EqualSimilarDissimilar };
struct Features {
    bool enableShading = true;
    bool enableTextureMapping = true;
    RayTraceMode rayTraceMode = RayTraceMode::ROMIS;
    bool initialSamplesVisibilityCheck = false;
    uint32_t numSamplesInReservoir = 2U;
    uint32_t initialLightSamples = 32U;
    uint32_t numNeighboursToSample = 5U;
    uint32_t spatialResampleRadius = 10U;
    bool neighbourSameGeometry = true;
    float neighbourMaxDepthDifferenceFraction = 0.10f;
    float neighbourMaxNormalAngleDifferenceRadians = 0.436332f;
    uint32_t maxIterationsMIS = 5U;
    NeighbourSelectionStrategy neighbourSelectionStrategy = NeighbourSelectionStrategy::Similar;
    MISWeightRMIS misWeightRMIS = MISWeightRMIS::Equal;
    bool useProgressiveROMIS = false;
    uint32_t progressiveUpdateMod = 1U;
    bool saveAlphasVisualisation = true;
    bool unbiasedCombination = false;
    bool spatialReuse = true;
    bool spatialReuseVisibilityCheck = false;
    bool temporalReuse = true;
    uint32_t spatialResamplingPasses = 2U;
    uint32_t temporalClampM = 20U;
    bool enableToneMapping = true;
    float gamma = 1.0f;
    float exposure = 1.5f;
};
}  // namespace ref

int main(int argc, char** argv) {
    if (argc < 7) { std::fprintf(stderr, "usage: %s scene.bin cameras.bin out_prefix W H frames\n", argv[0]); return 2; }
    const int W = std::atoi(argv[4]), H = std::atoi(argv[5]), frames = std::atoi(argv[6]);
    romis::Scene scene = read_scene(argv[1], nullptr);
    FILE* cf = std::fopen(argv[2], "rb");
    if (!cf) { std::perror("cameras"); return 2; }
    uint32_t nc = 0;
    rd(cf, &nc, 1);
    std::vector<romis::Camera> cams;
    for (uint32_t i = 0; i < nc; i++) cams.push_back(read_camera(cf));
    std::fclose(cf);

    ref::Features rf;
    rf.rayTraceMode = ref::RayTraceMode::ReSTIR;
    rf.numSamplesInReservoir = 1;
    rf.spatialResamplingPasses = 1;
    const romis::Features features = romis::fromReferenceFeatures(rf);

    romis::RendererPool pool(0, scene);
    std::vector<std::string> errors(nc);
    std::vector<std::thread> workers;
    for (uint32_t i = 0; i < nc; i++) {
        workers.emplace_back([&, i]() {
            try {
                romis::Screen screen(W, H);
                std::shared_ptr<romis::ReservoirGrid> prev;   // this camera's own predecessor
                for (int fr = 0; fr < frames; fr++) prev = romis::renderRayTraced(pool, prev, cams[i], screen, features);
                const std::string base = std::string(argv[3]) + std::to_string(i);
                FILE* o = std::fopen((base + ".rgb").c_str(), "wb");
                std::fwrite(screen.rgb.data(), sizeof(float), screen.rgb.size(), o);
                std::fclose(o);
                const std::vector<romis::ReservoirSample> g = prev->download();
                std::vector<float> pos, col, w;
                std::vector<uint32_t> m;
                for (const romis::ReservoirSample& r : g) {
                    pos.insert(pos.end(), r.position, r.position + 3);
                    col.insert(col.end(), r.color, r.color + 3);
                    w.push_back(r.W);
                    m.push_back(r.M);
                }
                o = std::fopen((base + ".grid").c_str(), "wb");
                std::fwrite(pos.data(), 4, pos.size(), o);
                std::fwrite(col.data(), 4, col.size(), o);
                std::fwrite(w.data(), 4, w.size(), o);
                std::fwrite(m.data(), 4, m.size(), o);
                std::fclose(o);
            } catch (const std::exception& e) {
                errors[i] = e.what();
            }
        });
    }
    for (auto& t : workers) t.join();
    for (uint32_t i = 0; i < nc; i++)
        if (!errors[i].empty()) { std::fprintf(stderr, "camera %u: %s\n", i, errors[i].c_str()); return 1; }
    return 0;
}

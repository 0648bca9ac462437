// screen_ref.cpp -- TEST INFRASTRUCTURE (oracle/_ref only): the reference's own frame-output code paths, to pin
// libromis_amd's restir_encode_bmp / restir_features_json byte for byte (tests/golden/make_screen_fixtures.py).
//   screen_ref bmp W H < rgb.f32 > out.bmp   : Screen::writeBitmapToFile's conversion (screen.cpp:47-51, restated
//                                              here on the reference's glm: screen.cpp itself pulls in OpenGL) fed to
//                                              the reference's vendored stb_image_write (stbi_write_bmp, 4 comp)
//   screen_ref json k=v ...                  : the reference's own struct Features (src/utils/common.h) with the
//                                              given fields set, serialised by its vendored cereal JSONOutputArchive
//                                              exactly as render.cpp:284-286 does
#include <utils/common.h>

#include <glm/common.hpp>
#include <glm/vec3.hpp>
#include <glm/vec4.hpp>
#include <glm/gtc/type_precision.hpp>
#define STB_IMAGE_WRITE_IMPLEMENTATION
#include <stb/stb_image_write.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

static void to_stdout(void*, void* data, int size) { std::fwrite(data, 1, (size_t)size, stdout); }

int main(int argc, char** argv) {
    if (argc >= 4 && !std::strcmp(argv[1], "bmp")) {
        const int W = std::atoi(argv[2]), H = std::atoi(argv[3]);
        std::vector<glm::vec3> tex((size_t)W * H);
        if (std::fread(tex.data(), sizeof(glm::vec3), tex.size(), stdin) != tex.size()) return 2;
        std::vector<glm::u8vec4> data8(tex.size());
        std::transform(std::begin(tex), std::end(tex), std::begin(data8), [](const glm::vec3& color) {
            const glm::vec3 clampedColor = glm::clamp(color, 0.0f, 1.0f);
            return glm::u8vec4(glm::vec4(clampedColor, 1.0f) * 255.0f);
        });
        return stbi_write_bmp_to_func(to_stdout, nullptr, W, H, 4, data8.data()) ? 0 : 3;
    }
    if (argc >= 2 && !std::strcmp(argv[1], "json")) {
        Features f;
        for (int i = 2; i < argc; i++) {
            std::string kv = argv[i];
            const size_t eq = kv.find('=');
            const std::string k = kv.substr(0, eq), v = kv.substr(eq + 1);
            const bool b = v == "1";
            const unsigned u = (unsigned)std::strtoul(v.c_str(), nullptr, 10);
            if (k == "enableShading") f.enableShading = b;
            else if (k == "enableRecursive") f.enableRecursive = b;
            else if (k == "enableHardShadow") f.enableHardShadow = b;
            else if (k == "enableSoftShadow") f.enableSoftShadow = b;
            else if (k == "enableNormalInterp") f.enableNormalInterp = b;
            else if (k == "enableTextureMapping") f.enableTextureMapping = b;
            else if (k == "enableAccelStructure") f.enableAccelStructure = b;
            else if (k == "maxReflectionRecursion") f.maxReflectionRecursion = u;
            else if (k == "rayTraceMode") f.rayTraceMode = static_cast<RayTraceMode>(u);
            else if (k == "initialSamplesVisibilityCheck") f.initialSamplesVisibilityCheck = b;
            else if (k == "numSamplesInReservoir") f.numSamplesInReservoir = u;
            else if (k == "initialLightSamples") f.initialLightSamples = u;
            else if (k == "numNeighboursToSample") f.numNeighboursToSample = u;
            else if (k == "spatialResampleRadius") f.spatialResampleRadius = u;
            else if (k == "maxIterationsMIS") f.maxIterationsMIS = u;
            else if (k == "neighbourSelectionStrategy") f.neighbourSelectionStrategy = static_cast<NeighbourSelectionStrategy>(u);
            else if (k == "misWeightRMIS") f.misWeightRMIS = static_cast<MISWeightRMIS>(u);
            else if (k == "useProgressiveROMIS") f.useProgressiveROMIS = b;
            else if (k == "progressiveUpdateMod") f.progressiveUpdateMod = u;
            else if (k == "saveAlphasVisualisation") f.saveAlphasVisualisation = b;
            else if (k == "unbiasedCombination") f.unbiasedCombination = b;
            else if (k == "spatialReuse") f.spatialReuse = b;
            else if (k == "spatialReuseVisibilityCheck") f.spatialReuseVisibilityCheck = b;
            else if (k == "temporalReuse") f.temporalReuse = b;
            else if (k == "spatialResamplingPasses") f.spatialResamplingPasses = u;
            else if (k == "temporalClampM") f.temporalClampM = u;
            else if (k == "enableToneMapping") f.enableToneMapping = b;
            else if (k == "gamma") { uint32_t bits = u; std::memcpy(&f.gamma, &bits, 4); }
            else if (k == "exposure") { uint32_t bits = u; std::memcpy(&f.exposure, &bits, 4); }
            else { std::fprintf(stderr, "unknown field %s\n", k.c_str()); return 4; }
        }
        {
            cereal::JSONOutputArchive configArchive(std::cout);
            f.serialize(configArchive);
        }
        return 0;
    }
    std::fprintf(stderr, "usage: screen_ref bmp W H < rgb | screen_ref json k=v ...\n");
    return 1;
}

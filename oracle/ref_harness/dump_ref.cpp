// Test-infrastructure harness: links the reference's OWN scene / mesh / tone-mapping translation units,
// compiled unmodified from /root/reference by oracle/Makefile, and dumps what they compute as golden
// fixtures for tests/golden/.  Nothing here is shipped or measured; it only pins the oracle's inputs.
//
//   scenes   : loadScenePrebuilt (src/scene/scene.cpp:68-132) -> loadMesh (framework/src/mesh.cpp:52-148,
//              incl. tinyobj triangulation and centerAndScaleToUnitMesh :150-175) + light lists
//              (regularLightGrid scene.cpp:5-28, constructNightClubLights :30-66)
//   tonemap  : exposureToneMapping (src/post_processing/tone_mapping.cpp:8-11)
//   textures : the Image a textured material carries (framework/src/image.cpp:13-34: stb RGB bytes / 255.0f),
//              as its bytes (the harness checks every texel is exactly byte / 255.0f), and acquireTexel
//              (src/scene/texture.cpp:4-9) on deterministic and edge texture coordinates
//   glm      : the vendored glm 0.9.9.9 primitives the hot path uses (normalize, dot, length, distance, cross,
//              mix, quat(euler) * v) on deterministic inputs, so the C restatement's operation order is pinned.
//
// Floats are written as their IEEE-754 bit patterns (uint32) so the fixtures are bit-exact.
#include <scene/scene.h>
#include <scene/texture.h>
#include <post_processing/tone_mapping.h>
#include <framework/image.h>

#include <glm/glm.hpp>
#include <glm/gtc/quaternion.hpp>

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <cstdio>
#include <cstring>
#include <string>
#include <variant>

static uint32_t fb(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
static void pv3(FILE* o, const glm::vec3& v) { std::fprintf(o, "[%u,%u,%u]", fb(v.x), fb(v.y), fb(v.z)); }
static void pv2(FILE* o, const glm::vec2& v) { std::fprintf(o, "[%u,%u]", fb(v.x), fb(v.y)); }

// Deterministic input stream (xorshift32) for the glm primitive vectors.
static uint32_t g_state = 0x12345678u;
static float frand(float lo, float hi) {
    g_state ^= g_state << 13; g_state ^= g_state >> 17; g_state ^= g_state << 5;
    return lo + (hi - lo) * (float)(g_state >> 8) * (1.0f / 16777216.0f);
}
static glm::vec3 vrand(float lo, float hi) { float a = frand(lo, hi), b = frand(lo, hi), c = frand(lo, hi); return {a, b, c}; }

static void dumpScene(FILE* o, SceneType type, const char* name, const std::filesystem::path& dataDir) {
    Scene scene = loadScenePrebuilt(type, dataDir);
    std::fprintf(o, "\"%s\":{\"meshes\":[", name);
    for (size_t m = 0; m < scene.meshes.size(); m++) {
        const Mesh& mesh = scene.meshes[m];
        if (m) std::fprintf(o, ",");
        std::fprintf(o, "{\"kd\":"); pv3(o, mesh.material.kd);
        std::fprintf(o, ",\"ks\":"); pv3(o, mesh.material.ks);
        std::fprintf(o, ",\"shininess\":%u,\"transparency\":%u,\"textured\":%d,",
                     fb(mesh.material.shininess), fb(mesh.material.transparency), mesh.material.kdTexture ? 1 : 0);
        if (mesh.material.kdTexture) {
            const Image& img = *mesh.material.kdTexture;
            std::fprintf(o, "\"texture\":{\"width\":%d,\"height\":%d,\"rgb_u8\":\"", img.width, img.height);
            for (const glm::vec3& px : img.pixels)
                for (int c = 0; c < 3; c++) {
                    const float v = px[c];
                    const int b = (int)(v * 255.0f + 0.5f);
                    if (b < 0 || b > 255 || fb((float)b / 255.0f) != fb(v)) {
                        std::fprintf(stderr, "texel %a is not a byte / 255.0f\n", (double)v);
                        std::exit(1);
                    }
                    std::fprintf(o, "%02x", b);
                }
            std::fprintf(o, "\"},");
        }
        std::fprintf(o, "\"vertices\":[");
        for (size_t v = 0; v < mesh.vertices.size(); v++) {
            if (v) std::fprintf(o, ",");
            std::fprintf(o, "[");
            pv3(o, mesh.vertices[v].position); std::fprintf(o, ",");
            pv3(o, mesh.vertices[v].normal); std::fprintf(o, ",");
            pv2(o, mesh.vertices[v].texCoord);
            std::fprintf(o, "]");
        }
        std::fprintf(o, "],\"triangles\":[");
        for (size_t t = 0; t < mesh.triangles.size(); t++) {
            if (t) std::fprintf(o, ",");
            std::fprintf(o, "[%u,%u,%u]", mesh.triangles[t].x, mesh.triangles[t].y, mesh.triangles[t].z);
        }
        std::fprintf(o, "]}");
    }
    std::fprintf(o, "],\"lights\":[");
    for (size_t l = 0; l < scene.lights.size(); l++) {
        if (l) std::fprintf(o, ",");
        const auto& light = scene.lights[l];
        if (std::holds_alternative<PointLight>(light)) {
            const auto& p = std::get<PointLight>(light);
            std::fprintf(o, "{\"type\":0,\"v\":["); pv3(o, p.position); std::fprintf(o, ","); pv3(o, p.color);
        } else if (std::holds_alternative<SegmentLight>(light)) {
            const auto& s = std::get<SegmentLight>(light);
            std::fprintf(o, "{\"type\":1,\"v\":["); pv3(o, s.endpoint0); std::fprintf(o, ","); pv3(o, s.endpoint1);
            std::fprintf(o, ","); pv3(o, s.color0); std::fprintf(o, ","); pv3(o, s.color1);
        } else {
            const auto& q = std::get<ParallelogramLight>(light);
            std::fprintf(o, "{\"type\":2,\"v\":["); pv3(o, q.v0); std::fprintf(o, ","); pv3(o, q.edge01);
            std::fprintf(o, ","); pv3(o, q.edge02); std::fprintf(o, ","); pv3(o, q.color0);
            std::fprintf(o, ","); pv3(o, q.color1); std::fprintf(o, ","); pv3(o, q.color2);
            std::fprintf(o, ","); pv3(o, q.color3);
        }
        std::fprintf(o, "]}");
    }
    std::fprintf(o, "]}");
}

int main(int argc, char** argv) {
    if (argc < 3) { std::fprintf(stderr, "usage: %s <reference data dir> <out.json>\n", argv[0]); return 2; }
    const std::filesystem::path dataDir = argv[1];
    FILE* o = std::fopen(argv[2], "w");
    if (!o) { std::perror("fopen"); return 1; }

    std::fprintf(o, "{\"scenes\":{");
    dumpScene(o, SceneType::SingleTriangle, "SingleTriangle", dataDir);               std::fprintf(o, ",");
    dumpScene(o, SceneType::Cube, "Cube", dataDir);                                   std::fprintf(o, ",");
    dumpScene(o, SceneType::CubeTextured, "CubeTextured", dataDir);                   std::fprintf(o, ",");
    dumpScene(o, SceneType::CornellBox, "CornellBox", dataDir);                       std::fprintf(o, ",");
    dumpScene(o, SceneType::CornellBoxParallelogramLight, "CornellBoxParallelogramLight", dataDir); std::fprintf(o, ",");
    dumpScene(o, SceneType::CornellNightClub, "CornellNightClub", dataDir);           std::fprintf(o, ",");
    dumpScene(o, SceneType::Monkey, "Monkey", dataDir);
    std::fprintf(o, "},");

    // regularLightGrid with explicit arguments (used by the synthetic many-light Cornell configs).
    {
        auto grid = regularLightGrid(glm::vec3(-0.45f, 0.49f, -0.45f), glm::ivec2(4, 3), glm::vec3(0.9f, 0.0f, 0.0f),
                                     glm::vec3(0.0f, 0.0f, 0.9f), glm::vec3(0.7f, 0.6f, 0.5f), 0.3f);
        std::fprintf(o, "\"light_grid\":{\"args\":{\"start\":[%u,%u,%u],\"counts\":[4,3],\"e01\":[%u,%u,%u],\"e02\":[%u,%u,%u],"
                        "\"color\":[%u,%u,%u],\"free\":%u},\"lights\":[",
                     fb(-0.45f), fb(0.49f), fb(-0.45f), fb(0.9f), fb(0.0f), fb(0.0f), fb(0.0f), fb(0.0f), fb(0.9f),
                     fb(0.7f), fb(0.6f), fb(0.5f), fb(0.3f));
        for (size_t i = 0; i < grid.size(); i++) {
            if (i) std::fprintf(o, ",");
            std::fprintf(o, "["); pv3(o, grid[i].v0); std::fprintf(o, ","); pv3(o, grid[i].edge01);
            std::fprintf(o, ","); pv3(o, grid[i].edge02); std::fprintf(o, "]");
        }
        std::fprintf(o, "]},");
    }

    // acquireTexel on the CubeTextured texture: random coordinates in [0, 1], the edges, the texture's vertex
    // coordinates and coordinates just below the texel boundaries (the float -> size_t truncation).
    {
        Scene cube = loadScenePrebuilt(SceneType::CubeTextured, dataDir);
        const Image& img = *cube.meshes.at(0).material.kdTexture;
        Features f{};
        std::vector<glm::vec2> tc;
        for (int i = 0; i < 512; i++) tc.push_back(glm::vec2(frand(0.0f, 1.0f), frand(0.0f, 1.0f)));
        for (float a : {0.0f, 1.0f, 0.5f, 0.125f, 0.375f, 0.625f, 0.875f, 0.99999994f, 1e-7f})
            for (float b : {0.0f, 1.0f, 0.25f, 0.75f, 0.99999994f}) tc.push_back(glm::vec2(a, b));
        for (int k = 1; k < 127; k += 7) {
            const float edge = (float)k / (float)(img.width - 1);
            tc.push_back(glm::vec2(edge, edge));
            tc.push_back(glm::vec2(std::nextafter(edge, 0.0f), std::nextafter(edge, 1.0f)));
        }
        std::fprintf(o, "\"texel\":{\"scene\":\"CubeTextured\",\"cases\":[");
        for (size_t i = 0; i < tc.size(); i++) {
            const glm::vec3 t = acquireTexel(img, tc[i], f);
            if (i) std::fprintf(o, ",");
            std::fprintf(o, "["); pv2(o, tc[i]); std::fprintf(o, ","); pv3(o, t); std::fprintf(o, "]");
        }
        std::fprintf(o, "]},");
    }

    // Tone mapping: colours x (exposure, gamma).
    {
        std::fprintf(o, "\"tonemap\":[");
        const float settings[][2] = {{1.5f, 1.0f}, {1.0f, 2.2f}, {0.5f, 1.8f}};
        bool first = true;
        for (const auto& s : settings) {
            Features f{};
            f.exposure = s[0];
            f.gamma = s[1];
            for (int i = 0; i < 64; i++) {
                glm::vec3 c = vrand(0.0f, 4.0f);
                if (i == 0) c = glm::vec3(0.0f);
                glm::vec3 m = exposureToneMapping(c, f);
                if (!first) std::fprintf(o, ",");
                first = false;
                std::fprintf(o, "[%u,%u,", fb(s[0]), fb(s[1])); pv3(o, c); std::fprintf(o, ","); pv3(o, m); std::fprintf(o, "]");
            }
        }
        std::fprintf(o, "],");
    }

    // glm primitives.
    {
        std::fprintf(o, "\"glm\":[");
        for (int i = 0; i < 256; i++) {
            glm::vec3 a = vrand(-10.0f, 10.0f), b = vrand(-10.0f, 10.0f);
            float t = frand(0.0f, 1.0f);
            glm::vec3 e = vrand(-3.2f, 3.2f);
            glm::quat q(e);
            glm::vec3 n = glm::normalize(a);
            float d = glm::dot(a, b);
            float len = glm::length(a);
            float dist = glm::distance(a, b);
            glm::vec3 cr = glm::cross(a, b);
            glm::vec3 mx = glm::mix(a, b, t);
            glm::vec3 rot = q * b;
            if (i) std::fprintf(o, ",");
            std::fprintf(o, "{\"a\":"); pv3(o, a); std::fprintf(o, ",\"b\":"); pv3(o, b);
            std::fprintf(o, ",\"t\":%u,\"e\":", fb(t)); pv3(o, e);
            std::fprintf(o, ",\"q\":[%u,%u,%u,%u]", fb(q.x), fb(q.y), fb(q.z), fb(q.w));
            std::fprintf(o, ",\"normalize\":"); pv3(o, n);
            std::fprintf(o, ",\"dot\":%u,\"length\":%u,\"distance\":%u,\"cross\":", fb(d), fb(len), fb(dist)); pv3(o, cr);
            std::fprintf(o, ",\"mix\":"); pv3(o, mx); std::fprintf(o, ",\"rotate\":"); pv3(o, rot);
            std::fprintf(o, "}");
        }
        std::fprintf(o, "]");
    }
    std::fprintf(o, "}\n");
    std::fclose(o);
    return 0;
}

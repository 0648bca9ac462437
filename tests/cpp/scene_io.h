// scene_io.h -- reads the scene / camera files tests/test_cpp_wrapper.py writes (format in render_scene.cpp).
#pragma once

#include <romis_amd/restir.hpp>

#include <cstdio>
#include <cstdlib>
#include <cstring>

template <class T>
static void rd(FILE* f, T* p, size_t n) {
    if (n && std::fread(p, sizeof(T), n, f) != n) { std::fprintf(stderr, "short read\n"); std::exit(2); }
}

static romis::Camera read_camera(FILE* f) {
    float cam[9];
    rd(f, cam, 9);
    romis::Camera camera;
    camera.fovy = cam[0];
    camera.aspect = cam[1];
    std::memcpy(camera.look_at, cam + 2, 12);
    camera.distance = cam[5];
    std::memcpy(camera.rotation, cam + 6, 12);
    return camera;
}

// scene.bin: meshes, lights, then one camera
static romis::Scene read_scene(const char* path, romis::Camera* camera) {
    FILE* f = std::fopen(path, "rb");
    if (!f) { std::perror("scene"); std::exit(2); }
    romis::Scene scene;
    uint32_t nm = 0;
    rd(f, &nm, 1);
    scene.meshes.resize(nm);
    for (auto& m : scene.meshes) {
        uint32_t V = 0, T = 0;
        rd(f, &V, 1);
        rd(f, &T, 1);
        m.positions.resize(3 * size_t(V));
        m.normals.resize(3 * size_t(V));
        m.triangles.resize(3 * size_t(T));
        rd(f, m.positions.data(), m.positions.size());
        rd(f, m.normals.data(), m.normals.size());
        rd(f, m.triangles.data(), m.triangles.size());
        float mat[8];
        rd(f, mat, 8);
        std::memcpy(m.material.kd, mat, 12);
        std::memcpy(m.material.ks, mat + 3, 12);
        m.material.shininess = mat[6];
        m.material.transparency = mat[7];
    }
    uint32_t nl = 0;
    rd(f, &nl, 1);
    scene.lights.resize(nl);
    rd(f, scene.lights.data(), nl);
    romis::Camera c = read_camera(f);
    if (camera) *camera = c;
    std::fclose(f);
    return scene;
}

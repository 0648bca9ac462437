// bvh.h -- host-side SAH BVH build, flattened into the stackless ("threaded") layout the kernels traverse.
// Replaces EmbreeInterface::initScene's rtcCommitScene(BUILD_QUALITY_HIGH) (embree_interface.cpp:30-51).
#pragma once

#include <cstdint>
#include <vector>

namespace romis {

struct BvhTriangle {
    float v0[3], v1[3], v2[3];
};

struct FlatBvh {
    // 8 floats per node: lo.xyz, bits(miss), hi.xyz, bits(leaf)   (see SceneDev in restir_types.h)
    std::vector<float> nodes;
    // triangle order: tri_order[k] = original index of the k-th triangle in BVH order
    std::vector<uint32_t> tri_order;
    uint32_t num_nodes = 0;
    uint32_t max_depth = 0;
};

// Builds a binned-SAH BVH (leaves of <= max_leaf triangles) and flattens it depth-first with miss links.
// Boxes are padded by `pad` in every direction so the device slab test is conservative.
FlatBvh build_bvh(const std::vector<BvhTriangle>& tris, uint32_t max_leaf = 4);

}  // namespace romis

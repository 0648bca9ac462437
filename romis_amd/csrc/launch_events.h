// launch_events.h -- host side shared by the launchers of kernels.hip and mis.hip: the timed-launch event pair and the
// launch shape constants.
#pragma once

#include <hip/hip_ext.h>

#include "restir_types.h"

namespace romis {

// Timed launches: restir.cpp's TIMED hands a start / stop event pair to the next launch, which records them inside its
// own dispatch (hipExtLaunchKernelGGL) -- no separate event packets, hence no stream gaps.
inline thread_local hipEvent_t g_ev_start = nullptr, g_ev_stop = nullptr;
inline thread_local bool g_launched = false;

#define ROMIS_LAUNCH(kernel, grid, block, lds, stream, ...)                                                    \
    do {                                                                                                      \
        /* a multi-launch stage: start event on its first kernel, stop event after its last */              \
        hipExtLaunchKernelGGL(kernel, grid, block, lds, stream, g_launched ? nullptr : g_ev_start, g_ev_stop, 0, \
                              __VA_ARGS__);                                                                   \
        g_launched = true;                                                                                    \
    } while (0)

constexpr uint32_t kBlock = 256;
constexpr size_t kLdsBudget = 64 * 1024;   // LDS a kernel may stage a BVH / light table into
inline size_t bvh_lds_bytes(const SceneDev& s) { return ((size_t)2 * s.num_nodes + (size_t)3 * s.num_tris) * 16; }

}  // namespace romis

// launch.h -- host-side launchers of the kernels in kernels.hip (all enqueue on `stream`, never synchronise).
#pragma once

#include "restir_types.h"

namespace romis {

// The target-pdf cache (N = 1, SoA planes, nullable): rp[p] = the target pdf of pixel p's held sample at p.
// RIS / temporal / the lean spatial passes write it for their output; temporal and the passes read it for the input's own
// sample instead of re-evaluating it (same pixel, same G-buffer, same sample: the same bits).
// n_t2 (nullable): a second record buffer that also receives the G-buffer n_t (the ping-pong partner)
hipError_t launch_primary(const SceneDev& s, const Region& rg, const CameraDev& cam, float4* n_t, float4* p_mat,
                          float4* n_t2, const Tuning& tu, hipStream_t stream);
hipError_t launch_ris(const SceneDev& s, const Region& rg, const FeaturesDev& f, uint32_t key, const float* origin,
                      const float4* n_t, const float4* p_mat, float4* ra, float4* rb, float2* rdbg, float* rp,
                      const Tuning& tu, hipStream_t stream);
// genPrimaryRayHits + genCanonicalSamples in one kernel over the same region (needs the BVH to fit in LDS)
hipError_t launch_primary_ris(const SceneDev& s, const Region& rg, const CameraDev& cam, const FeaturesDev& f, uint32_t key,
                              float4* n_t, float4* p_mat, float4* n_t2, float4* ra, float4* rb, float2* rdbg,
                              float* rp, const Tuning& tu, hipStream_t stream, uint8_t* tmiss = nullptr,
                              uint32_t skip_res = 0u,    // bit 0: background reservoirs, bit 1: background G-buffer
                              bool* tmiss_written = nullptr,    // the flags were written (else pass none on)
                              Handles h = Handles{nullptr, nullptr, 0u});   // N = 1 point-light kernels: sample handles
// restir_render's N = 1 biased passes over sample handles (k_spatial1h): the scene, features and knobs allow them and
// every M `passes` passes can produce fits the handle's 24 bits
bool spatial_handles_ok(const SceneDev& s, const FeaturesDev& f, const Tuning& tu, uint32_t passes);
// which: 0 point-light handles (8 B per pixel), 1 light-grid handles (16 B), -1 none
// m0: the largest M entering the passes when it exceeds RIS's f.M (temporal reuse); 0 = f.M
int spatial_handle_kind(const SceneDev& s, const FeaturesDev& f, const Tuning& tu, uint32_t passes, uint64_t m0 = 0);
bool primary_ris_fits(const SceneDev& s);
// primary rays + RIS + temporal reuse in one kernel (N = 1 / 2, point lights, the light table in LDS; fuse.temporal)
bool primary_ris_temporal_fits(const SceneDev& s, const FeaturesDev& f, const Tuning& tu);
hipError_t launch_primary_ris_temporal(const SceneDev& s, const Region& rg, const CameraDev& cam, const FeaturesDev& f,
                                       uint32_t key, float4* n_t, float4* p_mat, float4* n_t2, float4* ra, float4* rb,
                                       float2* rdbg, float* rp, const Tuning& tu, hipStream_t stream, TemporalIn tin,
                                       Handles h);   // h: the output's sample handles (N = 1; as launch_primary_ris)
// the N = 1 spatial pass reads background tiles through MissTiles for this scene / features / knobs (SoA planes)
bool spatial_reads_flags(const SceneDev& s, const FeaturesDev& f, const Tuning& tu);
// final shading writes background tiles from MissTiles without reading them (k_final_n1_sorted)
bool final_reads_flags(const SceneDev& s, const FeaturesDev& f, const Tuning& tu);
hipError_t launch_temporal(const SceneDev& s, const Region& rg, const FeaturesDev& f, uint32_t key, const float* origin,
                           const float4* n_t, const float4* p_mat, const float4* ca, const float4* cb,
                           const float4* pa, const float4* pb, float4* oa, float4* ob, float2* odbg,
                           const float* rp_in, float* rp_out, const Tuning& tu, hipStream_t stream);
hipError_t launch_spatial(const SceneDev& s, const Region& rg, const FeaturesDev& f, uint32_t key, const float* origin,
                          const float4* n_t, const float4* p_mat, const float4* ia, const float4* ib, float4* oa,
                          float4* ob, float2* odbg, const float* rp_in, const float* rp_nb, float* rp_out,
                          bool* rp_written, const Tuning& tu, hipStream_t stream, uint8_t* vis_out = nullptr,
                          bool* vis_written = nullptr, MissTiles mt = MissTiles{nullptr, 0u, 0u},
                          Handles hin = Handles{nullptr, nullptr, 0u},    // the input's sample handles (k_spatial1h)
                          Handles hout = Handles{nullptr, nullptr, 0u});  // the output's, for a later pass
hipError_t launch_final(const SceneDev& s, const Region& rg, const FeaturesDev& f, const float* origin,
                        const float4* n_t, const float4* p_mat, const float4* ra, const float4* rb, float* rgb,
                        const Tuning& tu, hipStream_t stream, const uint8_t* vis_in = nullptr,
                        MissTiles mt = MissTiles{nullptr, 0u, 0u});
hipError_t launch_halo_pack(const Region& rg, const HaloSegs& hs, uint32_t N, const float4* ra, const float4* rb, float4* out,
                            hipStream_t stream);
hipError_t launch_halo_unpack(const Region& rg, const HaloSegs& hs, uint32_t N, const float4* in, float4* ra, float4* rb,
                              hipStream_t stream);
// The next frame-kernel launch records `start` / `stop` (nullptr: none) within its dispatch; launch_events_used()
// tells whether a launch consumed them since the last set_launch_events.
void set_launch_events(hipEvent_t start, hipEvent_t stop);
bool launch_events_used();
hipError_t launch_read_stream(const float4* buf, size_t n4, float* sink, hipStream_t stream);
// R-MIS / R-OMIS over a whole W x H image (stage / frame buffers in the RESTIR_BUF_MIS_* layouts)
hipError_t launch_mis_neighbours(const SceneDev& s, uint32_t W, uint32_t H, const FeaturesDev& f, uint32_t key_s, uint32_t key_d,
                                 const float4* n_t, const float4* p_mat, uint32_t* nbr, hipStream_t stream);
hipError_t launch_mis_accumulate(const SceneDev& s, uint32_t W, uint32_t H, const FeaturesDev& f, const float* origin,
                                 const float4* n_t, const float4* p_mat, const uint32_t* nbr, const float4* ra,
                                 const float4* rb, const float2* rdbg, uint32_t iteration, float* acc, float* smp,
                                 uint32_t smp_samples, const Tuning& tu, hipStream_t stream);
hipError_t launch_mis_finish(uint32_t W, uint32_t H, const FeaturesDev& f, const float* acc, float* rgb, hipStream_t stream);
// R-OMIS alpha visualisation words: [3T images][W*H] (k_romis_vis_t{T})
hipError_t launch_romis_vis(uint32_t W, uint32_t H, uint32_t T, const float* acc, uint32_t* out, hipStream_t stream);
hipError_t launch_debug_cod(uint32_t n, const float* A, const float* b, float* x, uint32_t count, hipStream_t stream);
hipError_t launch_debug_math(const float* x, const float* y, float* pw, float* ex, uint32_t n, hipStream_t stream);

}  // namespace romis

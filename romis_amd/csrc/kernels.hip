// kernels.hip -- hand-written gfx950 (CDNA4) kernels of the ReSTIR direct-lighting path.
//
//   k_primary   genPrimaryRayHits (render_utils.cpp:13-34) + closestHit (embree_interface.cpp:64-90)
//   k_ris       genInitialSamples / genCanonicalSamples (render_utils.cpp:36-52, light.cpp:39-99)
//   k_temporal  temporalReuse + Reservoir::combineBiased (render_utils.cpp:142-177, reservoir.cpp:40-66)
//   k_spatial   spatialReuse, one pass (render_utils.cpp:87-140) + combineBiased / combineUnbiased
//               (reservoir.cpp:40-104)
//   k_final     final shading + tone map + Screen y-flip (render.cpp:38-58, render_utils.cpp:54-65,
//               tone_mapping.cpp:8-11, screen.cpp:37-43)
//
// One lane per pixel throughout: the reservoir update (Reservoir::update, reservoir.cpp:10-32) is a serial
// prefix over the candidate stream whose float rounding must match the reference order exactly, so it stays
// a per-lane loop; a wave's 64 lanes work on 64 pixels.  Reservoirs and the G-buffer are SoA float4 planes
// read with 16-byte coalesced loads.  Visibility uses a stackless threaded BVH (no scratch stack) that the
// ray kernels stage once per (persistent) workgroup into LDS; the light table is staged into LDS for RIS.
#include "kernels_common.h"

// ---------------------------------------------------------------------------------------------------------
// genPrimaryRayHits for pixel (x, y) at view index p: writes and returns the G-buffer records (n_t, p_mat)
// tl (nullable): the block's candidate triangles (tile_triangles: four 64-entry segments, tl_cnt[w] entries each),
// tested instead of walking the BVH
__device__ __forceinline__ void primary_pixel(const SceneDev& s, const Region& rg, const CameraDev& cam, const Bvh& bvh,
                                              uint32_t x, uint32_t y, size_t p, float4* __restrict__ n_t2,
                                              float4* __restrict__ n_t, float4* __restrict__ p_mat, float4& nt_out,
                                              float4& pm_out, bool store = true, const uint16_t* tl = nullptr,
                                              const uint32_t* tl_cnt = nullptr) {
    const v3 o = mk(cam.origin[0], cam.origin[1], cam.origin[2]);
    {
        float nx = (float)x / (float)rg.W * 2.0f - 1.0f;
        float ny = (float)y / (float)rg.H * 2.0f - 1.0f;
        v3 csd = vnormalize(mk(-nx * cam.half_w, ny * cam.half_h, 1.0f));
        v3 d = qrotate(cam.quat, csd);
        float t, u = 0.0f, v = 0.0f;
        uint32_t tri;
        v3 n = mk(0.0f, 0.0f, 0.0f);
        float2 tc = make_float2(0.0f, 0.0f);   // a miss keeps the value-initialised HitInfo::texCoord
        uint32_t m = s.num_materials - 1;
        if (tl ? closest_list(bvh, tl, tl_cnt, o, d, t, u, v, tri) : closest(bvh, o, d, t, u, v, tri)) {
            float w0 = (1.0f - u) - v;
            float4 a = s.tri_n0[tri], b = s.tri_n1[tri], c = s.tri_n2[tri];
            n = vadd(vadd(vscale(xyz(a), w0), vscale(xyz(b), u)), vscale(xyz(c), v));
            m = __float_as_uint(a.w);
            if (s.gbuf_uv) {   // texCoord: rtcInterpolate0 of attribute slot 1 (embree_interface.cpp:80-81)
                const float4 t01 = s.tri_uv[2 * tri], t2 = s.tri_uv[2 * tri + 1];
                tc.x = (t01.x * w0 + t01.z * u) + t2.x * v;
                tc.y = (t01.y * w0 + t01.w * u) + t2.y * v;
            }
        } else {
            t = ROMIS_FLT_MAX;
        }
        if (s.gbuf_uv) s.gbuf_uv[p] = tc;
        v3 P = vadd(o, vscale(d, t));
        const float4 nt = make_float4(n.x, n.y, n.z, t);
        pm_out = make_float4(P.x, P.y, P.z, __uint_as_float(m));
        nt_out = nt;
        if (store) {   // store = false: the caller stores the records (or not: primary_ris_body's background tiles)
            n_t[gidx(rg, p)] = nt;
            if (n_t2) n_t2[gidx(rg, p)] = nt;   // the other record buffer of the ping-pong pair
            p_mat[p] = pm_out;
        }
    }
}

// Candidate triangles of a 32 x 8 tile's primary rays (round 6, primary.tl).  Every ray of the tile leaves the camera
// origin o in the direction R (a, b, 1) (primary_pixel: R = the camera rotation, a = -nx half_w, b = ny half_h over the
// tile's pixel coordinates); the pyramid of those directions, widened by two pixels on each side, is bounded by the
// four planes through o with the world normals R (1, 0, -a0), R (-1, 0, a1), R (0, 1, -b0), R (0, -1, b1).  A triangle
// whose three vertices all lie outside one of them (beyond a relative margin of 1e-5, far above the rounding of this
// test and far below the two pixels) cannot be hit by any ray of the tile; the list keeps the others.  closest_list
// over it returns closest()'s hit (its selection does not depend on order), as the BVH walk does -- both skip only
// geometry the rays pass well clear of (the BVH's boxes are padded by 1e-5 of the scene).  Thread t tests triangle t
// (num_tris <= 256) from global memory and each wave compacts its survivors by ballot into its own 64-entry segment:
// no atomics, and no barrier of its own -- the caller's BVH staging barrier publishes the lists.
constexpr uint32_t kTlMaxTris = 256u;
__device__ __forceinline__ void tile_triangles(const SceneDev& s, const Region& rg, const CameraDev& cam, int x0, int x1,
                                               int y0, int y1, uint16_t* tl, uint32_t* tl_cnt) {
    const float W = (float)rg.W, H = (float)rg.H;
    // pixel coordinates two pixels beyond the tile (primary_pixel's nx = x / W * 2 - 1, ny = y / H * 2 - 1)
    const float nxl = (float)(x0 - 2) / W * 2.0f - 1.0f, nxh = (float)(x1 + 2) / W * 2.0f - 1.0f;
    const float nyl = (float)(y0 - 2) / H * 2.0f - 1.0f, nyh = (float)(y1 + 2) / H * 2.0f - 1.0f;
    const float a0 = fminf(-nxl * cam.half_w, -nxh * cam.half_w), a1 = fmaxf(-nxl * cam.half_w, -nxh * cam.half_w);
    const float b0 = fminf(nyl * cam.half_h, nyh * cam.half_h), b1 = fmaxf(nyl * cam.half_h, nyh * cam.half_h);
    // the rotation's columns: the camera axes in world space (the matrix of qrotate)
    const float qx = cam.quat.x, qy = cam.quat.y, qz = cam.quat.z, qw = cam.quat.w;
    const v3 rx = mk(1.0f - 2.0f * (qy * qy + qz * qz), 2.0f * (qx * qy + qw * qz), 2.0f * (qx * qz - qw * qy));
    const v3 ry = mk(2.0f * (qx * qy - qw * qz), 1.0f - 2.0f * (qx * qx + qz * qz), 2.0f * (qy * qz + qw * qx));
    const v3 rz = mk(2.0f * (qx * qz + qw * qy), 2.0f * (qy * qz - qw * qx), 1.0f - 2.0f * (qx * qx + qy * qy));
    const v3 pn[4] = {vsub(rx, vscale(rz, a0)), vsub(vscale(rz, a1), rx), vsub(ry, vscale(rz, b0)), vsub(vscale(rz, b1), ry)};
    const uint32_t t = threadIdx.x, lane = t & 63u;
    bool keep = false;
    if (t < s.num_tris) {
        const v3 o = mk(cam.origin[0], cam.origin[1], cam.origin[2]);
        const v3 v0 = xyz(s.tri_v0[t]);
        const v3 p0 = vsub(v0, o), p1 = vsub(vadd(v0, xyz(s.tri_e1[t])), o), p2 = vsub(vadd(v0, xyz(s.tri_e2[t])), o);
        const float l0 = fabsf(p0.x) + fabsf(p0.y) + fabsf(p0.z), l1 = fabsf(p1.x) + fabsf(p1.y) + fabsf(p1.z);
        const float l2 = fabsf(p2.x) + fabsf(p2.y) + fabsf(p2.z);
        bool out = false;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const float m = 1e-5f * (fabsf(pn[k].x) + fabsf(pn[k].y) + fabsf(pn[k].z));
            out = out || (vdot(pn[k], p0) < -m * l0 && vdot(pn[k], p1) < -m * l1 && vdot(pn[k], p2) < -m * l2);
        }
        keep = !out;
    }
    const unsigned long long bal = __ballot(keep);
    if (keep) tl[(t & ~63u) + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = (uint16_t)t;
    if (lane == 0u) tl_cnt[t >> 6] = (uint32_t)__popcll(bal);
}

// k_primary: persistent blocks stage the BVH into LDS once, then sweep 32x8 tiles; writes n_t / p_mat.
template <bool LDS_BVH>
__device__ __forceinline__ void primary_body(const SceneDev& s, const Region& rg, const CameraDev& cam, float4* __restrict__ n_t2,
                                             float4* __restrict__ n_t, float4* __restrict__ p_mat) {
    const Bvh bvh = LDS_BVH ? stage_bvh(s, g_lds) : global_bvh(s);
    const uint32_t nt = work_items(rg);
    for (uint32_t tile = blockIdx.x; tile < nt; tile += gridDim.x) {
        uint32_t x, y;
        size_t p;
        if (!work_pixel(rg, tile, x, y, p)) continue;
        float4 a, b;
        primary_pixel(s, rg, cam, bvh, x, y, p, n_t2, n_t, p_mat, a, b);
    }
}

extern "C" __global__ __launch_bounds__(256) void k_primary(SceneDev s, Region rg, CameraDev cam, float4* n_t, float4* p_mat,
                                                           float4* n_t2) {
    primary_body<false>(s, rg, cam, n_t2, n_t, p_mat);
}
extern "C" __global__ __launch_bounds__(256) void k_primary_lds(SceneDev s, Region rg, CameraDev cam, float4* n_t,
                                                               float4* p_mat, float4* n_t2) {
    primary_body<true>(s, rg, cam, n_t2, n_t, p_mat);
}

// ---------------------------------------------------------------------------------------------------------
// Combine state shared by temporal and spatial: out[] (Reservoir(N) of the current pixel) + routed M sums.
template <int NT>
struct Combiner {
    Sub out[NT > 0 ? NT : RESTIR_MAX_N_DEV];
    uint32_t macc[NT > 0 ? NT : RESTIR_MAX_N_DEV];
    uint32_t N_;
    uint32_t t;      // update counter (RNG slot offset)
    // compile-time trip count when N is a template constant (keeps out[] / macc[] in registers)
    __device__ __forceinline__ uint32_t n() const { return NT > 0 ? (uint32_t)NT : N_; }
    __device__ __forceinline__ void init(uint32_t nn) {
        N_ = nn;
        for (uint32_t j = 0; j < n(); j++) { sub_init(out[j]); macc[j] = 0u; }
        t = 0;
    }
    // combine one input sub-reservoir (reservoir.cpp:47-54 / :75-82)
    __device__ __forceinline__ void consume(const SceneDev& s, const FeaturesDev& f, const Px& cur, const Sub& in, uint32_t ps, uint32_t slot0) {
        consume_pd(target_pdf(s, f, cur, in.pos, in.col), in, ps, slot0);
    }
    // the same with the input's target pdf at the combining pixel already known (the rp cache)
    __device__ __forceinline__ void consume_pd(float pd, const Sub& in, uint32_t ps, uint32_t slot0) {
        float w = (pd * in.W) * (float)in.M;
        uint32_t k = res_update<NT>(out, n(), in.pos, in.col, w, rand01(draw(ps, slot0 + t)), pd);
        t++;
        macc_add<NT>(macc, k, in.M);
    }
    __device__ __forceinline__ void finish_biased(const SceneDev& s, const FeaturesDev& f, const Px& cur, float* pd_out = nullptr) {
        for (uint32_t j = 0; j < n(); j++) out[j].M = macc[j];
        for (uint32_t j = 0; j < n(); j++) {
            const float pj = out[j].has_pd ? out[j].pd : target_pdf(s, f, cur, out[j].pos, out[j].col);
            out[j].W = contribution_weight(pj, out[j].M, out[j].wsum);
            if (pd_out) pd_out[j] = pj;
        }
    }
};

// ---------------------------------------------------------------------------------------------------------
// genCanonicalSamples for one pixel whose G-buffer records are (nt, pm); lights = the light table (global or
// the block's LDS copy), bvh = the traversal arrays for the initial visibility rays.
// LT: the light table's form (host-detected scene properties; genCanonicalSamples' switch, light.cpp:55-78, reduces
// to one case, so the candidate loop carries no lane-divergent light-type branch):
//   kLtGeneral  7 float4 per light (SceneDev::lights);
//   kLtPoint    every light a point light (light_types == 1): the compact table SceneDev::light_c2, two planes (rows 0
//               and 3 of every record: positions, then colours -- a random light's 16-byte LDS read meets 16 bank
//               groups instead of the 8 of 32-byte records);
//   kLtGrid     every light a parallelogram with light 0's edges and one colour at all four of its corners
//               (SceneDev::lights_grid: the reference's regularLightGrid, scene.cpp:5-28): light_c2 holds its
//               corner v0 and colour; the shared edges are read from light 0's record, and the two identical
//               inner mixes of the colour interpolation are evaluated once.  The same operations on the same
//               values as the general case.
//   kLtPgram    every light a parallelogram with one colour at all four of its corners, edges free (the reference's
//               default nightclub set, scene.cpp:30-66: two wall grids): SceneDev::light_c4, rows 0..3 of each record
//               (v0, edge01, edge02, colour), 4 float4 per light instead of 7.
//   kLtRegular  a light grid laid out as regularLightGrid does (SceneDev::lights_regular, host-verified bit for bit):
//               the drawn light's corner is (start + s01 x) + s02 y, x = i >> log2(ny), y = i & (ny - 1), evaluated in
//               float as the reference built it; only its colour is read, from SceneDev::light_col (one float4 per
//               light instead of kLtGrid's two: C4 / C5's 1,024 / 4,096-light grids).
constexpr int kLtGeneral = 0, kLtPoint = 1, kLtGrid = 2, kLtPgram = 3, kLtRegular = 4;
// float4s per light of the table form LT
__host__ __device__ constexpr uint32_t lt_stride(int lt) {
    return lt == kLtGeneral ? 7u : lt == kLtPgram ? 4u : lt == kLtRegular ? 1u : 2u;
}
template <int NT, int LT = kLtGeneral, bool TEMP = false>
__device__ __forceinline__ void ris_pixel(const SceneDev& s, const Region& rg, const FeaturesDev& f, uint32_t key, v3 origin,
                                          const float4* lights, const Bvh& bvh, float4 nt, float4 pm, uint32_t x,
                                          uint32_t y, size_t p, float4* __restrict__ ra, float4* __restrict__ rb,
                                          float2* __restrict__ rdbg, float* __restrict__ rp, const GlTabs& tb,
                                          float* __restrict__ hw = nullptr, uint32_t* __restrict__ hm = nullptr,
                                          bool store_res = true, TemporalIn tin = TemporalIn{nullptr, nullptr, 0u}) {
    const uint32_t L = s.num_lights;
    uint32_t hidx = L;   // the held sample's light index for the handle planes (k_spatial1h; L = the zero sample)
    uint32_t hidx1 = L;  // N = 2: sub-reservoir 1's (the handle record of k_spatial2hg)
    float ha = 0.0f, hb = 0.0f;   // kLtRegular: its fractions (grid handles, k_spatial1g_t2)
    const size_t npx = (size_t)rg.vw * rg.vh;
    const uint32_t N = NT > 0 ? (uint32_t)NT : f.N;
    const float invL = 1.0f / (float)L;
    {
        Sub r[NT > 0 ? NT : RESTIR_MAX_N_DEV];
        for (uint32_t j = 0; j < N; j++) sub_init(r[j]);
        if (L != 0) {
            Px px = make_px(s, nt, pm, origin, p);
            const uint32_t ps = pix_state(key, y * rg.W + x);
            for (uint32_t j = 0; j < N; j++) r[j].M = 0u;
            // A primary-ray miss carries the value-initialised HitInfo (kd = ks = 0, N = 0): its target pdf is
            // exactly 0 for every finite light sample, so all M updates add w = 0 to sub-reservoir
            // 0 (the argmin over equal wSums), none is accepted and W = 0 -- the loop's result is known.
            const uint32_t c_end = (px.mat == s.num_materials - 1 && s.lights_finite && !__builtin_isnan(px.P.x + px.P.y + px.P.z))
                                       ? 0u : f.M;
            if (c_end == 0u) r[0].M = f.M;
            // candidate c: light sample (genCanonicalSamples' switch, light.cpp:55-78) from its table record lt,
            // whose rows 0 (first point, type) and 3 (first colour) the caller has already read
            auto sample_rec = [&](uint32_t c, const float4* lt, float4 l0, float4 l3, v3& pos, v3& col) {
                uint32_t type = __float_as_uint(l0.w);
                if (type == 0u) {
                    pos = xyz(l0);
                    col = xyz(l3);
                } else if (type == 1u) {
                    float fr = rand01(draw(ps, 4u * c + 1u));
                    pos = vmix(xyz(l0), xyz(lt[1]), fr);
                    col = vmix(xyz(l3), xyz(lt[4]), fr);
                } else {
                    float a = rand01(draw(ps, 4u * c + 1u));
                    float b = rand01(draw(ps, 4u * c + 2u));
                    pos = vadd(vadd(xyz(l0), vscale(xyz(lt[1]), a)), vscale(xyz(lt[2]), b));
                    v3 l01 = vmix(xyz(l3), xyz(lt[4]), a);
                    v3 l23 = vmix(xyz(lt[5]), xyz(lt[6]), a);
                    col = vmix(l01, l23, b);
                }
            };
            auto record = [&](uint32_t c) {
                return lights + lt_stride(LT) * uniform_index(draw(ps, 4u * c), L);
            };
            // kLtGrid: the shared edges, light 0's rows 1 and 2, read per candidate through the scalar cache (an
            // opaque pointer keeps the compiler from hoisting them into loop-long VGPRs, which spill)
            auto shared_row = [&](uint32_t r) {
                const float4* sh = s.lights;
                asm volatile("" : "+s"(sh));
                return xyz(sh[r]);
            };
            // kLtRegular: candidate c drew light i, whose colour is gc
            auto sample_reg = [&](uint32_t c, uint32_t i, v3 gc, v3& pos, v3& col) {
                const float xl = (float)(i >> s.grid_ny_log2), yl = (float)(i & ((1u << s.grid_ny_log2) - 1u));
                const v3 v0 = vadd(vadd(xyz(s.grid_start), vscale(xyz(s.grid_s01), xl)), vscale(xyz(s.grid_s02), yl));
                float a = rand01(draw(ps, 4u * c + 1u));
                float b = rand01(draw(ps, 4u * c + 2u));
                pos = vadd(vadd(v0, vscale(shared_row(1), a)), vscale(shared_row(2), b));
                const v3 m = vmix(gc, gc, a);
                col = vmix(m, m, b);
            };
            auto sample = [&](uint32_t c, v3& pos, v3& col) {
                const float4* lt = record(c);
                if (LT == kLtPoint) {   // the light_c2 planes: position at [i], colour at [L + i]
                    const uint32_t i = uniform_index(draw(ps, 4u * c), L);
                    pos = xyz(lights[i]); col = xyz(lights[L + i]);
                } else if (LT == kLtGrid) {   // sampleParallelogramLight, as sample_rec's type-2 case
                    const uint32_t i = uniform_index(draw(ps, 4u * c), L);
                    float a = rand01(draw(ps, 4u * c + 1u));
                    float b = rand01(draw(ps, 4u * c + 2u));
                    pos = vadd(vadd(xyz(lights[i]), vscale(shared_row(1), a)), vscale(shared_row(2), b));
                    const v3 gc = xyz(lights[L + i]);
                    const v3 m = vmix(gc, gc, a);   // = vmix(c0, c1, a) = vmix(c2, c3, a): all four corners are gc
                    col = vmix(m, m, b);
                } else if (LT == kLtRegular) {   // the corner of light i by arithmetic (scene.cpp:14-15)
                    const uint32_t i = uniform_index(draw(ps, 4u * c), L);
                    sample_reg(c, i, xyz(lights[i]), pos, col);
                } else if (LT == kLtPgram) {
                    float a = rand01(draw(ps, 4u * c + 1u));
                    float b = rand01(draw(ps, 4u * c + 2u));
                    pos = vadd(vadd(xyz(lt[0]), vscale(xyz(lt[1]), a)), vscale(xyz(lt[2]), b));
                    const v3 gc = xyz(lt[3]);
                    const v3 m = vmix(gc, gc, a);
                    col = vmix(m, m, b);
                } else {
                    sample_rec(c, lt, lt[0], lt[3], pos, col);
                }
            };
            auto weight = [&](float pd) { return s.light_scale != 0.0f ? pd * s.light_scale : pd / invL; };  // light.cpp:80
            if (NT == 1) {
                // Reservoir::update (reservoir.cpp:10-32) keeping the accepted candidate's index instead of its
                // sample: the sample is a function of the candidate's draws (slots 4c .. 4c + 2), so it is drawn
                // again once after the loop -- two selects per candidate instead of nine
                uint32_t best = 0xFFFFFFFFu;
                for (uint32_t c = 0; c < c_end; c++) {
                    v3 pos, col;
                    sample(c, pos, col);
                    const float pd = target_pdf(s, f, px, pos, col, tb);
                    const float w = weight(pd);
                    r[0].M += 1u;
                    r[0].wsum += w;
                    if (accept_u(rand01(draw(ps, 4u * c + 3u)), w, r[0].wsum)) { best = c; r[0].chosen = w; r[0].pd = pd; }
                }
                if (best != 0xFFFFFFFFu) {
                    sample(best, r[0].pos, r[0].col);
                    r[0].has_pd = true;
                    if (LT == kLtPoint || LT == kLtRegular) hidx = uniform_index(draw(ps, 4u * best), L);
                    if (LT == kLtRegular) { ha = rand01(draw(ps, 4u * best + 1u)); hb = rand01(draw(ps, 4u * best + 2u)); }
                }
            } else if constexpr (NT == 2) {
                // res_update<2> (Reservoir::update routed to the smaller wSum -- argmin from FLT_MAX, strict <, first
                // index) keeping each sub-reservoir's accepted candidate index, as the N = 1 loop does: the samples
                // are drawn again after the loop
                uint32_t best[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};
                for (uint32_t c = 0; c < c_end; c++) {
                    v3 pos, col;
                    sample(c, pos, col);
                    const float pd = target_pdf(s, f, px, pos, col, tb);
                    const float w = weight(pd);
                    const float b0 = r[0].wsum < ROMIS_FLT_MAX ? r[0].wsum : ROMIS_FLT_MAX;
                    const bool k1 = r[1].wsum < b0;
                    const float ws = (k1 ? r[1].wsum : r[0].wsum) + w;
                    const bool acc = accept_u(rand01(draw(ps, 4u * c + 3u)), w, ws);
                    r[0].M += k1 ? 0u : 1u;
                    r[1].M += k1 ? 1u : 0u;
                    r[0].wsum = k1 ? r[0].wsum : ws;
                    r[1].wsum = k1 ? ws : r[1].wsum;
                    if (acc) {
                        if (k1) { best[1] = c; r[1].chosen = w; r[1].pd = pd; }
                        else { best[0] = c; r[0].chosen = w; r[0].pd = pd; }
                    }
                }
#pragma unroll
                for (uint32_t j = 0; j < 2u; j++)
                    if (best[j] != 0xFFFFFFFFu) {
                        sample(best[j], r[j].pos, r[j].col);
                        r[j].has_pd = true;
                    }
                if (LT == kLtPoint) {
                    if (best[0] != 0xFFFFFFFFu) hidx = uniform_index(draw(ps, 4u * best[0]), L);
                    if (best[1] != 0xFFFFFFFFu) hidx1 = uniform_index(draw(ps, 4u * best[1]), L);
                }
            } else {
                for (uint32_t c = 0; c < c_end; c++) {
                    v3 pos, col;
                    sample(c, pos, col);
                    const float pd = target_pdf(s, f, px, pos, col, tb);
                    res_update<NT>(r, N, pos, col, weight(pd), rand01(draw(ps, 4u * c + 3u)), pd);
                }
            }
            float pj0 = 0.0f;
            for (uint32_t j = 0; j < N; j++) {
                // the held sample's target pdf: W's p-hat (light.cpp:90-93) and, N = 1, the pdf cache rp
                const float pj = r[j].has_pd ? r[j].pd : target_pdf(s, f, px, r[j].pos, r[j].col, tb);
                if (f.initial_vis && !visible(bvh, px.P, r[j].pos)) r[j].W = 0.0f;
                else r[j].W = contribution_weight(pj, r[j].M, r[j].wsum);
                if (j == 0) pj0 = pj;
                if (NT == 1 && rp && !TEMP) rp[p] = pj;
            }
            if (TEMP) {
                // temporalReuse (render_utils.cpp:142-177) fused: temporal_body's steps on the RIS reservoirs still in
                // registers -- the predecessor's M clamped to clampM * M_current + 1, the current reservoir (its
                // target pdf here: pj0 for N = 1, the pdf cache's value) then the predecessor's combined biased
                Sub prev[NT > 0 ? NT : 1];
                unsigned long long mcur = 0, mprev = 0;
                uint32_t phidx = L;   // the predecessor's light index (frame handles)
                uint32_t pidx2[2] = {L, L};   // N = 2: its sub-reservoirs' light indices (the 16-byte frame handle records)
                float4 prec = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                if (NT == 2 && LT == kLtPoint && tin.hw) prec = reinterpret_cast<const float4*>(tin.hw)[p];
#pragma unroll
                for (uint32_t j = 0; j < (uint32_t)NT; j++) {
                    if (NT == 2 && LT == kLtPoint && tin.hw) {
                        // sub-reservoir j from its handle record (W_j, M_j | i_j << 24): the values the planes hold
                        const uint32_t hv = __float_as_uint(j == 0 ? prec.y : prec.w);
                        sub_init(prev[j]);
                        pidx2[j] = hv >> 24;
                        prev[j].W = j == 0 ? prec.x : prec.z;
                        prev[j].M = hv & 0x00FFFFFFu;
                        if (pidx2[j] < L) { prev[j].pos = xyz(lights[pidx2[j]]); prev[j].col = xyz(lights[L + pidx2[j]]); }
                    } else if (NT == 1 && LT == kLtPoint && tin.hw) {
                        // the predecessor from its handle: the same W, M, position and colour the reservoir planes
                        // hold (index L: the zero sample)
                        const uint32_t hv = tin.hm[p];
                        sub_init(prev[j]);
                        phidx = hv >> 24;
                        prev[j].W = tin.hw[p];
                        prev[j].M = hv & 0x00FFFFFFu;
                        if (phidx < L) { prev[j].pos = xyz(lights[phidx]); prev[j].col = xyz(lights[L + phidx]); }
                    } else {
                        sub_load(prev[j], tin.pa, tin.pb, ridx(rg, j, p));
                    }
                    mcur += r[j].M;
                    mprev += prev[j].M;
                }
                const unsigned long long C = (unsigned long long)f.clamp_m * mcur + 1ull;
                if (mprev > C) {
#pragma unroll
                    for (uint32_t j = 0; j < (uint32_t)NT; j++)
                        if (prev[j].M != 0u) prev[j].M = (uint32_t)C;
                }
                const uint32_t pst = pix_state(tin.key, y * rg.W + x);
                Combiner<NT> cmb;
                cmb.init(N);
                if (NT == 1) cmb.consume_pd(pj0, r[0], pst, 0u);
                else for (uint32_t j = 0; j < N; j++) cmb.consume(s, f, px, r[j], pst, 0u);
                for (uint32_t j = 0; j < N; j++) cmb.consume(s, f, px, prev[j], pst, 0u);
                float pd_out[NT > 0 ? NT : 1];
                cmb.finish_biased(s, f, px, NT == 1 ? pd_out : nullptr);
                // the held sample's light index: the predecessor's when the output holds its sample (bit for bit --
                // a light with the current sample's position and colour rebuilds the same sample either way)
                if (NT == 1 && LT == kLtPoint && hw) {
                    const bool same = __float_as_uint(cmb.out[0].pos.x) == __float_as_uint(prev[0].pos.x) &&
                                      __float_as_uint(cmb.out[0].pos.y) == __float_as_uint(prev[0].pos.y) &&
                                      __float_as_uint(cmb.out[0].pos.z) == __float_as_uint(prev[0].pos.z) &&
                                      __float_as_uint(cmb.out[0].col.x) == __float_as_uint(prev[0].col.x) &&
                                      __float_as_uint(cmb.out[0].col.y) == __float_as_uint(prev[0].col.y) &&
                                      __float_as_uint(cmb.out[0].col.z) == __float_as_uint(prev[0].col.z);
                    if (same) hidx = phidx;
                }
                if (NT == 2 && LT == kLtPoint && hw) {
                    // N = 2: each output holds one of the four inputs' samples or the zero sample; its index is that of
                    // an input holding the same (position, colour) bit for bit -- any such index rebuilds the same sample
                    auto same = [](const Sub& a, const Sub& b) {
                        return __float_as_uint(a.pos.x) == __float_as_uint(b.pos.x) &&
                               __float_as_uint(a.pos.y) == __float_as_uint(b.pos.y) &&
                               __float_as_uint(a.pos.z) == __float_as_uint(b.pos.z) &&
                               __float_as_uint(a.col.x) == __float_as_uint(b.col.x) &&
                               __float_as_uint(a.col.y) == __float_as_uint(b.col.y) &&
                               __float_as_uint(a.col.z) == __float_as_uint(b.col.z);
                    };
                    uint32_t oidx[2];
#pragma unroll
                    for (int j = 0; j < 2; j++) {
                        const Sub& o = cmb.out[j];
                        oidx[j] = same(o, prev[0]) ? pidx2[0] : same(o, prev[1]) ? pidx2[1]
                                : same(o, r[0]) ? hidx : same(o, r[1]) ? hidx1 : L;
                    }
                    hidx = oidx[0];
                    hidx1 = oidx[1];
                }
#pragma unroll
                for (uint32_t j = 0; j < (uint32_t)NT; j++) r[j] = cmb.out[j];
                if (NT == 1 && rp) rp[p] = pd_out[0];
            }
        } else if (NT == 1 && rp) {
            rp[p] = target_pdf(s, f, make_px(s, nt, pm, origin, p), r[0].pos, r[0].col, tb);   // no lights: the initial sample
        }
        // store_res = false: the sample handles are the reservoirs' only reader (restir_render's handle passes)
        if (store_res || rdbg)
            for (uint32_t j = 0; j < N; j++) sub_store(r[j], ra, rb, rdbg, ridx(rg, j, p), j * npx + p);
        if (NT == 1 && LT == kLtPoint && hw) { hw[p] = r[0].W; hm[p] = r[0].M | (hidx << 24); }
        if (NT == 2 && LT == kLtPoint && hw)   // N = 2 handle record (W_0, M_0 | i_0 << 24, W_1, M_1 | i_1 << 24)
            reinterpret_cast<float4*>(hw)[p] = make_float4(r[0].W, __uint_as_float(r[0].M | (hidx << 24)), r[1].W,
                                                           __uint_as_float(r[1].M | (hidx1 << 24)));
        if (NT == 1 && LT == kLtRegular && hw)   // grid handle: (W, M | i << 19, a, b) in one float4 plane
            reinterpret_cast<float4*>(hw)[p] = make_float4(r[0].W, __uint_as_float(r[0].M | (hidx << 19)), ha, hb);
    }
}

// k_ris: genCanonicalSamples per pixel.  Lane-serial candidate loop (M iterations) -- VALU bound.  The light
// table is staged into LDS once per persistent block when it fits (LDS_LIGHTS), so the per-candidate random
// light fetch is an LDS read instead of a dependent global load.
// The light table of form LT: the 7-float4 records or the compact (row 0, row 3) table.
template <int LT>
__device__ __forceinline__ const float4* global_lights(const SceneDev& s) {
    return LT == kLtGeneral ? s.lights : LT == kLtPgram ? s.light_c4 : LT == kLtRegular ? s.light_col : s.light_c2;
}
// Stage it into LDS at dst.  No barrier.
template <int LT>
__device__ __forceinline__ void stage_lights(const SceneDev& s, float4* dst) {
    const float4* src = global_lights<LT>(s);
    const uint32_t n = lt_stride(LT) * s.num_lights;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
}

template <int NT, bool LDS_LIGHTS, int LT = kLtGeneral>
__device__ __forceinline__ void ris_body(const SceneDev& s, const Region& rg, const FeaturesDev& f, uint32_t key, v3 origin,
                                         const float4* __restrict__ n_t, const float4* __restrict__ p_mat,
                                         float4* __restrict__ ra, float4* __restrict__ rb, float2* __restrict__ rdbg,
                                         float* __restrict__ rp) {
    const float4* lights = global_lights<LT>(s);
    if (LDS_LIGHTS) {
        stage_lights<LT>(s, g_lds);
        __syncthreads();
        lights = g_lds;
    }
    const Bvh bvh = global_bvh(s);
    const GlTabs tb = gl_stage_tables();
    const uint32_t items = work_items(rg);
    for (uint32_t item = blockIdx.x; item < items; item += gridDim.x) {
        uint32_t x, y;
        size_t p;
        if (!work_pixel(rg, item, x, y, p)) continue;
        ris_pixel<NT, LT>(s, rg, f, key, origin, lights, bvh, n_t[gidx(rg, p)], p_mat[p], x, y, p, ra, rb, rdbg, rp, tb);
    }
}

// k_primary_ris: genPrimaryRayHits and genCanonicalSamples fused (they cover the same region in restir_render):
// the G-buffer records go to memory for the later passes and straight into the pixel's RIS, and the primary
// ray's latency-bound BVH traversal runs beside other waves' VALU-bound candidate loops.  The block stages the
// BVH and, when it fits beside it, the light table in LDS.
template <int NT, bool LDS_LIGHTS, int LT = kLtGeneral, bool TEMP = false>
__device__ __forceinline__ void primary_ris_body(const SceneDev& s, const Region& rg, const CameraDev& cam,
                                                 const FeaturesDev& f, uint32_t key, float4* __restrict__ n_t,
                                                 float4* __restrict__ p_mat, float4* __restrict__ n_t2,
                                                 float4* __restrict__ ra, float4* __restrict__ rb, float2* __restrict__ rdbg,
                                                 float* __restrict__ rp, uint32_t late_ok, uint8_t* __restrict__ tmiss,
                                                 uint32_t skip_res, float* __restrict__ hw, uint32_t* __restrict__ hm,
                                                 uint32_t res_dead, TemporalIn tin = TemporalIn{nullptr, nullptr, 0u}) {
    const uint32_t bvh_f4 = 2u * s.num_nodes + 3u * s.num_tris;
    const float4* lights = global_lights<LT>(s);
    const uint32_t items = work_items(rg);
    // One tile per block: the light table is staged after the primary rays, and only if one of the tile's pixels will
    // run the candidate loop (ris_pixel's miss test) -- at C4 / C5 87 % of the tiles see only background.  The same
    // vote is the tile's MissTiles flag (tmiss, one byte per tile; the launcher passes it only for one tile per block).
    const bool one = gridDim.x >= items;
    const bool late = LDS_LIGHTS && (late_ok & 1u) && one;   // late_ok bit 1: primary.tl (tile_triangles)
    if (LDS_LIGHTS) {
        if (!late) stage_lights<LT>(s, g_lds + bvh_f4);
        lights = g_lds + bvh_f4;
    }
    // primary.tl (late_ok bit 1): the tile's candidate triangles, published by the staging barrier below
    __shared__ uint16_t s_tl[kTlMaxTris];
    __shared__ uint32_t s_tlc[4];
    const bool tl = (late || (one && tmiss)) && (late_ok & 2u) && rg.map2d && s.num_tris <= kTlMaxTris &&
                    blockIdx.x < items && cam.half_w > 0.0f && cam.half_h > 0.0f;   // block-uniform
    if (tl) {
        const uint32_t ntx = (rg.rw + kTileW - 1) / kTileW;
        const int tx0 = (int)(rg.rx0 + (blockIdx.x % ntx) * kTileW), ty0 = (int)(rg.ry0 + (blockIdx.x / ntx) * kTileH);
        const int tx1 = min(tx0 + (int)kTileW, (int)(rg.rx0 + rg.rw)) - 1, ty1 = min(ty0 + (int)kTileH, (int)(rg.ry0 + rg.rh)) - 1;
        tile_triangles(s, rg, cam, tx0, tx1, ty0, ty1, s_tl, s_tlc);
    }
    // ends with the barrier that also covers the light copy (and the lists); the nodes only for rays that walk them
    const Bvh bvh = stage_bvh(s, g_lds, !tl || f.initial_vis);
    const GlTabs tb = gl_stage_tables();
    const v3 origin = mk(cam.origin[0], cam.origin[1], cam.origin[2]);
    if (late || (one && tmiss)) {
        if (blockIdx.x >= items) return;   // block-uniform
        uint32_t x, y;
        size_t p;
        const bool live = work_pixel(rg, blockIdx.x, x, y, p);
        float4 nt = make_float4(0.0f, 0.0f, 0.0f, 0.0f), pm = nt;
        const bool skip_gbuf = tmiss && (skip_res & 2u);   // bit 1: a background tile's G-buffer records too
        if (live) primary_pixel(s, rg, cam, bvh, x, y, p, n_t2, n_t, p_mat, nt, pm, !skip_gbuf, tl ? s_tl : nullptr, s_tlc);
        uint32_t m = __float_as_uint(pm.w);
        if (m >= s.num_materials) m = s.num_materials - 1u;
        const bool loop = live && s.num_lights != 0u &&
                          !(m == s.num_materials - 1u && s.lights_finite && !__builtin_isnan(pm.x + pm.y + pm.z));
        const bool any = __syncthreads_or(loop);
        // flag 0: every live pixel is a miss with the known RIS result (lights present: no loop means a known miss)
        if (tmiss && threadIdx.x == 0) tmiss[blockIdx.x] = (s.num_lights == 0u || any) ? 1u : 0u;
        if (skip_gbuf && live && any) {
            n_t[gidx(rg, p)] = nt;
            if (n_t2) n_t2[gidx(rg, p)] = nt;
            p_mat[p] = pm;
        }
        // TEMP with frame handles: a pixel that misses now may hold a predecessor whose handle names a real light (the
        // camera moved), rebuilt from this table -- staged for every tile then
        if (late && (any || (TEMP && tin.hw != nullptr))) {
            stage_lights<LT>(s, g_lds + bvh_f4);
            __syncthreads();
        }
        // skip_res (the launcher's promise that no reader needs them): bit 0, a background tile's known reservoirs and
        // pdfs are not stored -- the first spatial pass substitutes them from the flag; bit 1 (above), nor its G-buffer
        // records (a single unbiased pass, which substitutes those too)
        if (live && (any || !tmiss || !(skip_res & 1u)))
            ris_pixel<NT, LT, TEMP>(s, rg, f, key, origin, lights, bvh, nt, pm, x, y, p, ra, rb, rdbg, rp, tb, hw, hm,
                                    !(hw && res_dead), tin);
        return;
    }
    for (uint32_t item = blockIdx.x; item < items; item += gridDim.x) {
        uint32_t x, y;
        size_t p;
        if (!work_pixel(rg, item, x, y, p)) continue;
        float4 nt, pm;
        primary_pixel(s, rg, cam, bvh, x, y, p, n_t2, n_t, p_mat, nt, pm);
        ris_pixel<NT, LT, TEMP>(s, rg, f, key, origin, lights, bvh, nt, pm, x, y, p, ra, rb, rdbg, rp, tb, hw, hm,
                                !(hw && res_dead), tin);
    }
}

// RIS: capped at 96 VGPRs = 5 waves per SIMD (uncapped the allocator takes 100 = 4 waves; 5 waves run the
// latency-bound candidate loop 9 % faster, 6 waves spilled -- scripts/ablate.py, profiles/r1).  N = 2 the same:
// k_primary_ris_n2_lds 407 -> 381 us at C2 N = 2 (profiles/r3/r3_configs/n2_*_c2.json).  Round 4: with the accepted
// candidate kept as an index (ris_pixel) the N = 1 kernels fit 80 VGPRs without spilling, and 6 waves per SIMD run
// C2 RIS 319.5 -> 305.8 us, C4 379.6 -> 370.3, C5 2161 -> 2086 (cfg_kbench, profiles/r4/r4c).  (The unfused
// k_ris_n1_lds_{grid,reg,pg} would spill 12 B at 6 and keep 5.)
#ifndef ROMIS_RIS_WPE
#define ROMIS_RIS_WPE 5
#endif
#ifndef ROMIS_RIS1_WPE
#define ROMIS_RIS1_WPE 7   // round 4: 7 (72 VGPRs, 20-24 B of spills) beats 6 at C2 by 2.8 % (profiles/r4/r4n)
#endif
#define ROMIS_RIS_ATTR __attribute__((amdgpu_waves_per_eu(ROMIS_RIS_WPE)))
#define ROMIS_RIS1_ATTR __attribute__((amdgpu_waves_per_eu(ROMIS_RIS1_WPE)))
#define ROMIS_RIS_KERNEL_LT(NT, LDS, LT, NAME, ATTR)                                                                  \
    extern "C" __global__ __launch_bounds__(256) ATTR void NAME(SceneDev s, Region rg, FeaturesDev f, uint32_t key, float ox, \
                                                          float oy, float oz, const float4* n_t, const float4* p_mat,   \
                                                          float4* ra, float4* rb, float2* rdbg, float* rp) {           \
        ris_body<NT, LDS, LT>(s, rg, f, key, mk(ox, oy, oz), n_t, p_mat, ra, rb, rdbg, rp);                             \
    }
#define ROMIS_RIS_KERNEL(NT, LDS, NAME, ATTR) ROMIS_RIS_KERNEL_LT(NT, LDS, kLtGeneral, NAME, ATTR)
ROMIS_RIS_KERNEL(1, false, k_ris_n1, ROMIS_RIS1_ATTR)
ROMIS_RIS_KERNEL(2, false, k_ris_n2, ROMIS_RIS_ATTR)
ROMIS_RIS_KERNEL(0, false, k_ris_n0, )
ROMIS_RIS_KERNEL(1, true, k_ris_n1_lds, ROMIS_RIS1_ATTR)
ROMIS_RIS_KERNEL(2, true, k_ris_n2_lds, ROMIS_RIS_ATTR)
ROMIS_RIS_KERNEL(0, true, k_ris_n0_lds, )
ROMIS_RIS_KERNEL_LT(1, true, kLtPoint, k_ris_n1_lds_pt, ROMIS_RIS1_ATTR)
ROMIS_RIS_KERNEL_LT(2, true, kLtPoint, k_ris_n2_lds_pt, ROMIS_RIS_ATTR)
ROMIS_RIS_KERNEL_LT(1, false, kLtPoint, k_ris_n1_pt, ROMIS_RIS1_ATTR)
ROMIS_RIS_KERNEL_LT(2, false, kLtPoint, k_ris_n2_pt, ROMIS_RIS_ATTR)
ROMIS_RIS_KERNEL_LT(1, true, kLtGrid, k_ris_n1_lds_grid, ROMIS_RIS_ATTR)
ROMIS_RIS_KERNEL_LT(2, true, kLtGrid, k_ris_n2_lds_grid, ROMIS_RIS_ATTR)
ROMIS_RIS_KERNEL_LT(1, false, kLtGrid, k_ris_n1_grid, ROMIS_RIS1_ATTR)
ROMIS_RIS_KERNEL_LT(2, false, kLtGrid, k_ris_n2_grid, ROMIS_RIS_ATTR)
ROMIS_RIS_KERNEL_LT(1, false, kLtRegular, k_ris_n1_reg, ROMIS_RIS1_ATTR)
ROMIS_RIS_KERNEL_LT(1, true, kLtRegular, k_ris_n1_lds_reg, ROMIS_RIS_ATTR)
ROMIS_RIS_KERNEL_LT(1, true, kLtPgram, k_ris_n1_lds_pg, ROMIS_RIS_ATTR)
ROMIS_RIS_KERNEL_LT(2, true, kLtPgram, k_ris_n2_lds_pg, ROMIS_RIS_ATTR)
ROMIS_RIS_KERNEL_LT(1, false, kLtPgram, k_ris_n1_pg, ROMIS_RIS1_ATTR)
ROMIS_RIS_KERNEL_LT(2, false, kLtPgram, k_ris_n2_pg, ROMIS_RIS_ATTR)

#define ROMIS_PRIMARY_RIS_KERNEL_LT(NT, LDS, LT, NAME, ATTR)                                                           \
    extern "C" __global__ __launch_bounds__(256) ATTR void NAME(SceneDev s, Region rg, CameraDev cam, FeaturesDev f,   \
                                                          uint32_t key, float4* n_t, float4* p_mat, float4* n_t2,      \
                                                          float4* ra, float4* rb, float2* rdbg, float* rp,             \
                                                          uint32_t late_ok, uint8_t* tmiss, uint32_t skip_res,         \
                                                          float* hw, uint32_t* hm, uint32_t res_dead) {                \
        primary_ris_body<NT, LDS, LT>(s, rg, cam, f, key, n_t, p_mat, n_t2, ra, rb, rdbg, rp, late_ok, tmiss, skip_res,   \
                                      hw, hm, res_dead);                                                               \
    }
#define ROMIS_PRIMARY_RIS_KERNEL(NT, LDS, NAME, ATTR) ROMIS_PRIMARY_RIS_KERNEL_LT(NT, LDS, kLtGeneral, NAME, ATTR)
// primary rays + RIS + temporal reuse in one kernel (point lights, the table in LDS): restir_render with a predecessor
#define ROMIS_PRIMARY_RIS_TEMPORAL_KERNEL(NT, NAME, ATTR)                                                              \
    extern "C" __global__ __launch_bounds__(256) ATTR void NAME(SceneDev s, Region rg, CameraDev cam, FeaturesDev f,   \
                                                          uint32_t key, float4* n_t, float4* p_mat, float4* n_t2,      \
                                                          float4* ra, float4* rb, float2* rdbg, float* rp,             \
                                                          uint32_t late_ok, TemporalIn tin, float* hw, uint32_t* hm,   \
                                                          uint32_t res_dead) {                                         \
        primary_ris_body<NT, true, kLtPoint, true>(s, rg, cam, f, key, n_t, p_mat, n_t2, ra, rb, rdbg, rp, late_ok,    \
                                                   nullptr, 0u, hw, hm, res_dead, tin);                                \
    }
ROMIS_PRIMARY_RIS_KERNEL(1, true, k_primary_ris_n1_lds, ROMIS_RIS1_ATTR)
ROMIS_PRIMARY_RIS_KERNEL(1, false, k_primary_ris_n1, ROMIS_RIS1_ATTR)
ROMIS_PRIMARY_RIS_KERNEL(2, true, k_primary_ris_n2_lds, ROMIS_RIS_ATTR)
ROMIS_PRIMARY_RIS_KERNEL(2, false, k_primary_ris_n2, ROMIS_RIS_ATTR)
ROMIS_PRIMARY_RIS_KERNEL(0, true, k_primary_ris_n0_lds, )
ROMIS_PRIMARY_RIS_KERNEL(0, false, k_primary_ris_n0, )
ROMIS_PRIMARY_RIS_KERNEL_LT(1, true, kLtPoint, k_primary_ris_n1_lds_pt, ROMIS_RIS1_ATTR)
ROMIS_PRIMARY_RIS_KERNEL_LT(2, true, kLtPoint, k_primary_ris_n2_lds_pt, ROMIS_RIS_ATTR)
ROMIS_PRIMARY_RIS_KERNEL_LT(1, false, kLtPoint, k_primary_ris_n1_pt, ROMIS_RIS1_ATTR)
ROMIS_PRIMARY_RIS_KERNEL_LT(2, false, kLtPoint, k_primary_ris_n2_pt, ROMIS_RIS_ATTR)
ROMIS_PRIMARY_RIS_KERNEL_LT(1, true, kLtGrid, k_primary_ris_n1_lds_grid, ROMIS_RIS1_ATTR)
ROMIS_PRIMARY_RIS_KERNEL_LT(2, true, kLtGrid, k_primary_ris_n2_lds_grid, ROMIS_RIS_ATTR)
ROMIS_PRIMARY_RIS_KERNEL_LT(1, false, kLtGrid, k_primary_ris_n1_grid, ROMIS_RIS1_ATTR)
ROMIS_PRIMARY_RIS_KERNEL_LT(2, false, kLtGrid, k_primary_ris_n2_grid, ROMIS_RIS_ATTR)
ROMIS_PRIMARY_RIS_KERNEL_LT(1, false, kLtRegular, k_primary_ris_n1_reg, ROMIS_RIS1_ATTR)
ROMIS_PRIMARY_RIS_KERNEL_LT(1, true, kLtRegular, k_primary_ris_n1_lds_reg, ROMIS_RIS1_ATTR)
ROMIS_PRIMARY_RIS_KERNEL_LT(1, true, kLtPgram, k_primary_ris_n1_lds_pg, ROMIS_RIS1_ATTR)
ROMIS_PRIMARY_RIS_KERNEL_LT(2, true, kLtPgram, k_primary_ris_n2_lds_pg, ROMIS_RIS_ATTR)
ROMIS_PRIMARY_RIS_KERNEL_LT(1, false, kLtPgram, k_primary_ris_n1_pg, ROMIS_RIS1_ATTR)
ROMIS_PRIMARY_RIS_KERNEL_LT(2, false, kLtPgram, k_primary_ris_n2_pg, ROMIS_RIS_ATTR)
ROMIS_PRIMARY_RIS_TEMPORAL_KERNEL(1, k_primary_ris_n1_lds_pt_temporal, ROMIS_RIS1_ATTR)
ROMIS_PRIMARY_RIS_TEMPORAL_KERNEL(2, k_primary_ris_n2_lds_pt_temporal, ROMIS_RIS_ATTR)

// k_temporal: temporalReuse (render_utils.cpp:142-177).  cur = (ca, cb), prev = (pa, pb); writes (oa, ob).
template <int NT>
__device__ __forceinline__ void temporal_body(const SceneDev& s, const Region& rg, const FeaturesDev& f, uint32_t key,
                                              v3 origin, const float4* __restrict__ n_t, const float4* __restrict__ p_mat,
                                              const float4* ca, const float4* cb, const float4* __restrict__ pa,
                                              const float4* __restrict__ pb, float4* oa, float4* ob, float2* odbg,
                                              const float* rp_in, float* rp_out) {
    uint32_t x, y;
    size_t p;
    if (!region_pixel(rg, blockIdx.x * blockDim.x + threadIdx.x, x, y, p)) return;
    const size_t npx = (size_t)rg.vw * rg.vh;
    const uint32_t N = NT > 0 ? (uint32_t)NT : f.N;
    Px px = load_px(s, rg, n_t, p_mat, p, origin);
    Sub cur[NT > 0 ? NT : RESTIR_MAX_N_DEV], prev[NT > 0 ? NT : RESTIR_MAX_N_DEV];
    unsigned long long mcur = 0, mprev = 0;
    for (uint32_t j = 0; j < N; j++) {
        sub_load(cur[j], ca, cb, ridx(rg, j, p));
        sub_load(prev[j], pa, pb, ridx(rg, j, p));
        mcur += cur[j].M;
        mprev += prev[j].M;
    }
    unsigned long long C = (unsigned long long)f.clamp_m * mcur + 1ull;
    if (mprev > C) {
        for (uint32_t j = 0; j < N; j++)
            if (prev[j].M != 0u) prev[j].M = (uint32_t)C;   // wSum scaling: never read by combineBiased
    }
    const uint32_t ps = pix_state(key, y * rg.W + x);
    Combiner<NT> cmb;
    cmb.init(N);
    // N = 1 with the pdf cache: the current reservoir's target pdf here is the one its producer stored
    if (NT == 1 && rp_in) cmb.consume_pd(rp_in[p], cur[0], ps, 0u);
    else for (uint32_t j = 0; j < N; j++) cmb.consume(s, f, px, cur[j], ps, 0u);
    for (uint32_t j = 0; j < N; j++) cmb.consume(s, f, px, prev[j], ps, 0u);
    float pd_out[NT > 0 ? NT : 1];
    cmb.finish_biased(s, f, px, NT == 1 ? pd_out : nullptr);
    for (uint32_t j = 0; j < N; j++) sub_store(cmb.out[j], oa, ob, odbg, ridx(rg, j, p), j * npx + p);
    if (NT == 1 && rp_out) rp_out[p] = pd_out[0];
}

// register cap of the temporal kernels (build variants; unset = the compiler's choice)
#ifdef ROMIS_TEMPORAL_WPE
#define ROMIS_TEMPORAL_ATTR __attribute__((amdgpu_waves_per_eu(ROMIS_TEMPORAL_WPE)))
#else
#define ROMIS_TEMPORAL_ATTR
#endif
#define ROMIS_TEMPORAL_KERNEL(NT)                                                                                      \
    extern "C" __global__ __launch_bounds__(256) ROMIS_TEMPORAL_ATTR void k_temporal_n##NT(                           \
        SceneDev s, Region rg, FeaturesDev f, uint32_t key, float ox, float oy, float oz, const float4* n_t,          \
        const float4* p_mat, const float4* ca, const float4* cb, const float4* pa, const float4* pb, float4* oa,      \
        float4* ob, float2* odbg, const float* rp_in, float* rp_out) {                                                \
        temporal_body<NT>(s, rg, f, key, mk(ox, oy, oz), n_t, p_mat, ca, cb, pa, pb, oa, ob, odbg, rp_in, rp_out);    \
    }
ROMIS_TEMPORAL_KERNEL(1)
ROMIS_TEMPORAL_KERNEL(2)
ROMIS_TEMPORAL_KERNEL(0)

// ---------------------------------------------------------------------------------------------------------
// k_spatial: one spatialReuse pass.  Neighbours stream straight into the combine (accepted neighbours in draw
// order, current last -- render_utils.cpp:108-124), so no per-lane candidate list is kept.  The neighbour
// draws do not depend on data, so the loads of a batch of kBatch neighbours are all issued before the first
// is consumed (one memory latency per batch instead of a dependent chain per neighbour).
#ifndef ROMIS_SPATIAL_BATCH
#define ROMIS_SPATIAL_BATCH 5
#endif
constexpr uint32_t kBatch = ROMIS_SPATIAL_BATCH;

template <int NT, bool UNBIASED>
__device__ __forceinline__ void spatial_pixel(const SceneDev& s, const Region& rg, const FeaturesDev& f, uint32_t key,
                                              v3 origin, const float4* __restrict__ n_t, const float4* __restrict__ p_mat,
                                              const float4* __restrict__ ia, const float4* __restrict__ ib,
                                              float4* __restrict__ oa, float4* __restrict__ ob, float2* __restrict__ odbg,
                                              uint32_t x, uint32_t y, size_t p, const Bvh& bvh) {
    const size_t npx = (size_t)rg.vw * rg.vh;
    const uint32_t N = NT > 0 ? (uint32_t)NT : f.N;
    const uint32_t K = f.K;
    const Px cur = load_px(s, rg, n_t, p_mat, p, origin);
    const uint32_t ps = pix_state(key, y * rg.W + x);
    const uint32_t slot0 = 2u * K;
    Combiner<NT> cmb;
    cmb.init(N);
    for (uint32_t n0 = 0; n0 < K; n0 += kBatch) {
        uint32_t q[kBatch];
        float4 g[kBatch];
        bool ok[kBatch];
#pragma unroll
        for (uint32_t i = 0; i < kBatch; i++) {
            const uint32_t n = n0 + i;
            q[i] = (uint32_t)p;
            if (n < K)
                q[i] = (uint32_t)neighbour_index(rg, x, y, uniform_offset(draw(ps, 2u * n), f.R),
                                       uniform_offset(draw(ps, 2u * n + 1u), f.R));
        }
        if constexpr (!UNBIASED) {
#pragma unroll
            for (uint32_t i = 0; i < kBatch; i++) g[i] = n_t[gidx(rg, q[i])];
        }
#pragma unroll
        for (uint32_t i = 0; i < kBatch; i++) {
            ok[i] = n0 + i < K;
            if (!UNBIASED && ok[i]) {   // render_utils.cpp:114-118
                float depthFracDiff = fabsf(1.0f - (g[i].w / cur.t));
                float normalsDotProd = vdot(xyz(g[i]), cur.N);
                if (depthFracDiff > 0.1f || normalsDotProd < 0.90630778703f) ok[i] = false;
            }
        }
        if constexpr (NT == 1) {
            float4 a[kBatch], b[kBatch];
#pragma unroll
            for (uint32_t i = 0; i < kBatch; i++) {
                if (ok[i]) { a[i] = ia[gidx(rg, q[i])]; b[i] = ib[gidx(rg, q[i])]; }
            }
            // consume in draw order with ONE inlined combine body: the batch is shifted down a register per
            // step (static indices only; a rolled loop over a[i] would spill the batch to memory)
#pragma unroll 1
            for (uint32_t i = 0; i < kBatch; i++) {
                if (ok[0]) cmb.consume(s, f, cur, sub_from(a[0], b[0]), ps, slot0);
#pragma unroll
                for (uint32_t j = 0; j + 1 < kBatch; j++) { a[j] = a[j + 1]; b[j] = b[j + 1]; ok[j] = ok[j + 1]; }
            }
        } else {
#pragma unroll
            for (uint32_t i = 0; i < kBatch; i++) {
                if (!ok[i]) continue;
                for (uint32_t j = 0; j < N; j++) {
                    Sub in;
                    sub_load(in, ia, ib, ridx(rg, j, q[i]));
                    cmb.consume(s, f, cur, in, ps, slot0);
                }
            }
        }
    }
    for (uint32_t j = 0; j < N; j++) {
        Sub in;
        sub_load(in, ia, ib, ridx(rg, j, p));
        cmb.consume(s, f, cur, in, ps, slot0);
    }
    if (!UNBIASED) {
        cmb.finish_biased(s, f, cur);
    } else {
        // combineUnbiased (reservoir.cpp:84-103): Z_j = sum over the stream of the input's total M where
        // p_r(y_j) [* vis_r(y_j)] > 0.  The stream is re-derived from the same draws (no rejection here).
        // p * vis > 0 needs p > 0 whatever vis is (p is a length: >= 0 or NaN), so the shadow ray is cast only then.
        for (uint32_t j = 0; j < N; j++) cmb.out[j].M = cmb.macc[j];
        unsigned long long Z[NT > 0 ? NT : RESTIR_MAX_N_DEV];
        for (uint32_t j = 0; j < N; j++) Z[j] = 0ull;
        for (uint32_t n = 0; n <= K; n++) {
            size_t q = p;
            if (n < K) q = neighbour_index(rg, x, y, uniform_offset(draw(ps, 2u * n), f.R),
                                           uniform_offset(draw(ps, 2u * n + 1u), f.R));
            Px rp = load_px(s, rg, n_t, p_mat, q, origin);
            unsigned long long tot = 0;
            for (uint32_t j = 0; j < N; j++) tot += __float_as_uint(ib[ridx(rg, j, q)].w);
            for (uint32_t j = 0; j < N; j++) {
                if (target_pdf_positive(s, f, rp, cmb.out[j].pos, cmb.out[j].col, gl_global_tabs()) &&
                    (!f.spatial_vis || visible(bvh, rp.P, cmb.out[j].pos)))
                    Z[j] += tot;
            }
        }
        for (uint32_t j = 0; j < N; j++) {
            float pc = cmb.out[j].has_pd ? cmb.out[j].pd : target_pdf(s, f, cur, cmb.out[j].pos, cmb.out[j].col);
            if (pc == 0.0f || Z[j] == 0ull) cmb.out[j].W = 0.0f;
            else cmb.out[j].W = (rcp_rn(pc) * rcp_rn((float)Z[j])) * cmb.out[j].wsum;
        }
    }
    for (uint32_t j = 0; j < N; j++) sub_store(cmb.out[j], oa, ob, odbg, ridx(rg, j, p), j * npx + p);
}

template <int NT, bool UNBIASED>
__device__ __forceinline__ void spatial_body(const SceneDev& s, const Region& rg, const FeaturesDev& f, uint32_t key,
                                             v3 origin, const float4* __restrict__ n_t, const float4* __restrict__ p_mat,
                                             const float4* __restrict__ ia, const float4* __restrict__ ib,
                                             float4* __restrict__ oa, float4* __restrict__ ob, float2* __restrict__ odbg,
                                             uint32_t bvh_lds) {
    // unbiased combine with visibility reuse casts (k+1) N shadow rays per pixel: the block stages the BVH in
    // LDS first (every thread reaches this: bvh_lds is uniform over the launch)
    Bvh bvh = global_bvh(s);
    if (UNBIASED && bvh_lds) bvh = stage_bvh(s, g_lds);
    const uint32_t T = work_items(rg);
    if (!rg.map2d) {
        for (uint32_t item = blockIdx.x; item < T; item += gridDim.x) {
            uint32_t x, y;
            size_t p;
            if (work_pixel(rg, item, x, y, p))
                spatial_pixel<NT, UNBIASED>(s, rg, f, key, origin, n_t, p_mat, ia, ib, oa, ob, odbg, x, y, p, bvh);
        }
        return;
    }
    // XCD-banded tile order (see xcd_banded_tile): the blocks of XCD b % 8 sweep that XCD's contiguous band
    const uint32_t nb = gridDim.x, b = blockIdx.x, xcd = b % 8u;
    const uint32_t xcd_blocks = nb / 8u + (xcd < nb % 8u ? 1u : 0u);
    const uint32_t q = T / 8u, rem = T % 8u;
    const uint32_t band0 = xcd * q + min(xcd, rem), band_len = q + (xcd < rem ? 1u : 0u);
    for (uint32_t t = b / 8u; t < band_len; t += xcd_blocks) {
        uint32_t x, y;
        size_t p;
        if (work_pixel(rg, band0 + t, x, y, p))
            spatial_pixel<NT, UNBIASED>(s, rg, f, key, origin, n_t, p_mat, ia, ib, oa, ob, odbg, x, y, p, bvh);
    }
}

// Waves per SIMD the register allocator must leave room for (VGPRs <= 512 / waves).  Spatial: without the
// cap the allocator settles at 129 VGPRs = 3 waves; capped at 4 (128) it runs 12 % faster (ablate.py).
#ifndef ROMIS_SPATIAL_WPE
#define ROMIS_SPATIAL_WPE 4
#endif
#define ROMIS_SPATIAL_ATTR __attribute__((amdgpu_waves_per_eu(ROMIS_SPATIAL_WPE)))
#define ROMIS_SPATIAL_KERNEL(NT, UB, NAME)                                                                             \
    extern "C" __global__ __launch_bounds__(256) ROMIS_SPATIAL_ATTR void NAME(SceneDev s, Region rg, FeaturesDev f, uint32_t key, float ox, \
                                                          float oy, float oz, const float4* n_t, const float4* p_mat,    \
                                                          const float4* ia, const float4* ib, float4* oa, float4* ob,   \
                                                          float2* odbg, uint32_t bvh_lds) {                             \
        spatial_body<NT, UB>(s, rg, f, key, mk(ox, oy, oz), n_t, p_mat, ia, ib, oa, ob, odbg, bvh_lds);                          \
    }
ROMIS_SPATIAL_KERNEL(1, false, k_spatial_n1_biased)
ROMIS_SPATIAL_KERNEL(2, false, k_spatial_n2_biased)
ROMIS_SPATIAL_KERNEL(0, false, k_spatial_n0_biased)
ROMIS_SPATIAL_KERNEL(1, true, k_spatial_n1_unbiased)
ROMIS_SPATIAL_KERNEL(2, true, k_spatial_n2_unbiased)
ROMIS_SPATIAL_KERNEL(0, true, k_spatial_n0_unbiased)

// ---------------------------------------------------------------------------------------------------------
// The lean N = 1 / 2 passes (k_spatial1_ntl, k_spatial1h, k_spatial2_ntl, k_spatial1u): the arithmetic and RNG slots of
// spatial_pixel, laid out for a short VALU stream -- 32-bit byte offsets from the plane bases, neighbour clamping by
// v_med3, one shared double reciprocal of the pixel's depth for the depth tests, a fully unrolled consume sequence
// behind branches the wave skips when no lane accepted that neighbour.  SoA planes (Region ps = 1), K <= kLeanK.
constexpr uint32_t kLeanK = 5;

template <class T>
__device__ __forceinline__ T ld_at(const T* __restrict__ base, uint32_t byte_ofs) {
    return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + byte_ofs);
}
template <class T>
__device__ __forceinline__ void st_at(T* __restrict__ base, uint32_t byte_ofs, T v) {
    *reinterpret_cast<T*>(reinterpret_cast<char*>(base) + byte_ofs) = v;
}

// Combine state of one output sub-reservoir (N = 1): Reservoir::update (reservoir.cpp:10-32) without the M
// increment (combineBiased replaces M by the routed sum, reservoir.cpp:55-57).
struct Comb1 {
    v3 pos, col;
    float wsum, chosen, pd;
    uint32_t macc;
    bool has_pd;
    uint32_t h;   // ps + slot * 0x9E3779B9 of the next accept draw
    // returns whether the input's sample was accepted
    __device__ __forceinline__ bool take(float pd_in, float W, uint32_t M, v3 p, v3 c) {
        const float w = (pd_in * W) * (float)M;          // reservoir.cpp:50
        macc += M;
        wsum += w;
        const float u = rand01(mix32(h));
        h += 0x9E3779B9u;
        const bool acc = accept_u(u, w, wsum);
        if (acc) { pos = p; col = c; chosen = w; pd = pd_in; has_pd = true; }
        return acc;
    }
};

// Light-grid sample handles (round 5; SceneDev::lights_regular, the reference's regularLightGrid with RIS's kLtRegular
// form): a sample is a point of light i's parallelogram at the fractions (a, b) of its two RIS draws, its colour mixed
// at a and b -- a function of (i, a, b).  The handle is one float4 plane, (W, bits(M | i << 19), a, b): 16 B per pixel
// instead of the reservoir's 32, index L the initial (0, 0) sample.
constexpr uint32_t kHandleMG = 0x0007FFFFu;
// the (position, colour) of grid sample (i, a, b), evaluated as kLtRegular's sample_reg (ris_pixel) does; col_tab = the
// light colours (light_col or an LDS copy)
__device__ __forceinline__ void grid_sample(const SceneDev& s, const float4* __restrict__ col_tab, uint32_t i, float a,
                                            float b, v3& pos, v3& col) {
    const bool zero = i >= s.num_lights;
    const uint32_t j = zero ? 0u : i;
    const float xl = (float)(j >> s.grid_ny_log2), yl = (float)(j & ((1u << s.grid_ny_log2) - 1u));
    const v3 v0 = vadd(vadd(xyz(s.grid_start), vscale(xyz(s.grid_s01), xl)), vscale(xyz(s.grid_s02), yl));
    const v3 p = vadd(vadd(v0, vscale(xyz(s.lights[1]), a)), vscale(xyz(s.lights[2]), b));
    const v3 gc = xyz(col_tab[j]);
    const v3 m = vmix(gc, gc, a);
    const v3 c = vmix(m, m, b);
    pos = zero ? mk(0.0f, 0.0f, 0.0f) : p;
    col = zero ? mk(0.0f, 0.0f, 0.0f) : c;
}

#ifndef ROMIS_TAB_DMA
#define ROMIS_TAB_DMA 1   // the biased passes stage powf's tables by LDS-DMA behind their own loads (gl_stage_tables_dma)
#endif
#ifndef ROMIS_FLAG_SMEM
#define ROMIS_FLAG_SMEM 1   // a block's single background-tile flag through the scalar cache (tiles_known_miss)
#endif
// Tile of block b (XCD b % 8, block b runs on XCD b % 8): XCD x owns every 8th chunk of rg.xcd_rows tile
// rows (chunks x, x + 8, x + 16, ...), walked row-major, so its L2 holds the chunk's G-buffer and reservoirs
// while the neighbourhoods reach 10 px across tile borders; interleaving short chunks spreads cheap (background)
// and expensive rows evenly over the XCDs -- contiguous bands left the background XCDs idle (1.28x the mean
// work on the busiest XCD at C2, 1.02x with 2-row chunks).  rg.xcd_rows = 0: one contiguous band per XCD.
// (Round 5: splitting the last, partial round of chunks evenly over the XCDs instead measured no faster -- C2
// handle pass 67.2 vs 66.8 us, the n_t-window pass with 2-D chunks 74.5 vs 70.6, C4f 431 vs 434; profiles/r5.)
__device__ __forceinline__ bool xcd_tile(const Region& rg, uint32_t T, uint32_t b, uint32_t& tile) {
    const uint32_t x = b % 8u, j = b / 8u;
    if (rg.xcd_rows == 0u) {
        const uint32_t q = T / 8u, rem = T % 8u;
        tile = x * q + min(x, rem) + j;
        return j < q + (x < rem ? 1u : 0u);
    }
    const uint32_t ntx = (rg.rw + kTileW - 1) / kTileW;
    if (rg.xcd_cols == 0u || rg.xcd_cols >= ntx) {
        const uint32_t chunk = rg.xcd_rows * ntx;
        const uint32_t i = j / chunk;
        tile = ((x + 8u * i) * rg.xcd_rows) * ntx + (j - i * chunk);
        return tile < T;
    }
    // 2-D chunks of xcd_rows x xcd_cols tiles, numbered row-major over the image; XCD x takes chunks x, x + 8, ...
    const uint32_t cw = rg.xcd_cols, ncx = (ntx + cw - 1u) / cw, chunk = rg.xcd_rows * cw;
    const uint32_t i = j / chunk, k = j - i * chunk, c = x + 8u * i;
    const uint32_t cr = c / ncx, tr = k / cw;
    const uint32_t col = (c - cr * ncx) * cw + (k - tr * cw);
    tile = (cr * rg.xcd_rows + tr) * ntx + col;
    return col < ntx && tile < T;
}

// Blocks for xcd_tile's order over ntx x nty tiles (rg.xcd_rows, rg.xcd_cols set): every XCD gets as many as the one
// that owns the most chunks.
inline uint32_t xcd_grid(const Region& rg, uint32_t ntx, uint32_t nty) {
    if (rg.xcd_rows == 0u) return ntx * nty;
    const uint32_t cw = (rg.xcd_cols == 0u || rg.xcd_cols >= ntx) ? ntx : rg.xcd_cols;
    const uint32_t chunks = ((nty + rg.xcd_rows - 1u) / rg.xcd_rows) * ((ntx + cw - 1u) / cw);
    return 8u * ((chunks + 7u) / 8u) * rg.xcd_rows * cw;
}

// MissTiles (restir_types.h): every RIS tile (32 x 8, numbered row-major over the view) meeting the pixel rect
// [x0, x1] x [y0, y1] (global coordinates inside the view) is a background tile.  Block-uniform; the flags of the
// rect's tile rows are OR-ed without early exits so their loads issue together.
__device__ __forceinline__ bool tiles_known_miss(const MissTiles& mt, const Region& rg, int x0, int x1, int y0, int y1,
                                                 bool* some_known = nullptr) {
    const uint32_t ntxv = (rg.vw + kTileW - 1u) / kTileW;
    const uint32_t cx0 = (uint32_t)(x0 - (int)rg.vx0) / kTileW, cx1 = (uint32_t)(x1 - (int)rg.vx0) / kTileW;
    const uint32_t cy0 = (uint32_t)(y0 - (int)rg.vy0) / kTileH, cy1 = (uint32_t)(y1 - (int)rg.vy0) / kTileH;
    if (ROMIS_FLAG_SMEM && cx0 == cx1 && cy0 == cy1) {
        // one RIS tile (the biased pass's 32 x 8 tiles on the RIS grid): its flag's word by a scalar load -- the address
        // is block-uniform and the flags were written by an earlier kernel (the launcher rounds the buffer to words)
        const uint32_t c = cy0 * ntxv + cx0;
        const auto* w = (const __attribute__((address_space(4))) uint32_t*)(mt.flags + (c & ~3u));
        const uint32_t v = (*w >> (8u * (c & 3u))) & 0xFFu;
        if (some_known) *some_known = v == 0u;
        return v == 0u;
    }
    uint32_t any = 0u, all = 1u;
    for (uint32_t cy = cy0; cy <= cy1; cy++)
        for (uint32_t cx = cx0; cx <= cx1; cx++) {
            const uint32_t v = mt.flags[cy * ntxv + cx];
            any |= v;
            all &= v;
        }
    if (some_known) *some_known = all == 0u;   // some tile of the rect is a background tile
    return any == 0u;
}
// the flag of the RIS tile holding view pixel (x, y) (global coordinates)
__device__ __forceinline__ uint32_t tile_flag_at(const MissTiles& mt, const Region& rg, int x, int y) {
    const uint32_t ntxv = (rg.vw + kTileW - 1u) / kTileW;
    return mt.flags[((uint32_t)(y - (int)rg.vy0) / kTileH) * ntxv + (uint32_t)(x - (int)rg.vx0) / kTileW];
}

// ---------------------------------------------------------------------------------------------------------
// Screen-tile staging for the N = 1 / 2 biased passes: the tile's neighbourhood window, R <= kLdsSpatialR (host check).
// (Round 4 removed k_spatial1_lds / k_spatial1_ldsr, which staged the reservoirs too -- 70 / 46 KB per block, measured
// 130 / 106 us against 82 for n_t alone at C2, profiles/r2 -- their source is profiles/r4/pruned/spatial1_lds.diff.)
constexpr uint32_t kLdsSpatialR = 10;
constexpr uint32_t kApronMax = (kTileW + 2u * kLdsSpatialR) * (kTileH + 2u * kLdsSpatialR);   // 1456 px

// k_spatial1_ntl: the N = 1 biased pass with the tile's n_t neighbourhood staged in LDS: the block copies the
// (32 + 2R) x (8 + 2R) n_t window (23 KB at R = 10) with row-coalesced LDS-DMA loads issued with the pixel's own
// records, so the heuristic's five neighbour records are ds_reads, not 16-byte gathers (each touching ~50 distinct
// 128-byte lines).  The accepted neighbours' reservoirs stay global gathers, one neighbour ahead of
// the consume sequence (k_spatial1h reads sample handles from LDS instead, point-light scenes).  R <= kLdsSpatialR.
// The n_t window of an ntl spatial block: the tile grown by R, clipped, AW entries per row, copied to LDS by
// LDS-DMA.  Each wave's 64 consecutive window entries l_nt[256k + 64w + lane] are written straight from global
// memory (global_load_lds_dwordx4, lane l at the wave-uniform base + 16 l), no VGPR round trip; the caller waits
// for them (explicit s_waitcnt vmcnt(0)) before its barrier, so after it every wave may read every entry.
// TH: tile height in 8-row units (blocks of 256 TH threads, a (32 + 2R) x (8 TH + 2R) window).
constexpr uint32_t apron_max(uint32_t TH) { return (kTileW + 2u * kLdsSpatialR) * (kTileH * TH + 2u * kLdsSpatialR); }
template <uint32_t TH = 1>
__device__ __forceinline__ void ntl_stage_window(const Region& rg, const float4* __restrict__ n_t, float4* l_nt, int ax0,
                                                 int ay0, uint32_t AW, uint32_t n_apron) {
    constexpr uint32_t kThreads = 256u * TH, kPer = (apron_max(TH) + kThreads - 1u) / kThreads;
    const uint32_t magic = 0xFFFFFFFFu / AW + 1u;
    const uint32_t w64 = (threadIdx.x >> 6) << 6;
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
        const uint32_t i = threadIdx.x + kThreads * k;
        if (i < n_apron) {
            uint32_t r = __umulhi(i, magic);   // i / AW for i < 2^16
            if (r * AW > i) r--;
            const uint32_t c = i - r * AW;
            const float4* src = n_t + (((uint32_t)(ay0 - (int)rg.vy0) + r) * rg.vw + (uint32_t)(ax0 - (int)rg.vx0) + c);
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                             (__attribute__((address_space(3))) void*)(l_nt + kThreads * k + w64), 16, 0, 0);
        }
    }
}

// GH (k_spatial1g_t2, a regular light grid): the input reservoirs arrive as grid handles (hg_in; ia / ib unused), one
// 16-byte gather per accepted neighbour instead of two, the sample rebuilt by grid_sample from the light colours the
// block stages in LDS behind the window; the output is written as a handle too (hg_out) and, unless odead (a later
// handle pass is its only reader), as the reservoir planes.
template <bool DBG, uint32_t TH = 1, bool GH = false>
__device__ __forceinline__ void spatial1_ntl_body(const SceneDev& s, const Region& rg, const FeaturesDev& f, uint32_t key,
                                                  v3 origin, const float4* __restrict__ n_t,
                                                  const float4* __restrict__ p_mat, const float4* __restrict__ ia,
                                                  const float4* __restrict__ ib, float4* __restrict__ oa,
                                                  float4* __restrict__ ob, float2* __restrict__ odbg,
                                                  const float* __restrict__ rp_in, float* __restrict__ rp_out,
                                                  MissTiles mt, const float4* __restrict__ hg_in = nullptr,
                                                  float4* __restrict__ hg_out = nullptr, uint32_t odead = 0u) {
#if !ROMIS_TAB_DMA
    const GlTabs tb = gl_stage_tables<false>();   // made visible by the window's barrier below
#endif
    float4* const l_nt = g_lds;
    float4* const l_col = g_lds + apron_max(TH);   // GH: the L light colours
    const uint32_t L = s.num_lights;
    auto put_handle = [&](uint32_t ofs, float W, uint32_t M, uint32_t li, float a, float b) {
        if (GH && hg_out) st_at(hg_out, ofs, make_float4(W, __uint_as_float(M | (li << 19)), a, b));
    };
    uint32_t tile;
    constexpr uint32_t kTH = kTileH * TH;   // tile rows
    const uint32_t ntx = (rg.rw + kTileW - 1) / kTileW;
    if (!xcd_tile(rg, ntx * ((rg.rh + kTH - 1) / kTH), blockIdx.x, tile)) return;   // block-uniform
    const int tx0 = (int)(rg.rx0 + (tile % ntx) * kTileW), ty0 = (int)(rg.ry0 + (tile / ntx) * kTH);
    bool mixed = false;   // some of the tile's pixels lie in background tiles (whose RIS reservoirs may be unwritten)
    if (mt.m) {
        // a tile of background pixels holding (0, W = 0), (0, M = mt.m): the miss shortcut's result below (W = 0, M the
        // pixel's own, wSum FLT_MIN), written without reading the tile, its window or its neighbours
        const int x1 = min(tx0 + (int)kTileW, (int)(rg.rx0 + rg.rw)) - 1, y1 = min(ty0 + (int)kTH, (int)(rg.ry0 + rg.rh)) - 1;
        if (tiles_known_miss(mt, rg, tx0, x1, ty0, y1, &mixed)) {
            const uint32_t mw = threadIdx.x >> 6, ml = threadIdx.x & 63u;
            const int mx = tx0 + (int)((mw & 3u) * 8u + (ml & 7u)), my = ty0 + (int)((mw >> 2) * 8u + (ml >> 3));
            if (mx <= x1 && my <= y1) {
                const uint32_t mo = ((uint32_t)(my - (int)rg.vy0) * rg.vw + (uint32_t)(mx - (int)rg.vx0)) << 4;
                if (!odead) {
                    st_at(oa, mo, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
                    st_at(ob, mo, make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(mt.m)));
                }
                if (DBG) st_at(odbg, mo >> 1, make_float2(ROMIS_FLT_MIN, 0.0f));
                if (rp_out) st_at(rp_out, mo >> 2, 0.0f);
                put_handle(mo, 0.0f, mt.m, L, 0.0f, 0.0f);
            }
            return;   // block-uniform, before the window's barrier
        }
    }
    // neighbour clamp bounds (render_utils.cpp:109-110: the image; here also the stored view), global coords
    const int xlo = max(0, (int)rg.vx0), xhi = min((int)rg.W, (int)(rg.vx0 + rg.vw)) - 1;
    const int ylo = max(0, (int)rg.vy0), yhi = min((int)rg.H, (int)(rg.vy0 + rg.vh)) - 1;
    const int R = (int)f.R;
    const int ax0 = max(tx0 - R, xlo), ax1 = min(tx0 + (int)kTileW - 1 + R, xhi);
    const int ay0 = max(ty0 - R, ylo), ay1 = min(ty0 + (int)kTH - 1 + R, yhi);
    const uint32_t AW = (uint32_t)(ax1 - ax0 + 1), n_apron = AW * (uint32_t)(ay1 - ay0 + 1);
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63u;   // wave w: the 8x8 block (w % 4, w / 4)
    const int x = tx0 + (int)((w & 3u) * 8u + (l & 7u)), y = ty0 + (int)((w >> 2) * 8u + (l >> 3));
    const bool live = x < (int)(rg.rx0 + rg.rw) && y < (int)(rg.ry0 + rg.rh);
    const uint32_t pofs = ((uint32_t)(y - (int)rg.vy0) * rg.vw + (uint32_t)(x - (int)rg.vx0)) << 4;
    // the pixel's own records (coalesced), issued first
    float4 cpm = make_float4(0.0f, 0.0f, 0.0f, 0.0f), ca = cpm, cb = cpm;
    float4 ch = make_float4(0.0f, __uint_as_float(L << 19), 0.0f, 0.0f);   // GH: the own handle
    float pd_cached = 0.0f;
    if (live) {
        // a pixel of a background tile holds the known (0, W = 0), (0, M = mt.m) and pdf 0: RIS may not have stored
        // them (its skip_res), so they are not read (a block-uniform branch: only tiles that straddle RIS tiles); nor,
        // with mt.gbuf, its G-buffer records: the miss material and a P that is not NaN is all the shortcut uses
        if (mixed && tile_flag_at(mt, rg, x, y) == 0u) {
            cpm = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(s.num_materials - 1u));
            cb.w = __uint_as_float(mt.m);
            ch.y = __uint_as_float(mt.m | (L << 19));
        } else {
            cpm = ld_at(p_mat, pofs);
            if (GH) {
                ch = ld_at(hg_in, pofs);
            } else {
                ca = ld_at(ia, pofs);
                cb = ld_at(ib, pofs);
            }
            if (rp_in) pd_cached = ld_at(rp_in, pofs >> 2);
        }
    }
    ntl_stage_window<TH>(rg, n_t, l_nt, ax0, ay0, AW, n_apron);
    if (GH) {   // the light colours behind the window (LDS-DMA, the same wait and barrier)
        const uint32_t w64 = (threadIdx.x >> 6) << 6;
        for (uint32_t d0 = 0; d0 < L; d0 += 256u * TH)
            if (d0 + threadIdx.x < L)
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(s.light_col + d0 + threadIdx.x),
                                                 (__attribute__((address_space(3))) void*)(l_col + d0 + w64), 16, 0, 0);
    }
#if ROMIS_TAB_DMA
    const GlTabs tb = gl_stage_tables_dma();   // behind the block's own loads; made visible by the window's barrier
#endif
    // neighbour draws while the loads are in flight
    const uint32_t K = f.K;   // <= kLeanK (host check)
    const uint32_t ps = pix_state(key, (uint32_t)y * rg.W + (uint32_t)x);
    const uint32_t span = 2u * f.R + 1u;
    uint32_t qi[kLeanK], qo[kLeanK];
#pragma unroll
    for (uint32_t n = 0; n < kLeanK; n++) {
        qi[n] = 0u;
        qo[n] = pofs;
        if (n < K) {
            const int nx = min(max(x - R + (int)__umulhi(draw(ps, 2u * n), span), xlo), xhi);
            const int ny = min(max(y - R + (int)__umulhi(draw(ps, 2u * n + 1u), span), ylo), yhi);
            qi[n] = (uint32_t)(ny - ay0) * AW + (uint32_t)(nx - ax0);
            qo[n] = ((uint32_t)(ny - (int)rg.vy0) * rg.vw + (uint32_t)(nx - (int)rg.vx0)) << 4;
        }
    }
    // Other waves read this wave's LDS-DMA entries after the barrier.  The compiler only waits for a wave's own
    // DMA before that wave's ds_reads, and a workgroup-scope fence need not drain vmcnt on gfx950, so the wait
    // is explicit (scripts/kernel_isa.sh k_spatial1_ntl: s_waitcnt vmcnt(0) directly before s_barrier).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (mt.m && mt.gbuf) {
        // RIS stored no G-buffer for background tiles: this thread's window entries there (its own LDS-DMA copies,
        // landed after the wait above) become a miss's record, normal 0 and t = FLT_MAX -- what RIS would have stored
        constexpr uint32_t kThreads = 256u * TH, kPer = (apron_max(TH) + kThreads - 1u) / kThreads;
#pragma unroll
        for (uint32_t k = 0; k < kPer; k++) {
            const uint32_t i = threadIdx.x + kThreads * k;
            if (i < n_apron) {
                uint32_t r = __umulhi(i, 0xFFFFFFFFu / AW + 1u);   // i / AW for i < 2^16 (ntl_stage_window)
                if (r * AW > i) r--;
                const uint32_t c = i - r * AW;
                if (tile_flag_at(mt, rg, ax0 + (int)c, ay0 + (int)r) == 0u)
                    l_nt[i] = make_float4(0.0f, 0.0f, 0.0f, ROMIS_FLT_MAX);
            }
        }
    }
    __syncthreads();
    if (!live) return;   // no barrier follows
    const float4 cn = l_nt[(uint32_t)(y - ay0) * AW + (uint32_t)(x - ax0)];
    const uint32_t cli = __float_as_uint(ch.y) >> 19;
    if (GH) {   // the own reservoir from its handle
        v3 p, c;
        grid_sample(s, l_col, cli, ch.z, ch.w, p, c);
        ca = make_float4(p.x, p.y, p.z, ch.x);
        cb = make_float4(c.x, c.y, c.z, __uint_as_float(__float_as_uint(ch.y) & kHandleMG));
    }
    const Px cur = make_px(s, cn, cpm, origin, pofs >> 4);
    // A primary-ray miss (value-initialised HitInfo: material kd = ks = 0, normal 0, P not NaN): its zero normal
    // rejects every neighbour (finite neighbour normals, s.normals_bounded: dot = +-0 < 0.906), and the target pdf of
    // any finite-colour sample there is exactly 0, so the combine takes only the pixel's own reservoir
    // with w = (0 * W) * M = +-0 (W finite): nothing is accepted, wSum stays FLT_MIN, M = M_own, W = 0.
    if (cur.mat == s.num_materials - 1u && s.normals_bounded && !__builtin_isnan(cur.P.x + cur.P.y + cur.P.z) &&
        __builtin_isfinite(ca.w) && __builtin_isfinite(cb.x + cb.y + cb.z)) {
        if (!odead) {
            st_at(oa, pofs, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
            st_at(ob, pofs, make_float4(0.0f, 0.0f, 0.0f, cb.w));
        }
        if (DBG) st_at(odbg, pofs >> 1, make_float2(ROMIS_FLT_MIN, 0.0f));
        if (rp_out) st_at(rp_out, pofs >> 2, 0.0f);
        put_handle(pofs, 0.0f, __float_as_uint(cb.w), L, 0.0f, 0.0f);
        return;
    }
    // depth / normal heuristic (render_utils.cpp:114-118), one shared reciprocal of the pixel's depth; both tests
    // for every lane from one ds_read_b128 (a branch around the depth test only saved work on rejected lanes).  The
    // correctly rounded division for depths outside the reciprocal's range is a wave-uniform branch: left to the
    // compiler it is if-converted and evaluated for every neighbour of every lane.
    const double rt = rcp_d(cur.t);
    const bool rt_all = __all(div_fast_ok(cur.t));
    bool ok[kLeanK];
#pragma unroll
    for (uint32_t n = 0; n < kLeanK; n++) {
        ok[n] = false;
        if (n < K) {
            const float4 g = l_nt[qi[n]];
            const float nd = vdot(xyz(g), cur.N);
            float q = div_by_rcp_d(g.w, rt);
            if (__builtin_expect(!rt_all, 0)) {
                if (!div_fast_ok(cur.t)) q = g.w / cur.t;
            }
            ok[n] = !(nd < 0.90630778703f) && !(fabsf(1.0f - q) > 0.1f);
        }
    }
    float4 na[kLeanK], nb[kLeanK];   // GH: na = the neighbour's handle
    auto gather = [&](uint32_t n) {
        if (GH) { na[n] = ld_at(hg_in, qo[n]); }
        else { na[n] = ld_at(ia, qo[n]); nb[n] = ld_at(ib, qo[n]); }
    };
    if (ok[0]) gather(0);
    const float pd_cur = rp_in ? pd_cached : target_pdf(s, f, cur, xyz(ca), xyz(cb), tb);
    Comb1 cmb;
    cmb.pos = mk(0.0f, 0.0f, 0.0f); cmb.col = mk(0.0f, 0.0f, 0.0f);
    cmb.wsum = ROMIS_FLT_MIN; cmb.chosen = 0.0f; cmb.pd = 0.0f; cmb.macc = 0u; cmb.has_pd = false;
    cmb.h = ps + 2u * K * 0x9E3779B9u;
    uint32_t hli = L;          // GH: the held sample's handle fields
    float hfa = 0.0f, hfb = 0.0f;
#pragma unroll
    for (uint32_t n = 0; n < kLeanK; n++) {
        if (n + 1 < kLeanK && ok[n + 1]) gather(n + 1);
        if (ok[n]) {
            if (GH) {
                const uint32_t hm = __float_as_uint(na[n].y), li = hm >> 19;
                v3 p, c;
                grid_sample(s, l_col, li, na[n].z, na[n].w, p, c);
                if (cmb.take(target_pdf(s, f, cur, p, c, tb), na[n].x, hm & kHandleMG, p, c)) {
                    hli = li; hfa = na[n].z; hfb = na[n].w;
                }
            } else {
                const v3 p = xyz(na[n]), c = xyz(nb[n]);
                cmb.take(target_pdf(s, f, cur, p, c, tb), na[n].w, __float_as_uint(nb[n].w), p, c);
            }
        }
    }
    if (cmb.take(pd_cur, ca.w, __float_as_uint(cb.w), xyz(ca), xyz(cb))) { hli = cli; hfa = ch.z; hfb = ch.w; }
    float p = cmb.pd;
    if (!cmb.has_pd) p = (f.shading && !__builtin_isnan(cur.P.x + cur.P.y + cur.P.z)) ? 0.0f : target_pdf(s, f, cur, cmb.pos, cmb.col, tb);
    const float W = contribution_weight(p, cmb.macc, cmb.wsum);
    if (!odead) {
        st_at(oa, pofs, make_float4(cmb.pos.x, cmb.pos.y, cmb.pos.z, W));
        st_at(ob, pofs, make_float4(cmb.col.x, cmb.col.y, cmb.col.z, __uint_as_float(cmb.macc)));
    }
    if (DBG) st_at(odbg, pofs >> 1, make_float2(cmb.wsum, cmb.chosen));
    if (rp_out) st_at(rp_out, pofs >> 2, p);
    put_handle(pofs, W, cmb.macc, hli, hfa, hfb);
}

#ifndef ROMIS_SPATIAL1_NTL_WPE
#define ROMIS_SPATIAL1_NTL_WPE 5
#endif
#define ROMIS_SPATIAL1_NTL_KERNEL(DBG, NAME)                                                                          \
    extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ROMIS_SPATIAL1_NTL_WPE))) void     \
    NAME(SceneDev s, Region rg, FeaturesDev f, uint32_t key, float ox, float oy, float oz, const float4* n_t,        \
         const float4* p_mat, const float4* ia, const float4* ib, float4* oa, float4* ob, float2* odbg,               \
         const float* rp_in, float* rp_out, MissTiles mt) {                                                           \
        spatial1_ntl_body<DBG>(s, rg, f, key, mk(ox, oy, oz), n_t, p_mat, ia, ib, oa, ob, odbg, rp_in, rp_out, mt);   \
    }
ROMIS_SPATIAL1_NTL_KERNEL(false, k_spatial1_ntl)
ROMIS_SPATIAL1_NTL_KERNEL(true, k_spatial1_ntl_dbg)

// k_spatial1_ntl_t2: the same pass on 32x16 tiles, 512-thread blocks (8 waves of 8x8): the window's apron rows are
// shared by twice the pixels (30 KB per 8 waves instead of 23 KB per 4), so LDS allows 8 waves per SIMD when the
// registers do (ROMIS_SPATIAL1_T2_WPE caps them: 8 -> 64 VGPRs).
#ifndef ROMIS_SPATIAL1_T2_WPE
#define ROMIS_SPATIAL1_T2_WPE 6
#endif
#define ROMIS_SPATIAL1_T2_KERNEL(DBG, NAME)                                                                           \
    extern "C" __global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(ROMIS_SPATIAL1_T2_WPE))) void     \
    NAME(SceneDev s, Region rg, FeaturesDev f, uint32_t key, float ox, float oy, float oz, const float4* n_t,        \
         const float4* p_mat, const float4* ia, const float4* ib, float4* oa, float4* ob, float2* odbg,               \
         const float* rp_in, float* rp_out, MissTiles mt) {                                                           \
        spatial1_ntl_body<DBG, 2>(s, rg, f, key, mk(ox, oy, oz), n_t, p_mat, ia, ib, oa, ob, odbg, rp_in, rp_out, mt);\
    }
ROMIS_SPATIAL1_T2_KERNEL(false, k_spatial1_ntl_t2)
ROMIS_SPATIAL1_T2_KERNEL(true, k_spatial1_ntl_t2_dbg)
// k_spatial1g_t2: k_spatial1_ntl_t2 over light-grid handles (GH)
#define ROMIS_SPATIAL1G_T2_KERNEL(DBG, NAME)                                                                          \
    extern "C" __global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(ROMIS_SPATIAL1_T2_WPE))) void     \
    NAME(SceneDev s, Region rg, FeaturesDev f, uint32_t key, float ox, float oy, float oz, const float4* n_t,        \
         const float4* p_mat, float4* oa, float4* ob, float2* odbg, const float* rp_in, float* rp_out, MissTiles mt,  \
         const float4* hg_in, float4* hg_out, uint32_t odead) {                                                       \
        spatial1_ntl_body<DBG, 2, true>(s, rg, f, key, mk(ox, oy, oz), n_t, p_mat, nullptr, nullptr, oa, ob, odbg, rp_in, \
                                        rp_out, mt, hg_in, hg_out, odead);                                             \
    }
ROMIS_SPATIAL1G_T2_KERNEL(false, k_spatial1g_t2)
ROMIS_SPATIAL1G_T2_KERNEL(true, k_spatial1g_t2_dbg)

// ---------------------------------------------------------------------------------------------------------
// k_spatial1h[_t2]: the N = 1 biased pass over sample handles (round 5).  In a point-light scene
// (SceneDev::light_types == points) a reservoir's sample is a light's (position, colour) from the light table, or
// the initial (0, 0) sample; the producer (k_primary_ris_n1*_pt, or this pass for the next) also writes the handle
// planes Handles::w = W and Handles::m = M | light index << 24 (index L = the zero sample), 4 + 4 B per pixel.  The
// block LDS-DMAs both planes over the tile's +-R window beside the n_t window, and the light table (positions, then
// colours, entry L zero), so an accepted neighbour's input is three ds_reads -- no global gather in the combine, and
// the pixel's own reservoir is read from the window too.  The arithmetic, RNG slots and update order are
// spatial1_ntl_body's (render_utils.cpp:102-133, reservoir.cpp:40-66): the same (position, colour, W, M) values, in
// the same operations.  The host launches it only when every M the passes can produce fits 24 bits and L <= 254.
struct HandlesIn { const float* w; const uint32_t* m; };
constexpr uint32_t kHandleM = 0x00FFFFFFu;

// The combine state over handles: Comb1 with the held sample's light index instead of its (position, colour).
struct Comb1h {
    float wsum, chosen, pd;
    uint32_t macc, li;
    bool has_pd;
    uint32_t h;
    __device__ __forceinline__ void take(float pd_in, float W, uint32_t M, uint32_t l) {
        const float w = (pd_in * W) * (float)M;          // reservoir.cpp:50
        macc += M;
        wsum += w;
        const float u = rand01(mix32(h));
        h += 0x9E3779B9u;
        if (accept_u(u, w, wsum)) { li = l; chosen = w; pd = pd_in; has_pd = true; }
    }
};

// LDS of a handle block: the n_t window, the two handle windows, then the light table (2 (L + 1) float4)
__host__ __device__ constexpr uint32_t h_lds_f4(uint32_t TH) { return apron_max(TH) + apron_max(TH) / 2u; }

template <uint32_t TH, bool HG = false>
__device__ __forceinline__ void h_stage(const SceneDev& s, const Region& rg, const float4* __restrict__ n_t, HandlesIn hi,
                                        float4* l_nt, float* l_w, uint32_t* l_m, float4* l_lt, int ax0, int ay0, uint32_t AW,
                                        uint32_t n_apron) {
    constexpr uint32_t kThreads = 256u * TH, kPer = (apron_max(TH) + kThreads - 1u) / kThreads;
    const uint32_t magic = 0xFFFFFFFFu / AW + 1u;
    const uint32_t w64 = (threadIdx.x >> 6) << 6;
    const uint32_t base = (uint32_t)(ay0 - (int)rg.vy0) * rg.vw + (uint32_t)(ax0 - (int)rg.vx0);
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
        const uint32_t i = threadIdx.x + kThreads * k;
        if (i < n_apron) {
            uint32_t r = __umulhi(i, magic);   // i / AW for i < 2^16
            if (r * AW > i) r--;
            const uint32_t o = base + r * rg.vw + (i - r * AW);
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(n_t + o),
                                             (__attribute__((address_space(3))) void*)(l_nt + kThreads * k + w64), 16, 0, 0);
            if (!HG) {
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(hi.w + o),
                                                 (__attribute__((address_space(3))) void*)(l_w + kThreads * k + w64), 4, 0, 0);
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(hi.m + o),
                                                 (__attribute__((address_space(3))) void*)(l_m + kThreads * k + w64), 4, 0, 0);
            }
        }
    }
    // light table: entries d = 0 .. L positions, L + 1 .. 2L + 1 colours (the light_c2 planes); d = L and 2L + 1 are
    // the zero sample's, stored by two threads
    const uint32_t L = s.num_lights, nd = 2u * L + 2u;
    for (uint32_t d0 = 0; d0 < nd; d0 += kThreads) {
        const uint32_t d = d0 + threadIdx.x;
        if (d < nd && d != L && d != 2u * L + 1u) {
            const float4* src = d < L ? s.light_c2 + d : s.light_c2 + (d - 1u);
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                             (__attribute__((address_space(3))) void*)(l_lt + d0 + w64), 16, 0, 0);
        }
    }
    if (threadIdx.x < 2u) l_lt[threadIdx.x ? 2u * L + 1u : L] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}

// HG (round 6 probe): the handles are gathered from global memory (the own pixel's coalesced, an accepted
// neighbour's one 4 + 4 B gather) instead of staged in LDS: the block's LDS is the n_t window and the light table only
// (34 KB at 32 x 16: four blocks of 8 waves per CU instead of three)
template <bool DBG, uint32_t TH = 1, bool HG = false>
__device__ __forceinline__ void spatial1h_body(const SceneDev& s, const Region& rg, const FeaturesDev& f, uint32_t key,
                                               v3 origin, const float4* __restrict__ n_t, const float4* __restrict__ p_mat,
                                               HandlesIn hi, float4* __restrict__ oa, float4* __restrict__ ob,
                                               float2* __restrict__ odbg, const float* __restrict__ rp_in,
                                               float* __restrict__ rp_out, float* __restrict__ how,
                                               uint32_t* __restrict__ hom, MissTiles mt, uint32_t odead) {
    constexpr uint32_t kTH = kTileH * TH;
    float4* const l_nt = g_lds;
    float* const l_w = reinterpret_cast<float*>(g_lds + apron_max(TH));
    uint32_t* const l_m = reinterpret_cast<uint32_t*>(l_w + apron_max(TH));
    float4* const l_lt = g_lds + (HG ? apron_max(TH) : h_lds_f4(TH));
    const uint32_t L = s.num_lights;
    uint32_t tile;
    const uint32_t ntx = (rg.rw + kTileW - 1) / kTileW;
    if (!xcd_tile(rg, ntx * ((rg.rh + kTH - 1) / kTH), blockIdx.x, tile)) return;   // block-uniform
    const int tx0 = (int)(rg.rx0 + (tile % ntx) * kTileW), ty0 = (int)(rg.ry0 + (tile / ntx) * kTH);
    bool mixed = false;
    if (mt.m) {   // background tiles: spatial1_ntl_body
        const int x1 = min(tx0 + (int)kTileW, (int)(rg.rx0 + rg.rw)) - 1, y1 = min(ty0 + (int)kTH, (int)(rg.ry0 + rg.rh)) - 1;
        if (tiles_known_miss(mt, rg, tx0, x1, ty0, y1, &mixed)) {
            const uint32_t mw = threadIdx.x >> 6, ml = threadIdx.x & 63u;
            const int mx = tx0 + (int)((mw & 3u) * 8u + (ml & 7u)), my = ty0 + (int)((mw >> 2) * 8u + (ml >> 3));
            if (mx <= x1 && my <= y1) {
                const uint32_t mp = (uint32_t)(my - (int)rg.vy0) * rg.vw + (uint32_t)(mx - (int)rg.vx0);
                if (!odead) {
                    st_at(oa, mp << 4, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
                    st_at(ob, mp << 4, make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(mt.m)));
                }
                if (DBG) st_at(odbg, mp << 3, make_float2(ROMIS_FLT_MIN, 0.0f));
                if (rp_out) rp_out[mp] = 0.0f;
                if (how) { how[mp] = 0.0f; hom[mp] = mt.m | (L << 24); }
            }
            return;
        }
    }
    const int xlo = max(0, (int)rg.vx0), xhi = min((int)rg.W, (int)(rg.vx0 + rg.vw)) - 1;
    const int ylo = max(0, (int)rg.vy0), yhi = min((int)rg.H, (int)(rg.vy0 + rg.vh)) - 1;
    const int R = (int)f.R;
    const int ax0 = max(tx0 - R, xlo), ax1 = min(tx0 + (int)kTileW - 1 + R, xhi);
    const int ay0 = max(ty0 - R, ylo), ay1 = min(ty0 + (int)kTH - 1 + R, yhi);
    const uint32_t AW = (uint32_t)(ax1 - ax0 + 1), n_apron = AW * (uint32_t)(ay1 - ay0 + 1);
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63u;
    const int x = tx0 + (int)((w & 3u) * 8u + (l & 7u)), y = ty0 + (int)((w >> 2) * 8u + (l >> 3));
    const bool live = x < (int)(rg.rx0 + rg.rw) && y < (int)(rg.ry0 + rg.rh);
    const uint32_t pix = (uint32_t)(y - (int)rg.vy0) * rg.vw + (uint32_t)(x - (int)rg.vx0);
    float4 cpm = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    float pd_cached = 0.0f;
    float gw = 0.0f;
    uint32_t gm = 0u;
    const bool own_bg = live && mixed && tile_flag_at(mt, rg, x, y) == 0u;   // a background RIS tile: known, unread
    if (live) {
        if (own_bg) {
            cpm = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(s.num_materials - 1u));
        } else {
            cpm = p_mat[pix];
            if (rp_in) pd_cached = rp_in[pix];
            if (HG) { gw = hi.w[pix]; gm = hi.m[pix]; }
        }
    }
    h_stage<TH, HG>(s, rg, n_t, hi, l_nt, l_w, l_m, l_lt, ax0, ay0, AW, n_apron);
    const GlTabs tb = gl_stage_tables_dma();
    const uint32_t K = f.K;   // <= kLeanK (host check)
    const uint32_t ps = pix_state(key, (uint32_t)y * rg.W + (uint32_t)x);
    const uint32_t span = 2u * f.R + 1u;
    uint32_t qi[kLeanK], qp[kLeanK];
#pragma unroll
    for (uint32_t n = 0; n < kLeanK; n++) {
        qi[n] = 0u;
        qp[n] = 0u;
        if (n < K) {
            const int nx = min(max(x - R + (int)__umulhi(draw(ps, 2u * n), span), xlo), xhi);
            const int ny = min(max(y - R + (int)__umulhi(draw(ps, 2u * n + 1u), span), ylo), yhi);
            qi[n] = (uint32_t)(ny - ay0) * AW + (uint32_t)(nx - ax0);
            if (HG) qp[n] = (uint32_t)(ny - (int)rg.vy0) * rg.vw + (uint32_t)(nx - (int)rg.vx0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's DMA before the barrier (spatial1_ntl_body)
    if (mt.m && mt.gbuf) {   // background G-buffer records: spatial1_ntl_body's window fix-up
        constexpr uint32_t kThreads = 256u * TH, kPer = (apron_max(TH) + kThreads - 1u) / kThreads;
#pragma unroll
        for (uint32_t k = 0; k < kPer; k++) {
            const uint32_t i = threadIdx.x + kThreads * k;
            if (i < n_apron) {
                uint32_t r = __umulhi(i, 0xFFFFFFFFu / AW + 1u);
                if (r * AW > i) r--;
                const uint32_t c = i - r * AW;
                if (tile_flag_at(mt, rg, ax0 + (int)c, ay0 + (int)r) == 0u) l_nt[i] = make_float4(0.0f, 0.0f, 0.0f, ROMIS_FLT_MAX);
            }
        }
    }
    __syncthreads();
    if (!live) return;   // no barrier follows
    const uint32_t own = (uint32_t)(y - ay0) * AW + (uint32_t)(x - ax0);
    const float4 cn = l_nt[own];
    const float cw = own_bg ? 0.0f : (HG ? gw : l_w[own]);
    const uint32_t cm = own_bg ? (mt.m | (L << 24)) : (HG ? gm : l_m[own]);
    const uint32_t cli = cm >> 24;
    const v3 cpos = xyz(l_lt[cli]), ccol = xyz(l_lt[L + 1u + cli]);
    const Px cur = make_px(s, cn, cpm, origin, pix);
    if (cur.mat == s.num_materials - 1u && s.normals_bounded && !__builtin_isnan(cur.P.x + cur.P.y + cur.P.z) &&
        __builtin_isfinite(cw) && __builtin_isfinite(ccol.x + ccol.y + ccol.z)) {
        if (!odead) {
            st_at(oa, pix << 4, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
            st_at(ob, pix << 4, make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(cm & kHandleM)));
        }
        if (DBG) st_at(odbg, pix << 3, make_float2(ROMIS_FLT_MIN, 0.0f));
        if (rp_out) rp_out[pix] = 0.0f;
        if (how) { how[pix] = 0.0f; hom[pix] = (cm & kHandleM) | (L << 24); }
        return;
    }
    const double rt = rcp_d(cur.t);
    const bool rt_all = __all(div_fast_ok(cur.t));
    bool ok[kLeanK];
    uint32_t qm[kLeanK];
    float qw[kLeanK];
#pragma unroll
    for (uint32_t n = 0; n < kLeanK; n++) {
        ok[n] = false;
        qm[n] = 0u;
        qw[n] = 0.0f;
        if (n < K) {
            const float4 g = l_nt[qi[n]];
            if (!HG) {
                qm[n] = l_m[qi[n]];
                qw[n] = l_w[qi[n]];
            }
            const float nd = vdot(xyz(g), cur.N);
            float q = div_by_rcp_d(g.w, rt);
            if (__builtin_expect(!rt_all, 0)) {
                if (!div_fast_ok(cur.t)) q = g.w / cur.t;
            }
            ok[n] = !(nd < 0.90630778703f) && !(fabsf(1.0f - q) > 0.1f);
            if (HG && ok[n]) { qm[n] = hi.m[qp[n]]; qw[n] = hi.w[qp[n]]; }
        }
    }
    const float pd_cur = rp_in ? pd_cached : target_pdf(s, f, cur, cpos, ccol, tb);
    Comb1h cmb;
    cmb.wsum = ROMIS_FLT_MIN; cmb.chosen = 0.0f; cmb.pd = 0.0f; cmb.macc = 0u; cmb.li = L; cmb.has_pd = false;
    cmb.h = ps + 2u * K * 0x9E3779B9u;
#pragma unroll
    for (uint32_t n = 0; n < kLeanK; n++) {
        if (ok[n]) {
            const uint32_t li = qm[n] >> 24;
            cmb.take(target_pdf(s, f, cur, xyz(l_lt[li]), xyz(l_lt[L + 1u + li]), tb), qw[n], qm[n] & kHandleM, li);
        }
    }
    cmb.take(pd_cur, cw, cm & kHandleM, cli);
    const v3 pos = xyz(l_lt[cmb.li]), col = xyz(l_lt[L + 1u + cmb.li]);
    float p = cmb.pd;
    if (!cmb.has_pd) p = (f.shading && !__builtin_isnan(cur.P.x + cur.P.y + cur.P.z)) ? 0.0f : target_pdf(s, f, cur, pos, col, tb);
    const float W = contribution_weight(p, cmb.macc, cmb.wsum);
    if (!odead) {   // odead: a later handle pass is the output's only reader
        st_at(oa, pix << 4, make_float4(pos.x, pos.y, pos.z, W));
        st_at(ob, pix << 4, make_float4(col.x, col.y, col.z, __uint_as_float(cmb.macc)));
    }
    if (DBG) st_at(odbg, pix << 3, make_float2(cmb.wsum, cmb.chosen));
    if (rp_out) rp_out[pix] = p;
    if (how) { how[pix] = W; hom[pix] = cmb.macc | (cmb.li << 24); }
}

#ifndef ROMIS_SPATIAL1H_WPE
#define ROMIS_SPATIAL1H_WPE 5
#endif
#define ROMIS_SPATIAL1H_KERNEL(DBG, TH, NAME)                                                                          \
    extern "C" __global__ __launch_bounds__(256 * TH) __attribute__((amdgpu_waves_per_eu(ROMIS_SPATIAL1H_WPE))) void   \
    NAME(SceneDev s, Region rg, FeaturesDev f, uint32_t key, float ox, float oy, float oz, const float4* n_t,        \
         const float4* p_mat, HandlesIn hi, float4* oa, float4* ob, float2* odbg, const float* rp_in, float* rp_out,  \
         float* how, uint32_t* hom, MissTiles mt, uint32_t odead) {                                                   \
        spatial1h_body<DBG, TH>(s, rg, f, key, mk(ox, oy, oz), n_t, p_mat, hi, oa, ob, odbg, rp_in, rp_out, how, hom, mt,  \
                                odead);                                                                                \
    }
ROMIS_SPATIAL1H_KERNEL(false, 1, k_spatial1h)
ROMIS_SPATIAL1H_KERNEL(true, 1, k_spatial1h_dbg)
ROMIS_SPATIAL1H_KERNEL(false, 2, k_spatial1h_t2)
ROMIS_SPATIAL1H_KERNEL(true, 2, k_spatial1h_t2_dbg)
#ifndef ROMIS_SPATIAL1HG_WPE
#define ROMIS_SPATIAL1HG_WPE 8
#endif
#define ROMIS_SPATIAL1HG_KERNEL(DBG, NAME)                                                                             \
    extern "C" __global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(ROMIS_SPATIAL1HG_WPE))) void      \
    NAME(SceneDev s, Region rg, FeaturesDev f, uint32_t key, float ox, float oy, float oz, const float4* n_t,        \
         const float4* p_mat, HandlesIn hi, float4* oa, float4* ob, float2* odbg, const float* rp_in, float* rp_out,  \
         float* how, uint32_t* hom, MissTiles mt, uint32_t odead) {                                                   \
        spatial1h_body<DBG, 2, true>(s, rg, f, key, mk(ox, oy, oz), n_t, p_mat, hi, oa, ob, odbg, rp_in, rp_out, how, \
                                     hom, mt, odead);                                                                  \
    }
ROMIS_SPATIAL1HG_KERNEL(false, k_spatial1hg_t2)
ROMIS_SPATIAL1HG_KERNEL(true, k_spatial1hg_t2_dbg)



// k_spatial2_ntl: the biased pass for N = 2 sub-reservoirs (the reference's default, common.h:105), laid out like
// k_spatial1_ntl (32x8 tiles in the XCD chunk order, the n_t window in LDS by LDS-DMA, one shared depth
// reciprocal).  Each accepted neighbour contributes its N sub-reservoirs in order, then the pixel's own (render_utils
// .cpp:108-124); every input goes to the output sub-reservoir with the smallest wSum (strict <, first index:
// Reservoir::update, reservoir.cpp:10-32) and adds its M to that one's routed sum (combineBiased, reservoir.cpp:40-
// 66).  Same arithmetic, RNG slots (2K + input index) and order as spatial_pixel<N, false>; R <= kLdsSpatialR.
template <int NT>
struct CombN {
    v3 pos[NT], col[NT];
    float wsum[NT], chosen[NT], pd[NT];
    uint32_t macc[NT];
    bool has_pd[NT];
    uint32_t h;   // ps + slot * 0x9E3779B9 of the next accept draw
    __device__ __forceinline__ void init(uint32_t h0) {
#pragma unroll
        for (int j = 0; j < NT; j++) {
            pos[j] = mk(0.0f, 0.0f, 0.0f); col[j] = mk(0.0f, 0.0f, 0.0f);
            wsum[j] = ROMIS_FLT_MIN; chosen[j] = 0.0f; pd[j] = 0.0f; macc[j] = 0u; has_pd[j] = false;
        }
        h = h0;
    }
    __device__ __forceinline__ void take(float pd_in, float W, uint32_t M, v3 p, v3 c) {
        const float w = (pd_in * W) * (float)M;          // reservoir.cpp:50
        uint32_t k = 0;                                    // argmin wSum from FLT_MAX, strict <, first index
        float best = ROMIS_FLT_MAX;                        // (reservoir.cpp:12-19; a NaN wSum is never taken)
#pragma unroll
        for (int j = 0; j < NT; j++)
            if (wsum[j] < best) { k = (uint32_t)j; best = wsum[j]; }
        const float u = rand01(mix32(h));
        h += 0x9E3779B9u;
#pragma unroll
        for (int j = 0; j < NT; j++) {
            if ((uint32_t)j == k) {
                macc[j] += M;
                wsum[j] += w;
                if (accept_u(u, w, wsum[j])) { pos[j] = p; col[j] = c; chosen[j] = w; pd[j] = pd_in; has_pd[j] = true; }
            }
        }
    }
};

template <bool DBG, int NT>
__device__ __forceinline__ void spatialn_ntl_body(const SceneDev& s, const Region& rg, const FeaturesDev& f, uint32_t key,
                                                  v3 origin, const float4* __restrict__ n_t,
                                                  const float4* __restrict__ p_mat, const float4* __restrict__ ia,
                                                  const float4* __restrict__ ib, float4* __restrict__ oa,
                                                  float4* __restrict__ ob, float2* __restrict__ odbg, MissTiles mt) {
    const GlTabs tb = gl_stage_tables<false>();   // made visible by the window's barrier below
    float4* const l_nt = g_lds;
    uint32_t tile;
    if (!xcd_tile(rg, num_tiles(rg), blockIdx.x, tile)) return;   // block-uniform
    const uint32_t ntx = (rg.rw + kTileW - 1) / kTileW;
    const int tx0 = (int)(rg.rx0 + (tile % ntx) * kTileW), ty0 = (int)(rg.ry0 + (tile / ntx) * kTileH);
    if (mt.m) {
        // a tile of background pixels: after RIS and after every biased pass each holds sub-reservoir 0 = (0, W = 0),
        // (0, M = mt.m) and the others (0, W = 0), (0, M = 0) -- the miss shortcut's result below (M_0 = the sum of
        // the own Ms), written without reading the tile or its window
        const int x1 = min(tx0 + (int)kTileW, (int)(rg.rx0 + rg.rw)) - 1, y1 = min(ty0 + (int)kTileH, (int)(rg.ry0 + rg.rh)) - 1;
        if (tiles_known_miss(mt, rg, tx0, x1, ty0, y1)) {
            const uint32_t mw = threadIdx.x >> 6, ml = threadIdx.x & 63u;
            const int mx = tx0 + (int)(mw * 8u + (ml & 7u)), my = ty0 + (int)(ml >> 3);
            if (mx <= x1 && my <= y1) {
                const uint32_t mo = ((uint32_t)(my - (int)rg.vy0) * rg.vw + (uint32_t)(mx - (int)rg.vx0)) << 4;
                const uint32_t jo = rg.js << 4;
#pragma unroll
                for (int j = 0; j < NT; j++) {
                    st_at(oa, mo + (uint32_t)j * jo, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
                    st_at(ob, mo + (uint32_t)j * jo, make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(j == 0 ? mt.m : 0u)));
                    if (DBG) st_at(odbg, (mo + (uint32_t)j * jo) >> 1, make_float2(ROMIS_FLT_MIN, 0.0f));
                }
            }
            return;   // block-uniform, before the window's barrier
        }
    }
    const int xlo = max(0, (int)rg.vx0), xhi = min((int)rg.W, (int)(rg.vx0 + rg.vw)) - 1;
    const int ylo = max(0, (int)rg.vy0), yhi = min((int)rg.H, (int)(rg.vy0 + rg.vh)) - 1;
    const int R = (int)f.R;
    const int ax0 = max(tx0 - R, xlo), ax1 = min(tx0 + (int)kTileW - 1 + R, xhi);
    const int ay0 = max(ty0 - R, ylo), ay1 = min(ty0 + (int)kTileH - 1 + R, yhi);
    const uint32_t AW = (uint32_t)(ax1 - ax0 + 1), n_apron = AW * (uint32_t)(ay1 - ay0 + 1);
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63u;
    const int x = tx0 + (int)(w * 8u + (l & 7u)), y = ty0 + (int)(l >> 3);
    const bool live = x < (int)(rg.rx0 + rg.rw) && y < (int)(rg.ry0 + rg.rh);
    const uint32_t pofs = ((uint32_t)(y - (int)rg.vy0) * rg.vw + (uint32_t)(x - (int)rg.vx0)) << 4;
    const uint32_t jofs = rg.js << 4;   // bytes between sub-reservoir planes (host check: fits 32 bits)
    float4 cpm = make_float4(0.0f, 0.0f, 0.0f, 0.0f), ca[NT], cb[NT];
#pragma unroll
    for (int j = 0; j < NT; j++) { ca[j] = cpm; cb[j] = cpm; }
    if (live) {
        cpm = ld_at(p_mat, pofs);
#pragma unroll
        for (int j = 0; j < NT; j++) { ca[j] = ld_at(ia, pofs + (uint32_t)j * jofs); cb[j] = ld_at(ib, pofs + (uint32_t)j * jofs); }
    }
    ntl_stage_window(rg, n_t, l_nt, ax0, ay0, AW, n_apron);
    const uint32_t K = f.K;   // <= kLeanK (host check)
    const uint32_t ps = pix_state(key, (uint32_t)y * rg.W + (uint32_t)x);
    const uint32_t span = 2u * f.R + 1u;
    uint32_t qi[kLeanK], qo[kLeanK];
#pragma unroll
    for (uint32_t n = 0; n < kLeanK; n++) {
        qi[n] = 0u;
        qo[n] = pofs;
        if (n < K) {
            const int nx = min(max(x - R + (int)__umulhi(draw(ps, 2u * n), span), xlo), xhi);
            const int ny = min(max(y - R + (int)__umulhi(draw(ps, 2u * n + 1u), span), ylo), yhi);
            qi[n] = (uint32_t)(ny - ay0) * AW + (uint32_t)(nx - ax0);
            qo[n] = ((uint32_t)(ny - (int)rg.vy0) * rg.vw + (uint32_t)(nx - (int)rg.vx0)) << 4;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's window copies, before the barrier
    __syncthreads();
    if (!live) return;   // no barrier follows
    const float4 cn = l_nt[(uint32_t)(y - ay0) * AW + (uint32_t)(x - ax0)];
    const Px cur = make_px(s, cn, cpm, origin, pofs >> 4);
    // primary-ray miss (see spatial1_ntl_body): every neighbour is rejected and every own input weighs (0 W) M = +-0,
    // so both go to sub-reservoir 0 (equal wSums FLT_MIN), nothing is accepted: M_0 = sum of the own Ms, W = 0
    bool miss = cur.mat == s.num_materials - 1u && s.normals_bounded && !__builtin_isnan(cur.P.x + cur.P.y + cur.P.z);
#pragma unroll
    for (int j = 0; j < NT; j++) miss = miss && __builtin_isfinite(ca[j].w) && __builtin_isfinite(cb[j].x + cb[j].y + cb[j].z);
    if (miss) {
        uint32_t m = 0u;
#pragma unroll
        for (int j = 0; j < NT; j++) m += __float_as_uint(cb[j].w);
#pragma unroll
        for (int j = 0; j < NT; j++) {
            st_at(oa, pofs + (uint32_t)j * jofs, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
            st_at(ob, pofs + (uint32_t)j * jofs, make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(j == 0 ? m : 0u)));
            if (DBG) st_at(odbg, (pofs + (uint32_t)j * jofs) >> 1, make_float2(ROMIS_FLT_MIN, 0.0f));
        }
        return;
    }
    // depth / normal heuristic (render_utils.cpp:114-118), as in spatial1_ntl_body
    const double rt = rcp_d(cur.t);
    const bool rt_all = __all(div_fast_ok(cur.t));
    bool ok[kLeanK];
#pragma unroll
    for (uint32_t n = 0; n < kLeanK; n++) {
        ok[n] = false;
        if (n < K) {
            const float4 g = l_nt[qi[n]];
            const float nd = vdot(xyz(g), cur.N);
            float q = div_by_rcp_d(g.w, rt);
            if (__builtin_expect(!rt_all, 0)) {
                if (!div_fast_ok(cur.t)) q = g.w / cur.t;
            }
            ok[n] = !(nd < 0.90630778703f) && !(fabsf(1.0f - q) > 0.1f);
        }
    }
    CombN<NT> cmb;
    cmb.init(ps + 2u * K * 0x9E3779B9u);
    float4 na[NT], nb[NT];
#pragma unroll
    for (uint32_t n = 0; n < kLeanK; n++) {
        if (ok[n]) {
#pragma unroll
            for (int j = 0; j < NT; j++) { na[j] = ld_at(ia, qo[n] + (uint32_t)j * jofs); nb[j] = ld_at(ib, qo[n] + (uint32_t)j * jofs); }
#pragma unroll
            for (int j = 0; j < NT; j++) {
                const v3 p = xyz(na[j]), c = xyz(nb[j]);
                cmb.take(target_pdf(s, f, cur, p, c, tb), na[j].w, __float_as_uint(nb[j].w), p, c);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < NT; j++) {
        const v3 p = xyz(ca[j]), c = xyz(cb[j]);
        cmb.take(target_pdf(s, f, cur, p, c, tb), ca[j].w, __float_as_uint(cb[j].w), p, c);
    }
    // finish_biased: M = routed sum, W from the held sample's target pdf (light.cpp:90-93 / reservoir.cpp:61-64);
    // nothing accepted: the initial (0, 0) sample, whose shaded value is +-0 at a non-NaN position (W = 0)
#pragma unroll
    for (int j = 0; j < NT; j++) {
        float p = cmb.pd[j];
        if (!cmb.has_pd[j])
            p = (f.shading && !__builtin_isnan(cur.P.x + cur.P.y + cur.P.z)) ? 0.0f : target_pdf(s, f, cur, cmb.pos[j], cmb.col[j], tb);
        const float W = contribution_weight(p, cmb.macc[j], cmb.wsum[j]);
        st_at(oa, pofs + (uint32_t)j * jofs, make_float4(cmb.pos[j].x, cmb.pos[j].y, cmb.pos[j].z, W));
        st_at(ob, pofs + (uint32_t)j * jofs, make_float4(cmb.col[j].x, cmb.col[j].y, cmb.col[j].z, __uint_as_float(cmb.macc[j])));
        if (DBG) st_at(odbg, (pofs + (uint32_t)j * jofs) >> 1, make_float2(cmb.wsum[j], cmb.chosen[j]));
    }
}

// k_spatial2hg[_t2]: the N = 2 biased pass over sample handles (round 6), point lights.  The producer
// (k_primary_ris_n2*_pt, or this pass for the next) writes one 16-byte handle record per pixel, (W_0, M_0 | i_0 << 24,
// W_1, M_1 | i_1 << 24) -- sub-reservoir j's W, M and light index (L = the zero sample) -- instead of the four 16-byte
// reservoir records; an accepted neighbour is one 16-byte gather, its samples rebuilt from the light table the block
// stages in LDS behind the n_t window (k_spatial2_ntl gathers 64 B).  The combine is spatialn_ntl_body's: each accepted
// neighbour's two sub-reservoirs in order, then the pixel's own, each routed to the output with the smallest wSum
// (strict <, first index: reservoir.cpp:10-32) and adding its M there (combineBiased, reservoir.cpp:40-66); the same
// RNG slots and arithmetic on the same (position, colour, W, M) values.  The host enables it only while every M fits 24
// bits and L <= 254.
struct Comb2h {
    float wsum[2], chosen[2], pd[2];
    uint32_t macc[2], li[2];
    bool has_pd[2];
    uint32_t h;
    __device__ __forceinline__ void init(uint32_t h0, uint32_t L) {
#pragma unroll
        for (int j = 0; j < 2; j++) {
            wsum[j] = ROMIS_FLT_MIN; chosen[j] = 0.0f; pd[j] = 0.0f; macc[j] = 0u; li[j] = L; has_pd[j] = false;
        }
        h = h0;
    }
    __device__ __forceinline__ void take(float pd_in, float W, uint32_t M, uint32_t l) {
        const float w = (pd_in * W) * (float)M;          // reservoir.cpp:50
        const bool k1 = wsum[1] < (wsum[0] < ROMIS_FLT_MAX ? wsum[0] : ROMIS_FLT_MAX);   // CombN's argmin, N = 2
        const float u = rand01(mix32(h));
        h += 0x9E3779B9u;
#pragma unroll
        for (int j = 0; j < 2; j++) {
            if ((j == 1) == k1) {
                macc[j] += M;
                wsum[j] += w;
                if (accept_u(u, w, wsum[j])) { li[j] = l; chosen[j] = w; pd[j] = pd_in; has_pd[j] = true; }
            }
        }
    }
};

template <bool DBG, uint32_t TH>
__device__ __forceinline__ void spatial2hg_body(const SceneDev& s, const Region& rg, const FeaturesDev& f, uint32_t key,
                                                v3 origin, const float4* __restrict__ n_t, const float4* __restrict__ p_mat,
                                                const float4* __restrict__ hin, float4* __restrict__ oa,
                                                float4* __restrict__ ob, float2* __restrict__ odbg, float4* __restrict__ hout,
                                                MissTiles mt, uint32_t odead) {
    constexpr uint32_t kTH = kTileH * TH;
    float4* const l_nt = g_lds;
    float4* const l_lt = g_lds + apron_max(TH);
    const uint32_t L = s.num_lights;
    const uint32_t jofs = rg.js << 4;   // bytes between the sub-reservoir planes
    uint32_t tile;
    const uint32_t ntx = (rg.rw + kTileW - 1) / kTileW;
    if (!xcd_tile(rg, ntx * ((rg.rh + kTH - 1) / kTH), blockIdx.x, tile)) return;   // block-uniform
    const int tx0 = (int)(rg.rx0 + (tile % ntx) * kTileW), ty0 = (int)(rg.ry0 + (tile / ntx) * kTH);
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63u;   // wave w: the 8x8 block (w % 4, w / 4)
    auto put = [&](uint32_t pix, const float* W, const uint32_t* M, const uint32_t* li, const float* ws, const float* ch) {
#pragma unroll
        for (int j = 0; j < 2; j++) {
            if (!odead) {
                const float4 pos = l_lt[li[j]], col = l_lt[L + 1u + li[j]];
                st_at(oa, (pix << 4) + (uint32_t)j * jofs, make_float4(pos.x, pos.y, pos.z, W[j]));
                st_at(ob, (pix << 4) + (uint32_t)j * jofs, make_float4(col.x, col.y, col.z, __uint_as_float(M[j])));
            }
            if (DBG) st_at(odbg, ((pix << 4) + (uint32_t)j * jofs) >> 1, make_float2(ws[j], ch[j]));
        }
        if (hout) hout[pix] = make_float4(W[0], __uint_as_float(M[0] | (li[0] << 24)), W[1], __uint_as_float(M[1] | (li[1] << 24)));
    };
    bool mixed = false;
    if (mt.m) {
        // a tile of background pixels: sub-reservoir 0 = (0, W = 0), (0, M = mt.m), sub-reservoir 1 = (0, W = 0), (0, M = 0)
        // -- the miss shortcut's result below, written without reading the tile, its window or its neighbours.  The
        // light table is not staged: the zero sample's (position, colour) are written as zeros
        const int x1 = min(tx0 + (int)kTileW, (int)(rg.rx0 + rg.rw)) - 1, y1 = min(ty0 + (int)kTH, (int)(rg.ry0 + rg.rh)) - 1;
        if (tiles_known_miss(mt, rg, tx0, x1, ty0, y1, &mixed)) {
            const int mx = tx0 + (int)((w & 3u) * 8u + (l & 7u)), my = ty0 + (int)((w >> 2) * 8u + (l >> 3));
            if (mx <= x1 && my <= y1) {
                const uint32_t mp = (uint32_t)(my - (int)rg.vy0) * rg.vw + (uint32_t)(mx - (int)rg.vx0);
#pragma unroll
                for (int j = 0; j < 2; j++) {
                    if (!odead) {
                        st_at(oa, (mp << 4) + (uint32_t)j * jofs, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
                        st_at(ob, (mp << 4) + (uint32_t)j * jofs, make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(j == 0 ? mt.m : 0u)));
                    }
                    if (DBG) st_at(odbg, ((mp << 4) + (uint32_t)j * jofs) >> 1, make_float2(ROMIS_FLT_MIN, 0.0f));
                }
                if (hout) hout[mp] = make_float4(0.0f, __uint_as_float(mt.m | (L << 24)), 0.0f, __uint_as_float(L << 24));
            }
            return;   // block-uniform, before the window's barrier
        }
    }
    const int xlo = max(0, (int)rg.vx0), xhi = min((int)rg.W, (int)(rg.vx0 + rg.vw)) - 1;
    const int ylo = max(0, (int)rg.vy0), yhi = min((int)rg.H, (int)(rg.vy0 + rg.vh)) - 1;
    const int R = (int)f.R;
    const int ax0 = max(tx0 - R, xlo), ax1 = min(tx0 + (int)kTileW - 1 + R, xhi);
    const int ay0 = max(ty0 - R, ylo), ay1 = min(ty0 + (int)kTH - 1 + R, yhi);
    const uint32_t AW = (uint32_t)(ax1 - ax0 + 1), n_apron = AW * (uint32_t)(ay1 - ay0 + 1);
    const int x = tx0 + (int)((w & 3u) * 8u + (l & 7u)), y = ty0 + (int)((w >> 2) * 8u + (l >> 3));
    const bool live = x < (int)(rg.rx0 + rg.rw) && y < (int)(rg.ry0 + rg.rh);
    const uint32_t pix = (uint32_t)(y - (int)rg.vy0) * rg.vw + (uint32_t)(x - (int)rg.vx0);
    float4 cpm = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    float4 ch = make_float4(0.0f, __uint_as_float(L << 24), 0.0f, __uint_as_float(L << 24));   // the own handle record
    const bool own_bg = live && mixed && tile_flag_at(mt, rg, x, y) == 0u;   // a background RIS tile: known, unread
    if (live) {
        if (own_bg) {
            cpm = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(s.num_materials - 1u));
            ch.y = __uint_as_float(mt.m | (L << 24));
        } else {
            cpm = p_mat[pix];
            ch = hin[pix];
        }
    }
    ntl_stage_window<TH>(rg, n_t, l_nt, ax0, ay0, AW, n_apron);
    {   // the light table behind the window: positions, zero, colours, zero (h_stage)
        constexpr uint32_t kThreads = 256u * TH;
        const uint32_t nd = 2u * L + 2u, w64 = (threadIdx.x >> 6) << 6;
        for (uint32_t d0 = 0; d0 < nd; d0 += kThreads) {
            const uint32_t d = d0 + threadIdx.x;
            if (d < nd && d != L && d != 2u * L + 1u)
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(d < L ? s.light_c2 + d : s.light_c2 + (d - 1u)),
                                                 (__attribute__((address_space(3))) void*)(l_lt + d0 + w64), 16, 0, 0);
        }
        if (threadIdx.x < 2u) l_lt[threadIdx.x ? 2u * L + 1u : L] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    const GlTabs tb = gl_stage_tables_dma();
    const uint32_t K = f.K;   // <= kLeanK (host check)
    const uint32_t ps = pix_state(key, (uint32_t)y * rg.W + (uint32_t)x);
    const uint32_t span = 2u * f.R + 1u;
    uint32_t qi[kLeanK], qp[kLeanK];
#pragma unroll
    for (uint32_t n = 0; n < kLeanK; n++) {
        qi[n] = 0u;
        qp[n] = pix;
        if (n < K) {
            const int nx = min(max(x - R + (int)__umulhi(draw(ps, 2u * n), span), xlo), xhi);
            const int ny = min(max(y - R + (int)__umulhi(draw(ps, 2u * n + 1u), span), ylo), yhi);
            qi[n] = (uint32_t)(ny - ay0) * AW + (uint32_t)(nx - ax0);
            qp[n] = (uint32_t)(ny - (int)rg.vy0) * rg.vw + (uint32_t)(nx - (int)rg.vx0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's DMA before the barrier (spatial1_ntl_body)
    if (mt.m && mt.gbuf) {   // background G-buffer records: spatial1_ntl_body's window fix-up
        constexpr uint32_t kThreads = 256u * TH, kPer = (apron_max(TH) + kThreads - 1u) / kThreads;
#pragma unroll
        for (uint32_t k = 0; k < kPer; k++) {
            const uint32_t i = threadIdx.x + kThreads * k;
            if (i < n_apron) {
                uint32_t r = __umulhi(i, 0xFFFFFFFFu / AW + 1u);
                if (r * AW > i) r--;
                const uint32_t c = i - r * AW;
                if (tile_flag_at(mt, rg, ax0 + (int)c, ay0 + (int)r) == 0u) l_nt[i] = make_float4(0.0f, 0.0f, 0.0f, ROMIS_FLT_MAX);
            }
        }
    }
    __syncthreads();
    if (!live) return;   // no barrier follows
    const float4 cn = l_nt[(uint32_t)(y - ay0) * AW + (uint32_t)(x - ax0)];
    const float cw[2] = {ch.x, ch.z};
    const uint32_t cm[2] = {__float_as_uint(ch.y), __float_as_uint(ch.w)};
    const Px cur = make_px(s, cn, cpm, origin, pix);
    // primary-ray miss (spatialn_ntl_body): both own inputs go to sub-reservoir 0, nothing is accepted
    bool miss = cur.mat == s.num_materials - 1u && s.normals_bounded && !__builtin_isnan(cur.P.x + cur.P.y + cur.P.z);
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const v3 cc = xyz(l_lt[L + 1u + (cm[j] >> 24)]);
        miss = miss && __builtin_isfinite(cw[j]) && __builtin_isfinite(cc.x + cc.y + cc.z);
    }
    if (miss) {
        const float W0[2] = {0.0f, 0.0f}, ws[2] = {ROMIS_FLT_MIN, ROMIS_FLT_MIN}, c0[2] = {0.0f, 0.0f};
        const uint32_t M[2] = {(cm[0] & kHandleM) + (cm[1] & kHandleM), 0u}, li[2] = {L, L};
        put(pix, W0, M, li, ws, c0);
        return;
    }
    const double rt = rcp_d(cur.t);
    const bool rt_all = __all(div_fast_ok(cur.t));
    bool ok[kLeanK];
    float4 qh[kLeanK];
#pragma unroll
    for (uint32_t n = 0; n < kLeanK; n++) {
        ok[n] = false;
        qh[n] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (n < K) {
            const float4 g = l_nt[qi[n]];
            const float nd = vdot(xyz(g), cur.N);
            float q = div_by_rcp_d(g.w, rt);
            if (__builtin_expect(!rt_all, 0)) {
                if (!div_fast_ok(cur.t)) q = g.w / cur.t;
            }
            ok[n] = !(nd < 0.90630778703f) && !(fabsf(1.0f - q) > 0.1f);
            if (ok[n]) qh[n] = hin[qp[n]];
        }
    }
    Comb2h cmb;
    cmb.init(ps + 2u * K * 0x9E3779B9u, L);
    auto take = [&](float W, uint32_t hm) {
        const uint32_t li = hm >> 24;
        cmb.take(target_pdf(s, f, cur, xyz(l_lt[li]), xyz(l_lt[L + 1u + li]), tb), W, hm & kHandleM, li);
    };
#pragma unroll
    for (uint32_t n = 0; n < kLeanK; n++) {
        if (ok[n]) {
            take(qh[n].x, __float_as_uint(qh[n].y));
            take(qh[n].z, __float_as_uint(qh[n].w));
        }
    }
    take(cw[0], cm[0]);
    take(cw[1], cm[1]);
    float W[2];
#pragma unroll
    for (int j = 0; j < 2; j++) {
        float p = cmb.pd[j];
        if (!cmb.has_pd[j])
            p = (f.shading && !__builtin_isnan(cur.P.x + cur.P.y + cur.P.z))
                    ? 0.0f : target_pdf(s, f, cur, xyz(l_lt[cmb.li[j]]), xyz(l_lt[L + 1u + cmb.li[j]]), tb);
        W[j] = contribution_weight(p, cmb.macc[j], cmb.wsum[j]);
    }
    put(pix, W, cmb.macc, cmb.li, cmb.wsum, cmb.chosen);
}

#ifndef ROMIS_SPATIAL2HG_WPE
#define ROMIS_SPATIAL2HG_WPE 5
#endif
#define ROMIS_SPATIAL2HG_KERNEL(DBG, TH, NAME)                                                                         \
    extern "C" __global__ __launch_bounds__(256 * TH) __attribute__((amdgpu_waves_per_eu(ROMIS_SPATIAL2HG_WPE))) void  \
    NAME(SceneDev s, Region rg, FeaturesDev f, uint32_t key, float ox, float oy, float oz, const float4* n_t,        \
         const float4* p_mat, const float4* hin, float4* oa, float4* ob, float2* odbg, float4* hout, MissTiles mt,     \
         uint32_t odead) {                                                                                            \
        spatial2hg_body<DBG, TH>(s, rg, f, key, mk(ox, oy, oz), n_t, p_mat, hin, oa, ob, odbg, hout, mt, odead);        \
    }
ROMIS_SPATIAL2HG_KERNEL(false, 1, k_spatial2hg)
ROMIS_SPATIAL2HG_KERNEL(true, 1, k_spatial2hg_dbg)
ROMIS_SPATIAL2HG_KERNEL(false, 2, k_spatial2hg_t2)
ROMIS_SPATIAL2HG_KERNEL(true, 2, k_spatial2hg_t2_dbg)

#ifndef ROMIS_SPATIAL2_NTL_WPE
#define ROMIS_SPATIAL2_NTL_WPE 4
#endif
#define ROMIS_SPATIALN_NTL_KERNEL(DBG, NT, NAME)                                                                      \
    extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ROMIS_SPATIAL2_NTL_WPE))) void     \
    NAME(SceneDev s, Region rg, FeaturesDev f, uint32_t key, float ox, float oy, float oz, const float4* n_t,        \
         const float4* p_mat, const float4* ia, const float4* ib, float4* oa, float4* ob, float2* odbg, MissTiles mt) { \
        spatialn_ntl_body<DBG, NT>(s, rg, f, key, mk(ox, oy, oz), n_t, p_mat, ia, ib, oa, ob, odbg, mt);               \
    }
ROMIS_SPATIALN_NTL_KERNEL(false, 2, k_spatial2_ntl)
ROMIS_SPATIALN_NTL_KERNEL(true, 2, k_spatial2_ntl_dbg)


// ---------------------------------------------------------------------------------------------------------
// k_spatial1u: the N = 1 unbiased pass (combineUnbiased, reservoir.cpp:68-104; C5 runs it with visibility reuse).
// Same arithmetic, RNG slots and order as spatial_pixel<1, true>; what changes is how much of it runs:
//  - the K neighbours' reservoirs are gathered once (one ahead of the consume sequence) and their M is kept for
//    the Z sum, instead of being re-read;
//  - the pixel's own target pdf comes from the producer's pdf cache (rp_in) when there is one;
//  - Z only matters when the held sample's p-hat at the pixel is non-zero (W = 0 otherwise, reservoir.cpp:99), so
//    the whole Z loop (K + 1 target pdfs at the inputs' pixels and their shadow rays) is skipped exactly then;
//  - Z's own-pixel term is p-hat(pixel, held sample) = the value W uses (the same evaluation), and the term of the
//    input the held sample came from is that input's p-hat of its own sample at its own pixel = the producer's pdf
//    cache there (rp_nb[q], the same evaluation on the same G-buffer record): one target pdf each instead of a
//    recomputation.  rp_nb is the cache as seen at neighbour pixels: the caller passes null when a neighbour may lie
//    where the producer did not write it (a halo pass's border strips read the exchanged ring, whose reservoirs
//    arrive without their pdfs), and the term is then evaluated;
//  - the shadow rays (VIS) traverse the block's LDS copy of the BVH.
// Only SoA planes (Region ps = 1) and K <= kLeanK take this path (launch_spatial checks).
template <bool DBG, bool VIS>
__device__ __forceinline__ void spatial1u_body(const SceneDev& s, const Region& rg, const FeaturesDev& f, uint32_t key,
                                               v3 origin, const float4* __restrict__ n_t, const float4* __restrict__ p_mat,
                                               const float4* __restrict__ ia, const float4* __restrict__ ib,
                                               float4* __restrict__ oa, float4* __restrict__ ob, float2* __restrict__ odbg,
                                               const float* __restrict__ rp_in, const float* __restrict__ rp_nb,
                                               float* __restrict__ rp_out, uint8_t* __restrict__ vis_out, MissTiles mt) {
    uint32_t tile;
    if (!xcd_tile(rg, num_tiles(rg), blockIdx.x, tile)) return;   // block-uniform, before any barrier
    const uint32_t ntx = (rg.rw + kTileW - 1) / kTileW;
    const int tx0 = (int)(rg.rx0 + (tile % ntx) * kTileW), ty0 = (int)(rg.ry0 + (tile / ntx) * kTileH);
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63u;
    const int x = tx0 + (int)(w * 8u + (l & 7u)), y = ty0 + (int)(l >> 3);
    const uint32_t K = f.K;   // <= kLeanK (host check)
    bool mixed = false;   // some input lies in a background tile (whose RIS reservoir may be unwritten: substituted)
    if (mt.m) {
        // the tile and every pixel its neighbour draws can reach (grown by R, clamped to the image and the view) are
        // background pixels holding (0, W = 0), (0, M = mt.m): the miss shortcut's result below with M = (K + 1) mt.m
        const int x1 = min(tx0 + (int)kTileW, (int)(rg.rx0 + rg.rw)) - 1, y1 = min(ty0 + (int)kTileH, (int)(rg.ry0 + rg.rh)) - 1;
        const int gx0 = max(max(tx0 - (int)f.R, 0), (int)rg.vx0), gy0 = max(max(ty0 - (int)f.R, 0), (int)rg.vy0);
        const int gx1 = min(min(x1 + (int)f.R, (int)rg.W - 1), (int)(rg.vx0 + rg.vw) - 1);
        const int gy1 = min(min(y1 + (int)f.R, (int)rg.H - 1), (int)(rg.vy0 + rg.vh) - 1);
        if (tiles_known_miss(mt, rg, gx0, gx1, gy0, gy1, &mixed)) {
            if (x <= x1 && y <= y1) {
                const uint32_t mo = ((uint32_t)(y - (int)rg.vy0) * rg.vw + (uint32_t)(x - (int)rg.vx0)) << 4;
                st_at(oa, mo, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
                st_at(ob, mo, make_float4(0.0f, 0.0f, 0.0f, __uint_as_float((K + 1u) * mt.m)));
                if (DBG) st_at(odbg, mo >> 1, make_float2(ROMIS_FLT_MIN, 0.0f));
                if (rp_out) st_at(rp_out, mo >> 2, 0.0f);
                if (vis_out) vis_out[mo >> 4] = 0u;
            }
            return;   // block-uniform, before the BVH's barrier
        }
    }
    const Bvh bvh = VIS ? stage_bvh(s, g_lds) : global_bvh(s);   // ends with a barrier (every thread gets here)
    const GlTabs tb = gl_stage_tables();
    if (x >= (int)(rg.rx0 + rg.rw) || y >= (int)(rg.ry0 + rg.rh)) return;
    const int rx = x - (int)rg.vx0, ry = y - (int)rg.vy0;
    const uint32_t pofs = ((uint32_t)ry * rg.vw + (uint32_t)rx) << 4;
    // an input pixel of a background tile holds the known (0, W = 0), (0, M = mt.m), pdf 0 (RIS may not have stored
    // them, its skip_res): in blocks whose neighbourhood meets such a tile (block-uniform) they are not read
    const uint32_t ntxv = (rg.vw + kTileW - 1u) / kTileW;
    auto known = [&](int vx, int vy) {   // view-relative pixel in a background tile
        return mixed && mt.flags[((uint32_t)vy / kTileH) * ntxv + (uint32_t)vx / kTileW] == 0u;
    };
    // ... nor its G-buffer records (skip_res bit 1): a miss's normal 0 and t = FLT_MAX; for its P, what the pass
    // uses of it -- not NaN (the flag's promise) -- holds for 0, and its material is the miss material
    float4 cn, cpm;
    if (known(rx, ry)) {
        cn = make_float4(0.0f, 0.0f, 0.0f, ROMIS_FLT_MAX);
        cpm = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(s.num_materials - 1u));
    } else {
        cn = ld_at(n_t, pofs);
        cpm = ld_at(p_mat, pofs);
    }
    auto ld_res = [&](uint32_t q, bool kn, float4& a, float4& b) {
        if (kn) {
            a = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            b = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(mt.m));
        } else {
            a = ld_at(ia, q);
            b = ld_at(ib, q);
        }
    };
    float4 ca, cb;
    const bool own_known = known(rx, ry);
    ld_res(pofs, own_known, ca, cb);
    const float pd_cached = (rp_in && !own_known) ? ld_at(rp_in, pofs >> 2) : 0.0f;
    // neighbour draws (render_utils.cpp:108-111), clamped to the image, then to the stored view
    const int xlo = max(0, (int)rg.vx0) - (int)rg.vx0, xhi = min((int)rg.W, (int)(rg.vx0 + rg.vw)) - 1 - (int)rg.vx0;
    const int ylo = max(0, (int)rg.vy0) - (int)rg.vy0, yhi = min((int)rg.H, (int)(rg.vy0 + rg.vh)) - 1 - (int)rg.vy0;
    const uint32_t ps = pix_state(key, (uint32_t)y * rg.W + (uint32_t)x);
    const uint32_t span = 2u * f.R + 1u;
    const int bx = rx - (int)f.R, by = ry - (int)f.R;
    uint32_t qo[kLeanK];
    bool qk[kLeanK];
#pragma unroll
    for (uint32_t n = 0; n < kLeanK; n++) {
        qo[n] = pofs;
        qk[n] = own_known;
        if (n < K) {
            const int nx = min(max(bx + (int)__umulhi(draw(ps, 2u * n), span), xlo), xhi);
            const int ny = min(max(by + (int)__umulhi(draw(ps, 2u * n + 1u), span), ylo), yhi);
            qo[n] = ((uint32_t)ny * rg.vw + (uint32_t)nx) << 4;
            qk[n] = known(nx, ny);
        }
    }
    float4 na[kLeanK], nb[kLeanK];
    ld_res(qo[0], qk[0], na[0], nb[0]);
    const Px cur = make_px(s, cn, cpm, origin, pofs >> 4);
    // A primary-ray miss: the target pdf of any sample there is exactly 0 (zero normal, kd = ks = 0: the biased pass's
    // shortcut), so with every input's W finite each weighs (0 W) M = +-0 -- nothing is accepted, wSum
    // stays FLT_MIN, the held sample is the initial (0, 0) one and W = 0 (p-hat 0, reservoir.cpp:99).  Unlike the biased
    // pass nothing is rejected (combineUnbiased takes every neighbour), so M sums all K + 1 inputs: their reservoirs are
    // still read, their K target pdfs and the Z loop are not.  (C5: 87 % of the 8K frame's pixels miss the box.)
    if (cur.mat == s.num_materials - 1u && s.normals_bounded && !__builtin_isnan(cur.P.x + cur.P.y + cur.P.z) &&
        (!rp_in || pd_cached == 0.0f)) {
        bool fin = __builtin_isfinite(ca.w) && __builtin_isfinite(na[0].w);
        uint32_t m = __float_as_uint(cb.w) + __float_as_uint(nb[0].w);
#pragma unroll
        for (uint32_t n = 1; n < kLeanK; n++) {
            if (n < K) {
                float4 a, b;
                ld_res(qo[n], qk[n], a, b);
                fin = fin && __builtin_isfinite(a.w);
                m += __float_as_uint(b.w);
            }
        }
        if (K == 0u) { fin = __builtin_isfinite(ca.w); m = __float_as_uint(cb.w); }
        if (fin) {
            st_at(oa, pofs, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
            st_at(ob, pofs, make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(m)));
            if (DBG) st_at(odbg, pofs >> 1, make_float2(ROMIS_FLT_MIN, 0.0f));
            if (rp_out) st_at(rp_out, pofs >> 2, 0.0f);
            if (vis_out) vis_out[pofs >> 4] = 0u;
            return;
        }
    }
    const float pd_cur = rp_in ? pd_cached : target_pdf(s, f, cur, xyz(ca), xyz(cb), tb);
    Comb1 cmb;
    cmb.pos = mk(0.0f, 0.0f, 0.0f); cmb.col = mk(0.0f, 0.0f, 0.0f);
    cmb.wsum = ROMIS_FLT_MIN; cmb.chosen = 0.0f; cmb.pd = 0.0f; cmb.macc = 0u; cmb.has_pd = false;
    cmb.h = ps + 2u * K * 0x9E3779B9u;
    uint32_t Mn[kLeanK];
    uint32_t src = kLeanK;   // the input the held sample came from (kLeanK = the pixel itself)
#pragma unroll
    for (uint32_t n = 0; n < kLeanK; n++) {
        if (n + 1 < kLeanK && n + 1 < K) ld_res(qo[n + 1], qk[n + 1], na[n + 1], nb[n + 1]);
        Mn[n] = 0u;
        if (n < K) {
            const v3 p = xyz(na[n]), c = xyz(nb[n]);
            Mn[n] = __float_as_uint(nb[n].w);
            if (cmb.take(target_pdf(s, f, cur, p, c, tb), na[n].w, Mn[n], p, c)) src = n;
        }
    }
    if (cmb.take(pd_cur, ca.w, __float_as_uint(cb.w), xyz(ca), xyz(cb))) src = kLeanK;
    float pc = cmb.pd;
    if (!cmb.has_pd) pc = (f.shading && !__builtin_isnan(cur.P.x + cur.P.y + cur.P.z)) ? 0.0f : target_pdf(s, f, cur, cmb.pos, cmb.col, tb);
    float W = 0.0f;
    uint8_t vis_own = 0u;
    if (pc != 0.0f) {   // W = 0 whatever Z is when p-hat(pixel, held sample) == 0 (reservoir.cpp:99)
        unsigned long long Z = 0ull;
#pragma unroll
        for (uint32_t n = 0; n < kLeanK; n++) {
            if (n < K && !qk[n]) {
                // (a background neighbour: the miss material's p-hat of any sample is +-0 or a cleaned-up NaN, never
                // positive -- no term, and its G-buffer is not read)
                const float4 qn = ld_at(n_t, qo[n]), qp = ld_at(p_mat, qo[n]);
                const Px rp = make_px(s, qn, qp, origin, qo[n] >> 4);
                const bool pos = (src == n && rp_nb) ? ld_at(rp_nb, qo[n] >> 2) > 0.0f
                                                     : target_pdf_positive(s, f, rp, cmb.pos, cmb.col, tb);
                if (pos && (!VIS || visible(bvh, rp.P, cmb.pos))) Z += Mn[n];
            }
        }
        if (pc > 0.0f) {
            const bool v = !VIS || visible(bvh, cur.P, cmb.pos);
            if (v) Z += __float_as_uint(cb.w);
            vis_own = VIS ? (v ? 1u : 2u) : 0u;
        }
        if (Z != 0ull) W = (rcp_rn(pc) * rcp_rn((float)Z)) * cmb.wsum;
    }
    // the pixel's own shadow ray to the held sample is the ray final shading casts for this pixel (the same P and
    // sample): its result is handed on (1 visible, 2 occluded, 0 not cast) when this pass's output is shaded next
    if (vis_out) vis_out[pofs >> 4] = vis_own;
    st_at(oa, pofs, make_float4(cmb.pos.x, cmb.pos.y, cmb.pos.z, W));
    st_at(ob, pofs, make_float4(cmb.col.x, cmb.col.y, cmb.col.z, __uint_as_float(cmb.macc)));
    if (DBG) st_at(odbg, pofs >> 1, make_float2(cmb.wsum, cmb.chosen));
    if (rp_out) st_at(rp_out, pofs >> 2, pc);
}

#define ROMIS_SPATIAL1U_KERNEL(DBG, VIS, NAME)                                                                         \
    extern "C" __global__ __launch_bounds__(256) ROMIS_SPATIAL_ATTR void NAME(SceneDev s, Region rg, FeaturesDev f,     \
                                                                           uint32_t key, float ox, float oy, float oz,  \
                                                                           const float4* n_t, const float4* p_mat,      \
                                                                           const float4* ia, const float4* ib,          \
                                                                           float4* oa, float4* ob, float2* odbg,        \
                                                                           const float* rp_in, const float* rp_nb,      \
                                                                           float* rp_out, uint8_t* vis_out,             \
                                                                           MissTiles mt) {                              \
        spatial1u_body<DBG, VIS>(s, rg, f, key, mk(ox, oy, oz), n_t, p_mat, ia, ib, oa, ob, odbg, rp_in, rp_nb, rp_out, \
                                 vis_out, mt);                                                                        \
    }
ROMIS_SPATIAL1U_KERNEL(false, false, k_spatial1u)
ROMIS_SPATIAL1U_KERNEL(true, false, k_spatial1u_dbg)
ROMIS_SPATIAL1U_KERNEL(false, true, k_spatial1u_vis)
ROMIS_SPATIAL1U_KERNEL(true, true, k_spatial1u_vis_dbg)


// ---------------------------------------------------------------------------------------------------------
// k_final: finalShading + exposureToneMapping + Screen::setPixel y-flip.  rgb rows: row 0 = top of rect.
// Persistent blocks stage the BVH into LDS once (shadow rays are the kernel's main cost).
template <int NT, bool LDS_BVH>
__device__ __forceinline__ void final_body(const SceneDev& s, const Region& rg, const FeaturesDev& f, v3 origin,
                                           const float4* __restrict__ n_t, const float4* __restrict__ p_mat,
                                           const float4* __restrict__ ra, const float4* __restrict__ rb,
                                           float* __restrict__ rgb) {
    const Bvh bvh = LDS_BVH ? stage_bvh(s, g_lds) : global_bvh(s);
    const GlTabs tb = gl_stage_tables();
    const size_t npx = (size_t)rg.vw * rg.vh;
    const uint32_t N = NT > 0 ? (uint32_t)NT : f.N;
    const uint32_t nt = work_items(rg);
    const float g = 1.0f / f.gamma;
    for (uint32_t tile = blockIdx.x; tile < nt; tile += gridDim.x) {
        uint32_t x, y;
        size_t p;
        if (!work_pixel(rg, tile, x, y, p)) continue;
        Px px = load_px(s, rg, n_t, p_mat, p, origin);
        v3 color = mk(0.0f, 0.0f, 0.0f);
        for (uint32_t j = 0; j < N; j++) {
            Sub r;
            sub_load(r, ra, rb, ridx(rg, j, p));
            v3 sc = shade(s, f, px, r.pos, r.col, tb);
            // The visibility test can only matter when the shaded value is non-zero: (vis ? sc : 0) * W equals
            // sc * W when sc == 0 (both are 0 * W), so the shadow ray is skipped exactly then.
            if ((sc.x != 0.0f || sc.y != 0.0f || sc.z != 0.0f) && !visible(bvh, px.P, r.pos)) sc = mk(0.0f, 0.0f, 0.0f);
            sc = vscale(sc, r.W);
            color = vadd(color, sc);
        }
        color = vdivs(color, (float)N);
        if (f.tone_map) {
            v3 e = vscale(mk(-color.x, -color.y, -color.z), f.exposure);
            v3 mapped = mk(1.0f - gl_expf(tb, e.x), 1.0f - gl_expf(tb, e.y), 1.0f - gl_expf(tb, e.z));
            // pm_powf(x, 1) == x for every x (gamma = 1, the Features default): skip the call
            color = g == 1.0f ? mapped : mk(gl_powf(tb, mapped.x, g), gl_powf(tb, mapped.y, g), gl_powf(tb, mapped.z, g));
        }
        const uint32_t row = rg.rh - 1u - (y - rg.ry0);
        float* o = rgb + 3 * ((size_t)row * rg.rw + (x - rg.rx0));
        o[0] = color.x; o[1] = color.y; o[2] = color.z;
    }
}

// N = 1 with ray binning: a wave's shadow rays are traversed in lockstep, so its cost is the union of its
// lanes' paths; rays from one 32x8 tile toward nearby targets follow nearly the same path.  The block bins its
// rays by a 256-cell grid of the target position (scene bounds = the BVH root box), lays them out in bin order
// in LDS, traces ray i on thread i, and hands each result back to its pixel.  Same rays, same arithmetic:
// only which lane traces which ray changes.  One 32x8 tile per block (every thread reaches the barriers).
// (The bin only decides which lane traces which ray, never a result: the scale is an approximate reciprocal.)
__device__ __forceinline__ uint32_t target_bin(const Bvh& b, v3 y) {
    const float4 lo = b.nodes[0], hi = b.nodes[1];
    auto q = [](float v, float l, float h, float cells) {
        float t = (v - l) * __builtin_amdgcn_rcpf(fmaxf(h - l, 1e-30f)) * cells;
        return (uint32_t)fminf(fmaxf(t, 0.0f), cells - 1.0f);
    };
    const uint32_t qx = q(y.x, lo.x, hi.x, 8.0f), qy = q(y.y, lo.y, hi.y, 8.0f), qz = q(y.z, lo.z, hi.z, 4.0f);
    // interleave (x2 y2 z1 x1 y1 z0 x0 y0) so that nearby cells get nearby bins
    return ((qx >> 2) << 7) | ((qy >> 2) << 6) | ((qz >> 1) << 5) | (((qx >> 1) & 1u) << 4) | (((qy >> 1) & 1u) << 3) |
           ((qz & 1u) << 2) | ((qx & 1u) << 1) | (qy & 1u);
}

// exposureToneMapping (tone_mapping.cpp:8-11) of a finalShading colour; gamma = 1 (the Features default) skips the power
// (pm_powf(x, 1) == x for every x)
__device__ __forceinline__ v3 tone_map_rgb(const FeaturesDev& f, v3 color, const GlTabs& tb) {
    if (!f.tone_map) return color;
    const float g = 1.0f / f.gamma;
    v3 e = vscale(mk(-color.x, -color.y, -color.z), f.exposure);
    v3 mapped = mk(1.0f - gl_expf(tb, e.x), 1.0f - gl_expf(tb, e.y), 1.0f - gl_expf(tb, e.z));
    return g == 1.0f ? mapped : mk(gl_powf(tb, mapped.x, g), gl_powf(tb, mapped.y, g), gl_powf(tb, mapped.z, g));
}

// QB: the shadow rays walk the 16-byte nodes (occluded_q, SceneDev::nodes_q; round 6) staged in LDS instead of the
// 32-byte ones -- the walk is bound by LDS throughput (probes/s6)
template <bool LDS_BVH, int NT, bool QB = false>
__device__ __forceinline__ void final_sorted_body(const SceneDev& s, const Region& rg, const FeaturesDev& f, v3 origin,
                                                  const float4* __restrict__ n_t, const float4* __restrict__ p_mat,
                                                  const float4* __restrict__ ra, const float4* __restrict__ rb,
                                                  float* __restrict__ rgb, const uint8_t* __restrict__ vis_in,
                                                  MissTiles mt) {
    // NT shadow rays per pixel (one per sub-reservoir): ray j * 256 + t is pixel t's sub-reservoir j
    constexpr uint32_t kRays = 256u * NT;
    if (mt.flags) {
        // a tile of background pixels (MissTiles): after RIS and any biased / unbiased passes each holds W = 0 and the
        // initial (0, 0) sample, which a miss pixel shades to +-0 (kd = ks = 0; a non-finite dotNL or power is cleaned
        // up; the distance |P| is not NaN): the colour is +0 -- tone mapped as below, without reading anything
        const uint32_t ntx = (rg.rw + kTileW - 1) / kTileW;
        const int tx0 = (int)(rg.rx0 + (blockIdx.x % ntx) * kTileW), ty0 = (int)(rg.ry0 + (blockIdx.x / ntx) * kTileH);
        const int x1 = min(tx0 + (int)kTileW, (int)(rg.rx0 + rg.rw)) - 1, y1 = min(ty0 + (int)kTileH, (int)(rg.ry0 + rg.rh)) - 1;
        if (tiles_known_miss(mt, rg, tx0, x1, ty0, y1)) {
            uint32_t x, y;
            size_t p;
            if (work_pixel(rg, blockIdx.x, x, y, p)) {
                const v3 color = tone_map_rgb(f, vdivs(mk(0.0f, 0.0f, 0.0f), (float)NT), gl_global_tabs());
                const uint32_t row = rg.rh - 1u - (y - rg.ry0);
                float* o = rgb + 3 * ((size_t)row * rg.rw + (x - rg.rx0));
                o[0] = color.x; o[1] = color.y; o[2] = color.z;
            }
            return;   // block-uniform, before the BVH's barrier
        }
    }
    __shared__ uint32_t s_hist[256];
    __shared__ uint32_t s_wsum[4];
    __shared__ float4 s_from[kRays], s_to[kRays];
    __shared__ uint32_t s_vis[kRays];
    Bvh bvh;
    BvhQ bq;
    if (QB) {
        bq = stage_bvh_q(s, g_lds);
        bvh = global_bvh(s);   // target_bin's root box
    } else {
        bvh = LDS_BVH ? stage_bvh(s, g_lds) : global_bvh(s);
    }
    const GlTabs tb = gl_stage_tables();
    const uint32_t t = threadIdx.x;
    uint32_t x, y;
    size_t p;
    const bool valid = work_pixel(rg, blockIdx.x, x, y, p);
    Px px;
    Sub r[NT];
    v3 sc[NT];
    bool need[NT];
#pragma unroll
    for (int j = 0; j < NT; j++) { sc[j] = mk(0.0f, 0.0f, 0.0f); need[j] = false; }
    if (valid) {
        // A primary-ray miss (the miss material: kd = ks = 0) shades every light sample to +-0 when the scene's light
        // colours are bounded (s.miss_shade_zero: the sample colour is finite, so colour x 0 x dotNL is +-0 or a NaN the
        // clean-up zeroes) and the distance is not NaN; then sum_j (+-0) W_j = +0 for finite W_j, which is what
        // W_j = 0 and sc_j = 0 give below.  Such a lane reads p_mat and the sub-reservoirs' (pos, W) only (C4 / C5:
        // 87 % of the pixels; 32 of the 64 bytes per pixel).
        const float4 pm = p_mat[p];
        bool miss = false;
        if (s.miss_shade_zero) {
            const uint32_t m = min(__float_as_uint(pm.w), s.num_materials - 1u);
            miss = m == s.num_materials - 1u && !__builtin_isnan(pm.x + pm.y + pm.z);
        }
        float4 a[NT];
#pragma unroll
        for (int j = 0; j < NT; j++) {
            a[j] = ra[ridx(rg, (uint32_t)j, p)];
            miss = miss && __builtin_isfinite(a[j].w) && !__builtin_isnan((a[j].x - pm.x) + (a[j].y - pm.y) + (a[j].z - pm.z));
        }
        if (!miss) {
            px = make_px(s, n_t[gidx(rg, p)], pm, origin, p);
#pragma unroll
            for (int j = 0; j < NT; j++) {
                r[j] = sub_from(a[j], rb[ridx(rg, (uint32_t)j, p)]);
                sc[j] = shade(s, f, px, r[j].pos, r[j].col, tb);
                need[j] = sc[j].x != 0.0f || sc[j].y != 0.0f || sc[j].z != 0.0f;   // see final_body: no ray when sc == 0
            }
        } else {
#pragma unroll
            for (int j = 0; j < NT; j++) { r[j].pos = xyz(a[j]); r[j].W = 0.0f; }
        }
    }
    // N = 1 after an unbiased + visibility pass: that pass's own-pixel ray (same P, same sample) where it cast one
    uint8_t known = 0u;
    if (NT == 1 && vis_in && valid && need[0]) {
        known = vis_in[p];
        if (known) need[0] = false;
    }
    s_hist[t] = 0u;
    __syncthreads();
    uint32_t bin[NT], rank[NT];
#pragma unroll
    for (int j = 0; j < NT; j++) {
        bin[j] = need[j] ? target_bin(bvh, r[j].pos) : 0u;
        rank[j] = need[j] ? atomicAdd(&s_hist[bin[j]], 1u) : 0u;
    }
    __syncthreads();
    // exclusive scan of the 256 bin counts: wave scan + wave totals
    const uint32_t cnt = s_hist[t];
    uint32_t inc = cnt;
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t v = __shfl_up(inc, d, 64);
        if ((t & 63u) >= d) inc += v;
    }
    if ((t & 63u) == 63u) s_wsum[t >> 6] = inc;
    __syncthreads();
    uint32_t base = 0;
    for (uint32_t w = 0; w < (t >> 6); w++) base += s_wsum[w];
    const uint32_t excl = base + inc - cnt;
    const uint32_t total = s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
    __syncthreads();
    s_hist[t] = excl;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NT; j++) {
        if (need[j]) {
            const uint32_t slot = s_hist[bin[j]] + rank[j];
            s_from[slot] = make_float4(px.P.x, px.P.y, px.P.z, __uint_as_float((uint32_t)j * 256u + t));
            s_to[slot] = make_float4(r[j].pos.x, r[j].pos.y, r[j].pos.z, 0.0f);
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NT; j++) {
        const uint32_t i = (uint32_t)j * 256u + t;
        if (i < total) {
            const float4 a = s_from[i], b = s_to[i];
            s_vis[__float_as_uint(a.w)] = (QB ? visible_q(bq, xyz(a), xyz(b)) : visible(bvh, xyz(a), xyz(b))) ? 1u : 0u;
        }
    }
    __syncthreads();
    if (!valid) return;
    // finalShading's sum in sub-reservoir order from 0 (final_body: -0 -> +0), then / N
    v3 color = mk(0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int j = 0; j < NT; j++) {
        v3 c = sc[j];
        if (need[j] && !s_vis[(uint32_t)j * 256u + t]) c = mk(0.0f, 0.0f, 0.0f);
        if (j == 0 && known == 2u) c = mk(0.0f, 0.0f, 0.0f);   // the spatial pass's ray was occluded
        color = vadd(color, vscale(c, r[j].W));
    }
    color = tone_map_rgb(f, vdivs(color, (float)NT), tb);
    const uint32_t row = rg.rh - 1u - (y - rg.ry0);
    float* o = rgb + 3 * ((size_t)row * rg.rw + (x - rg.rx0));
    o[0] = color.x; o[1] = color.y; o[2] = color.z;
}

extern "C" __global__ __launch_bounds__(256) void k_final_n1_sorted(SceneDev s, Region rg, FeaturesDev f, float ox, float oy,
                                                                   float oz, const float4* n_t, const float4* p_mat,
                                                                   const float4* ra, const float4* rb, float* rgb,
                                                                   const uint8_t* vis_in, MissTiles mt) {
    final_sorted_body<true, 1>(s, rg, f, mk(ox, oy, oz), n_t, p_mat, ra, rb, rgb, vis_in, mt);
}
extern "C" __global__ __launch_bounds__(256) void k_final_n2_sorted(SceneDev s, Region rg, FeaturesDev f, float ox, float oy,
                                                                   float oz, const float4* n_t, const float4* p_mat,
                                                                   const float4* ra, const float4* rb, float* rgb, MissTiles mt) {
    final_sorted_body<true, 2>(s, rg, f, mk(ox, oy, oz), n_t, p_mat, ra, rb, rgb, nullptr, mt);
}
extern "C" __global__ __launch_bounds__(256) void k_final_n1_sorted_q(SceneDev s, Region rg, FeaturesDev f, float ox, float oy,
                                                                     float oz, const float4* n_t, const float4* p_mat,
                                                                     const float4* ra, const float4* rb, float* rgb,
                                                                     const uint8_t* vis_in, MissTiles mt) {
    final_sorted_body<true, 1, true>(s, rg, f, mk(ox, oy, oz), n_t, p_mat, ra, rb, rgb, vis_in, mt);
}
extern "C" __global__ __launch_bounds__(256) void k_final_n2_sorted_q(SceneDev s, Region rg, FeaturesDev f, float ox, float oy,
                                                                     float oz, const float4* n_t, const float4* p_mat,
                                                                     const float4* ra, const float4* rb, float* rgb, MissTiles mt) {
    final_sorted_body<true, 2, true>(s, rg, f, mk(ox, oy, oz), n_t, p_mat, ra, rb, rgb, nullptr, mt);
}

#define ROMIS_FINAL_KERNEL(NT, LDS, NAME)                                                                              \
    extern "C" __global__ __launch_bounds__(256) void NAME(SceneDev s, Region rg, FeaturesDev f, float ox, float oy,     \
                                                          float oz, const float4* n_t, const float4* p_mat,             \
                                                          const float4* ra, const float4* rb, float* rgb) {             \
        final_body<NT, LDS>(s, rg, f, mk(ox, oy, oz), n_t, p_mat, ra, rb, rgb);                                         \
    }
ROMIS_FINAL_KERNEL(1, false, k_final_n1)
ROMIS_FINAL_KERNEL(2, false, k_final_n2)
ROMIS_FINAL_KERNEL(0, false, k_final_n0)
ROMIS_FINAL_KERNEL(1, true, k_final_n1_lds)
ROMIS_FINAL_KERNEL(2, true, k_final_n2_lds)
ROMIS_FINAL_KERNEL(0, true, k_final_n0_lds)

// ---------------------------------------------------------------------------------------------------------
// Test hooks: device powf / expf on arrays (parity of the portable math with the oracle).
extern "C" __global__ void k_debug_math(const float* x, const float* y, float* pw, float* ex, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    pw[i] = pm_powf(x[i], y[i]);
    ex[i] = pm_expf(x[i]);
}

// Halo exchange (restir_halo_pack / restir_halo_unpack): segment i's pixels, row-major, each as N x (res_a,
// res_b) pairs laid out [j][pixel] inside the segment (include/restir_c.h, restir_halo_plan).
__device__ __forceinline__ bool halo_locate(const HaloSegs& hs, uint32_t g, uint32_t& seg, uint32_t& x, uint32_t& y) {
    if (g >= hs.px0[hs.n]) return false;
    seg = 0;
    while (g >= hs.px0[seg + 1]) seg++;
    const uint32_t l = g - hs.px0[seg];
    x = hs.x0[seg] + l % hs.w[seg];
    y = hs.y0[seg] + l / hs.w[seg];
    return true;
}

extern "C" __global__ __launch_bounds__(256) void k_halo_pack(Region rg, HaloSegs hs, uint32_t N, const float4* __restrict__ ra,
                                                             const float4* __restrict__ rb, float4* __restrict__ out) {
    uint32_t seg, x, y;
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (!halo_locate(hs, g, seg, x, y)) return;
    const size_t npx = (size_t)rg.vw * rg.vh, p = (size_t)(y - rg.vy0) * rg.vw + (x - rg.vx0);
    const uint32_t spx = hs.px0[seg + 1] - hs.px0[seg], l = g - hs.px0[seg];
    for (uint32_t j = 0; j < N; j++) {
        const size_t o = 2 * ((size_t)hs.px0[seg] * N + (size_t)j * spx + l);
        out[o] = ra[ridx(rg, j, p)];
        out[o + 1] = rb[ridx(rg, j, p)];
    }
}

extern "C" __global__ __launch_bounds__(256) void k_halo_unpack(Region rg, HaloSegs hs, uint32_t N, const float4* __restrict__ in,
                                                               float4* __restrict__ ra, float4* __restrict__ rb) {
    uint32_t seg, x, y;
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (!halo_locate(hs, g, seg, x, y)) return;
    const size_t npx = (size_t)rg.vw * rg.vh, p = (size_t)(y - rg.vy0) * rg.vw + (x - rg.vx0);
    const uint32_t spx = hs.px0[seg + 1] - hs.px0[seg], l = g - hs.px0[seg];
    for (uint32_t j = 0; j < N; j++) {
        const size_t o = 2 * ((size_t)hs.px0[seg] * N + (size_t)j * spx + l);
        ra[ridx(rg, j, p)] = in[o];
        rb[ridx(rg, j, p)] = in[o + 1];
    }
}

// Streaming read (restir_measure_read_bandwidth): grid-stride 16-byte loads, 4 in flight per lane, one partial
// sum per block so nothing is dead code.
extern "C" __global__ __launch_bounds__(256) void k_read_stream(const float4* __restrict__ buf, size_t n4, float* sink) {
    // The HBM read-bandwidth probe (restir_measure_read_bandwidth): each wave sweeps its own contiguous slice in
    // order, eight 1-KiB non-temporal loads in flight per lane-iteration (8 KiB per wave, 256 KiB per CU at 8
    // blocks per CU), so DRAM pages are read sequentially and the L2 keeps none of the once-read bytes.
    const size_t waves = (size_t)gridDim.x * (blockDim.x >> 6);
    const size_t wave = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const size_t lane = threadIdx.x & 63u;
    const size_t per = (n4 / waves) & ~(size_t)511;            // whole 8-load steps per wave
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v* p = reinterpret_cast<const f4v*>(buf) + wave * per + lane;
    float acc = 0.0f;
    for (size_t k = 0; k < per; k += 512) {
        f4v v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = __builtin_nontemporal_load(p + k + 64 * u);
#pragma unroll
        for (int u = 0; u < 8; u++) acc += v[u].x + v[u].w;
    }
    for (size_t i = waves * per + wave * 64 + lane; i < n4; i += waves * 64) acc += buf[i].x;   // the remainder
    if (acc == 12345.0f) sink[blockIdx.x % 256u] = acc;   // buffers are zero: never taken, but not provably so
}

// ---------------------------------------------------------------------------------------------------------
// Host launchers (launch.h)
#include "launch.h"
#include "launch_events.h"

#include <mutex>
#include <set>

namespace romis {

void set_launch_events(hipEvent_t start, hipEvent_t stop) {
    g_ev_start = start;
    g_ev_stop = stop;
    g_launched = false;
}
bool launch_events_used() { return g_launched; }

namespace {
static_assert(kTileW * kTileH == kBlock, "one lane per tile pixel");

inline uint32_t items_of(const Region& rg) {
    return rg.map2d ? ((rg.rw + kTileW - 1) / kTileW) * ((rg.rh + kTileH - 1) / kTileH) : (rg.rw * rg.rh + kBlock - 1) / kBlock;
}
inline size_t lights_lds_bytes(const SceneDev& s) { return (size_t)7 * s.num_lights * 16; }
// The RIS light-table form (ris_pixel's LT) for this scene and N: the compact tables of the _pt / _grid kernels
// (N = 1, 2) when the scene's lights allow them and ris.compact is on, else the general records.
inline int ris_light_form(const SceneDev& s, const FeaturesDev& f, const Tuning& tu) {
    if (!tu.ris_compact || s.num_lights == 0 || (f.N != 1 && f.N != 2)) return kLtGeneral;
    if (s.light_types == 1u) return kLtPoint;
    // N = 1 (at N = 2 the form spills): ris.compact = 2 keeps the grid table (A/B runs)
    if (s.lights_regular && tu.ris_compact == 1u && f.N == 1) return kLtRegular;
    if (s.lights_grid) return kLtGrid;
    if (s.lights_pgram) return kLtPgram;
    return kLtGeneral;
}
inline size_t ris_lights_lds_bytes(const SceneDev& s, int lt) { return (size_t)lt_stride(lt) * s.num_lights * 16; }
inline Region with_map(Region rg, uint32_t map2d) { rg.map2d = map2d; return rg; }
}  // namespace

hipError_t launch_primary(const SceneDev& s, const Region& rg0, const CameraDev& cam, float4* n_t, float4* p_mat,
                          float4* n_t2, const Tuning& tu, hipStream_t stream) {
    if (rg0.rw == 0 || rg0.rh == 0) return hipSuccess;
    const Region rg = with_map(rg0, 1u);
    const size_t lds = bvh_lds_bytes(s);
    const dim3 grid(items_of(rg));
    if (tu.primary_lds && lds <= kLdsBudget)
        ROMIS_LAUNCH(k_primary_lds, grid, dim3(kBlock), lds, stream, s, rg, cam, n_t, p_mat, n_t2);
    else
        ROMIS_LAUNCH(k_primary, grid, dim3(kBlock), 0, stream, s, rg, cam, n_t, p_mat, n_t2);
    return hipGetLastError();
}

hipError_t launch_ris(const SceneDev& s, const Region& rg0, const FeaturesDev& f, uint32_t key, const float* o,
                      const float4* n_t, const float4* p_mat, float4* ra, float4* rb, float2* rdbg, float* rp,
                      const Tuning& tu, hipStream_t stream) {
    if (rg0.rw == 0 || rg0.rh == 0) return hipSuccess;
    const Region rg = with_map(rg0, 0);
    const dim3 grid(items_of(rg));
    const int lt = ris_light_form(s, f, tu);
    const size_t lds = ris_lights_lds_bytes(s, lt);
    const bool staged = tu.ris_lds && s.num_lights > 0 && lds <= kLdsBudget;
    auto k = lt == kLtRegular ? (staged ? k_ris_n1_lds_reg : k_ris_n1_reg)
           : lt == kLtPoint ? (staged ? (f.N == 1 ? k_ris_n1_lds_pt : k_ris_n2_lds_pt) : (f.N == 1 ? k_ris_n1_pt : k_ris_n2_pt))
           : lt == kLtGrid ? (staged ? (f.N == 1 ? k_ris_n1_lds_grid : k_ris_n2_lds_grid)
                                     : (f.N == 1 ? k_ris_n1_grid : k_ris_n2_grid))
           : lt == kLtPgram ? (staged ? (f.N == 1 ? k_ris_n1_lds_pg : k_ris_n2_lds_pg) : (f.N == 1 ? k_ris_n1_pg : k_ris_n2_pg))
           : staged ? (f.N == 1 ? k_ris_n1_lds : (f.N == 2 ? k_ris_n2_lds : k_ris_n0_lds))
                    : (f.N == 1 ? k_ris_n1 : (f.N == 2 ? k_ris_n2 : k_ris_n0));
    const size_t lds_used = lds;
    ROMIS_LAUNCH(k, grid, dim3(kBlock), staged ? lds_used : 0, stream, s, rg, f, key, o[0], o[1], o[2], n_t, p_mat, ra,
                       rb, rdbg, f.N == 1 ? rp : nullptr);
    return hipGetLastError();
}

hipError_t launch_primary_ris(const SceneDev& s, const Region& rg0, const CameraDev& cam, const FeaturesDev& f, uint32_t key,
                              float4* n_t, float4* p_mat, float4* n_t2, float4* ra, float4* rb, float2* rdbg,
                              float* rp, const Tuning& tu, hipStream_t stream, uint8_t* tmiss, uint32_t skip_res,
                              bool* tmiss_written, Handles h) {
    if (tmiss_written) *tmiss_written = false;
    if (rg0.rw == 0 || rg0.rh == 0) return hipSuccess;
    const Region rg = with_map(rg0, 1u);
    // MissTiles flags: one 32 x 8 tile per block, N <= 2 (the caller allocates one byte per tile and passes them on
    // only when *tmiss_written)
    if (!rg.map2d || f.N > 2) tmiss = nullptr;
    if (tmiss_written) *tmiss_written = tmiss != nullptr;
    const size_t bvh = bvh_lds_bytes(s);
    if (bvh > kLdsBudget) return hipErrorInvalidValue;   // caller checks primary_ris_fits()
    const int lt = ris_light_form(s, f, tu);
    const size_t lights = ris_lights_lds_bytes(s, lt);
    const bool use_lights = tu.ris_lds && s.num_lights > 0 && bvh + lights <= kLdsBudget;
    auto k = lt == kLtRegular ? (use_lights ? k_primary_ris_n1_lds_reg : k_primary_ris_n1_reg)
           : lt == kLtPoint ? (use_lights ? (f.N == 1 ? k_primary_ris_n1_lds_pt : k_primary_ris_n2_lds_pt)
                                          : (f.N == 1 ? k_primary_ris_n1_pt : k_primary_ris_n2_pt))
           : lt == kLtGrid ? (use_lights ? (f.N == 1 ? k_primary_ris_n1_lds_grid : k_primary_ris_n2_lds_grid)
                                         : (f.N == 1 ? k_primary_ris_n1_grid : k_primary_ris_n2_grid))
           : lt == kLtPgram ? (use_lights ? (f.N == 1 ? k_primary_ris_n1_lds_pg : k_primary_ris_n2_lds_pg)
                                          : (f.N == 1 ? k_primary_ris_n1_pg : k_primary_ris_n2_pg))
           : use_lights ? (f.N == 1 ? k_primary_ris_n1_lds : (f.N == 2 ? k_primary_ris_n2_lds : k_primary_ris_n0_lds))
                        : (f.N == 1 ? k_primary_ris_n1 : (f.N == 2 ? k_primary_ris_n2 : k_primary_ris_n0));
    ROMIS_LAUNCH(k, dim3(items_of(rg)), dim3(kBlock), bvh + (use_lights ? lights : 0), stream, s, rg,
                 cam, f, key, n_t, p_mat, n_t2, ra, rb, rdbg, f.N == 1 ? rp : nullptr,
                 (tu.ris_late ? 1u : 0u) | (tu.primary_tl ? 2u : 0u), tmiss,
                 tmiss ? skip_res : 0u, ((lt == kLtPoint || lt == kLtRegular) && f.N == 1) || (lt == kLtPoint && f.N == 2) ? h.w : nullptr,
                 lt == kLtPoint && f.N == 1 ? h.m : nullptr, h.w && (lt == kLtPoint || lt == kLtRegular) ? h.res_dead : 0u);
    return hipGetLastError();
}

bool primary_ris_temporal_fits(const SceneDev& s, const FeaturesDev& f, const Tuning& tu) {
    const int lt = ris_light_form(s, f, tu);
    return tu.fuse_temporal && (f.N == 1 || f.N == 2) && lt == kLtPoint && tu.ris_lds && s.num_lights > 0 &&
           bvh_lds_bytes(s) + ris_lights_lds_bytes(s, lt) <= kLdsBudget;
}

hipError_t launch_primary_ris_temporal(const SceneDev& s, const Region& rg0, const CameraDev& cam, const FeaturesDev& f,
                                       uint32_t key, float4* n_t, float4* p_mat, float4* n_t2, float4* ra, float4* rb,
                                       float2* rdbg, float* rp, const Tuning& tu, hipStream_t stream, TemporalIn tin,
                                       Handles h) {
    if (rg0.rw == 0 || rg0.rh == 0) return hipSuccess;
    if (!primary_ris_temporal_fits(s, f, tu)) return hipErrorInvalidValue;   // the caller checks
    if (f.N != 1 && f.N != 2 && (h.w || tin.hw)) return hipErrorInvalidValue;   // handles: N = 1 / 2
    const Region rg = with_map(rg0, 1u);
    const size_t lds = bvh_lds_bytes(s) + ris_lights_lds_bytes(s, kLtPoint);
    auto k = f.N == 1 ? k_primary_ris_n1_lds_pt_temporal : k_primary_ris_n2_lds_pt_temporal;
    ROMIS_LAUNCH(k, dim3(items_of(rg)), dim3(kBlock), lds, stream, s, rg, cam, f, key, n_t, p_mat, n_t2, ra, rb, rdbg,
                 f.N == 1 ? rp : nullptr, (tu.ris_late ? 1u : 0u) | (tu.primary_tl ? 2u : 0u), tin, h.w, h.m,
                 h.w ? h.res_dead : 0u);
    return hipGetLastError();
}

bool primary_ris_fits(const SceneDev& s) { return bvh_lds_bytes(s) <= kLdsBudget; }

int spatial_handle_kind(const SceneDev& s, const FeaturesDev& f, const Tuning& tu, uint32_t passes, uint64_t m0) {
    if (!tu.spatial_handles || passes == 0 || (f.N != 1 && f.N != 2) || f.unbiased || f.K > kLeanK || f.R > kLdsSpatialR)
        return -1;
    if (!tu.spatial_lean || !tu.ris_compact || s.num_lights == 0) return -1;
    int hk;
    uint32_t mmax;
    if (f.N == 2) {   // point lights: the 16-byte handle records of k_spatial2hg (spatial.n2h)
        if (!tu.spatial_n2h || s.light_types != 1u || s.num_lights > 254u) return -1;
        hk = 2; mmax = kHandleM;
    } else if (s.light_types == 1u && s.num_lights <= 254u) {   // point lights (k_spatial1h); index L = the zero sample
        hk = 0; mmax = kHandleM;
    } else if (ris_light_form(s, f, tu) == kLtRegular && tu.spatial_th != 1u && s.num_lights <= 1024u) {
        // a regular light grid (RIS's kLtRegular form; k_spatial1g_t2, 32 x 16 tiles, <= 16 KB of colours in LDS)
        hk = 1; mmax = kHandleMG;
    } else {
        return -1;
    }
    // every M: RIS M (or m0: after temporal reuse), then each biased pass sums at most K + 1 inputs
    uint64_t m = m0 ? m0 : f.M;
    if (m > mmax) return -1;
    for (uint32_t p = 0; p < passes && m <= mmax; p++) m *= (uint64_t)(f.K + 1u);
    return m <= mmax ? hk : -1;
}
bool spatial_handles_ok(const SceneDev& s, const FeaturesDev& f, const Tuning& tu, uint32_t passes) {
    return spatial_handle_kind(s, f, tu, passes) >= 0;
}

// launch_spatial's N = 1 pass reads background tiles through MissTiles (k_spatial1_ntl / _t2 biased, k_spatial1u[_vis]
// unbiased) for these features and knobs, SoA planes -- the condition for RIS's skip_res
// launch_final's k_final_n1_sorted writes background tiles from the flags without reading them
bool final_reads_flags(const SceneDev& s, const FeaturesDev& f, const Tuning& tu) {
    return f.N == 1 && tu.final_sort && tu.final_lds && bvh_lds_bytes(s) <= kLdsBudget;
}

bool spatial_reads_flags(const SceneDev& s, const FeaturesDev& f, const Tuning& tu) {
    if (f.N != 1 || f.K > kLeanK || !tu.spatial_lean) return false;
    if (f.unbiased) return !f.spatial_vis || bvh_lds_bytes(s) <= kLdsBudget;   // k_spatial1u[_vis]
    return f.R <= kLdsSpatialR;                                               // k_spatial1_ntl / _t2, k_spatial1h
}

hipError_t launch_temporal(const SceneDev& s, const Region& rg0, const FeaturesDev& f, uint32_t key, const float* o,
                           const float4* n_t, const float4* p_mat, const float4* ca, const float4* cb,
                           const float4* pa, const float4* pb, float4* oa, float4* ob, float2* odbg,
                           const float* rp_in, float* rp_out, const Tuning& tu, hipStream_t stream) {
    (void)tu;
    if (rg0.rw == 0 || rg0.rh == 0) return hipSuccess;
    const Region rg = with_map(rg0, 0);
    auto k = f.N == 1 ? k_temporal_n1 : (f.N == 2 ? k_temporal_n2 : k_temporal_n0);
    ROMIS_LAUNCH(k, dim3(items_of(rg)), dim3(kBlock), 0, stream, s, rg, f, key, o[0], o[1], o[2], n_t, p_mat, ca, cb,
                       pa, pb, oa, ob, odbg, f.N == 1 ? rp_in : nullptr, f.N == 1 ? rp_out : nullptr);
    return hipGetLastError();
}

hipError_t launch_spatial(const SceneDev& s, const Region& rg0, const FeaturesDev& f, uint32_t key, const float* o,
                          const float4* n_t, const float4* p_mat, const float4* ia, const float4* ib, float4* oa,
                          float4* ob, float2* odbg, const float* rp_in, const float* rp_nb, float* rp_out,
                          bool* rp_written, const Tuning& tu, hipStream_t stream, uint8_t* vis_out, bool* vis_written,
                          MissTiles mt, Handles hin, Handles hout) {
    if (rp_written) *rp_written = false;
    if (!mt.flags) mt.m = mt.gbuf = 0u;
    if (vis_written) *vis_written = false;
    if (rg0.rw == 0 || rg0.rh == 0) return hipSuccess;
    Region rg = with_map(rg0, 2u);   // 32 x 8 tiles of 8 x 8 waves (the lean kernels' XCD tile order, xcd_tile)
    uint32_t grid = items_of(rg);
    const size_t bvh_bytes = bvh_lds_bytes(s);
    const bool lean = tu.spatial_lean && f.N == 1 && f.K <= kLeanK && rg.ps == 1u && rg.map2d == 2u &&
                      (size_t)rg.vw * rg.vh * 16u <= 0xFFFFFFFFull;
    // N = 2 planes: byte offsets of both sub-reservoir planes within 32 bits
    const bool lean2 = tu.spatial_lean && f.N == 2 && f.K <= kLeanK && rg.ps == 1u && rg.map2d == 2u &&
                       (size_t)rg.js * 16u + (size_t)rg.vw * rg.vh * 16u <= 0xFFFFFFFFull;
    if (lean && f.unbiased && (!f.spatial_vis || bvh_bytes <= kLdsBudget)) {
        // combineUnbiased, N = 1: one block per tile in the XCD order of the biased pass (xcd_tile)
        const uint32_t ntx = (rg.rw + kTileW - 1) / kTileW, nty = (rg.rh + kTileH - 1) / kTileH;
        rg.xcd_rows = tu.spatial_xcd_rows == kXcdRowsAuto ? std::max(1u, std::min(8u, 8192u / std::max(rg.rw, 1u)))
                                                          : tu.spatial_xcd_rows;
        rg.xcd_cols = tu.spatial_xcd_cols == kXcdColsAuto ? 0u : tu.spatial_xcd_cols;
        if (rg.xcd_rows) grid = xcd_grid(rg, ntx, nty);
        auto k = f.spatial_vis ? (odbg ? k_spatial1u_vis_dbg : k_spatial1u_vis) : (odbg ? k_spatial1u_dbg : k_spatial1u);
        uint8_t* vo = f.spatial_vis ? vis_out : nullptr;   // the own-pixel shadow ray, for final shading (N = 1)
        ROMIS_LAUNCH(k, dim3(grid), dim3(kBlock), f.spatial_vis ? bvh_bytes : 0, stream, s, rg, f, key, o[0], o[1], o[2],
                     n_t, p_mat, ia, ib, oa, ob, odbg, rp_in, rp_in ? rp_nb : nullptr, rp_out, vo, mt);
        if (rp_written) *rp_written = rp_out != nullptr;
        if (vis_written) *vis_written = vo != nullptr;
        return hipGetLastError();
    }
    if (lean2 && !f.unbiased && f.R <= kLdsSpatialR) {
        // N = 2 biased: one block per tile in the XCD chunk order (xcd_tile); spatial.lds != 3 selects the general
        // kernel for A/B runs, as for N = 1.  No pdf cache at N = 2 (*rp_written stays false)
        const uint32_t ntx = (rg.rw + kTileW - 1) / kTileW, nty = (rg.rh + kTileH - 1) / kTileH;
        rg.xcd_rows = tu.spatial_xcd_rows == kXcdRowsAuto ? std::max(1u, std::min(8u, 8192u / std::max(rg.rw, 1u)))
                                                          : tu.spatial_xcd_rows;
        rg.xcd_cols = tu.spatial_xcd_cols == kXcdColsAuto ? 0u : tu.spatial_xcd_cols;
        if (hin.w) {
            // handle records (k_spatial2hg[_t2], spatial_handle_kind 2): 32 x 8 TH tiles, TH = spatial.th (auto 1)
            if (s.light_types != 1u) return hipErrorInvalidValue;
            const uint32_t th = tu.spatial_th == 2u ? 2u : 1u, ntyh = (rg.rh + th * kTileH - 1) / (th * kTileH);
            if (th == 2u && rg.xcd_rows && tu.spatial_xcd_rows == kXcdRowsAuto) rg.xcd_rows = std::max(1u, rg.xcd_rows / 2u);
            grid = rg.xcd_rows ? xcd_grid(rg, ntx, ntyh) : ntx * ntyh;
            const size_t lds = (size_t)apron_max(th) * 16u + (size_t)(2u * s.num_lights + 2u) * 16u;
            auto k = th == 2u ? (odbg ? k_spatial2hg_t2_dbg : k_spatial2hg_t2) : (odbg ? k_spatial2hg_dbg : k_spatial2hg);
            ROMIS_LAUNCH(k, dim3(grid), dim3(th * kBlock), lds, stream, s, rg, f, key, o[0], o[1], o[2], n_t, p_mat,
                         reinterpret_cast<const float4*>(hin.w), oa, ob, odbg, reinterpret_cast<float4*>(hout.w), mt,
                         hout.res_dead);
            return hipGetLastError();
        }
        if (rg.xcd_rows) grid = xcd_grid(rg, ntx, nty);
        ROMIS_LAUNCH(odbg ? k_spatial2_ntl_dbg : k_spatial2_ntl, dim3(grid), dim3(kBlock), kApronMax * 16u, stream, s, rg, f,
                     key, o[0], o[1], o[2], n_t, p_mat, ia, ib, oa, ob, odbg, mt);
        return hipGetLastError();
    }
    if (lean && !f.unbiased && f.R <= kLdsSpatialR) {
        // one block per tile (the lean kernels do not loop over tiles, so spatial.blocks does not apply here),
        // grid rounded to the XCD that owns the most tiles (xcd_tile)
        const uint32_t ntx = (rg.rw + kTileW - 1) / kTileW, nty = (rg.rh + kTileH - 1) / kTileH;
        rg.xcd_rows = tu.spatial_xcd_rows;
        if (rg.xcd_rows == kXcdRowsAuto) {
            // a chunk's records (n_t, p_mat, res_a, res_b: 64 B/px over 8-px tile rows) within one XCD's 4 MB L2:
            // 4 tile rows at 1920 px, 2 at 3840 (kbench: 4K 239 -> 225 us with 2, 1080p best with 4; r2bb)
            rg.xcd_rows = std::max(1u, std::min(8u, 8192u / std::max(rg.rw, 1u)));
        }
        rg.xcd_cols = tu.spatial_xcd_cols == kXcdColsAuto ? 0u : tu.spatial_xcd_cols;
        if (rg.xcd_rows) grid = xcd_grid(rg, ntx, nty);
        // 32x16 tiles (k_spatial1_ntl_t2) where the auto XCD chunk is at most 2 tile rows (wide images): C4 222 ->
        // 203 us, C2 76.8 -> 79.0 (cfg_kbench, profiles/r3/r3k); spatial.th = 1 / 2 forces either
        const uint32_t th = tu.spatial_th ? tu.spatial_th : (8192u / std::max(rg.rw, 1u) <= 2u ? 2u : 1u);
        if (hin.w && s.light_types != 1u) {
            // light-grid handles (spatial_handle_kind 1): k_spatial1_ntl_t2's grid, the colours behind the window
            if (tu.spatial_th == 1u) return hipErrorInvalidValue;
            const uint32_t nty2 = (rg.rh + 2u * kTileH - 1) / (2u * kTileH);
            if (rg.xcd_rows) {
                if (tu.spatial_xcd_rows == kXcdRowsAuto) rg.xcd_rows = std::max(1u, rg.xcd_rows / 2u);
                if (tu.spatial_xcd_rows == kXcdRowsAuto && tu.spatial_xcd_cols == kXcdColsAuto && ntx >= 64u) {
                    // wide frames: 2-D chunks of 4 x 8 tiles (128 x 64 px), so the +-R window rows of vertically
                    // adjacent tiles are re-read from one XCD's L2: C4f HBM traffic 1.30 -> 1.01x algorithmic (FETCH
                    // 770 -> 541 MB a launch), spatial 404.5 -> 398.2 us (round 6, profiles/r6/probes/s4)
                    rg.xcd_rows = 4u;
                    rg.xcd_cols = 8u;
                }
                grid = xcd_grid(rg, ntx, nty2);
            } else {
                grid = ntx * nty2;
            }
            ROMIS_LAUNCH(odbg ? k_spatial1g_t2_dbg : k_spatial1g_t2, dim3(grid), dim3(2u * kBlock),
                         apron_max(2) * 16u + s.num_lights * 16u, stream, s, rg, f, key, o[0], o[1], o[2], n_t, p_mat, oa,
                         ob, odbg, rp_in, rp_out, mt, reinterpret_cast<const float4*>(hin.w),
                         reinterpret_cast<float4*>(hout.w), hout.res_dead);
        } else if (hin.w && tu.spatial_gather && tu.spatial_th != 1u) {
            // sample handles gathered instead of staged (k_spatial1hg_t2, spatial.gather; round 6): 32 x 16 tiles, the
            // automatic XCD chunk one tile row as for k_spatial1h_t2
            const uint32_t ntyh = (rg.rh + 2u * kTileH - 1) / (2u * kTileH);
            if (rg.xcd_rows) {
                if (tu.spatial_xcd_rows == kXcdRowsAuto) rg.xcd_rows = 1u;
                grid = xcd_grid(rg, ntx, ntyh);
            } else {
                grid = ntx * ntyh;
            }
            const size_t lds = (size_t)apron_max(2) * 16u + (size_t)(2u * s.num_lights + 2u) * 16u;
            const HandlesIn hi{hin.w, hin.m};
            ROMIS_LAUNCH(odbg ? k_spatial1hg_t2_dbg : k_spatial1hg_t2, dim3(grid), dim3(2u * kBlock), lds, stream, s, rg, f,
                         key, o[0], o[1], o[2], n_t, p_mat, hi, oa, ob, odbg, rp_in, rp_out, hout.w, hout.m, mt,
                         hout.res_dead);
        } else if (hin.w) {
            // sample handles (k_spatial1h[_t2]): 32 x 8 TH tiles, TH = spatial.th (auto: 2 -- C2 66.9 us against 76.2 for
            // 32 x 8, 70.6 / 68.4 for 32 x 24 / 32 x 32, kbench, profiles/r5); the XCD chunks hold xcd_rows tile rows,
            // automatically one 32 x 16 row (C2: 66.1 / 65.7 us against 66.7 / 66.3 with two, 72.9 / 72.5 with four;
            // profiles/r5/probes/r5p23)
            const uint32_t hth = tu.spatial_th ? tu.spatial_th : 2u;
            if (hth > 1u) {
                const uint32_t ntyh = (rg.rh + hth * kTileH - 1) / (hth * kTileH);
                if (rg.xcd_rows) {
                    if (tu.spatial_xcd_rows == kXcdRowsAuto) rg.xcd_rows = 1u;
                    grid = xcd_grid(rg, ntx, ntyh);
                } else {
                    grid = ntx * ntyh;
                }
            } else if (tu.spatial_xcd_cols == kXcdColsAuto && rg.xcd_rows && ntx >= 24u) {
                if (tu.spatial_xcd_rows == kXcdRowsAuto) rg.xcd_rows = 8u;
                rg.xcd_cols = (ntx + 2u) / 3u;
                grid = xcd_grid(rg, ntx, nty);
            }
            const size_t lds = (size_t)h_lds_f4(hth) * 16u + (size_t)(2u * s.num_lights + 2u) * 16u;
            const HandlesIn hi{hin.w, hin.m};
            auto k = hth == 2u ? (odbg ? k_spatial1h_t2_dbg : k_spatial1h_t2) : (odbg ? k_spatial1h_dbg : k_spatial1h);
            ROMIS_LAUNCH(k, dim3(grid), dim3(hth * kBlock), lds, stream, s, rg, f, key, o[0], o[1], o[2], n_t, p_mat, hi, oa,
                         ob, odbg, rp_in, rp_out, hout.w, hout.m, mt, hout.res_dead);
        } else if (th >= 2u) {
            // 32x16 tiles: the chunks hold half as many (twice as tall) tile rows
            const uint32_t nty2 = (rg.rh + 2u * kTileH - 1) / (2u * kTileH);
            if (rg.xcd_rows) {
                // an explicit spatial.xcd_rows counts 32 x 16 tile rows here; the automatic one is halved
                if (tu.spatial_xcd_rows == kXcdRowsAuto) rg.xcd_rows = std::max(1u, rg.xcd_rows / 2u);
                grid = xcd_grid(rg, ntx, nty2);
            } else {
                grid = ntx * nty2;
            }
            ROMIS_LAUNCH(odbg ? k_spatial1_ntl_t2_dbg : k_spatial1_ntl_t2, dim3(grid), dim3(2u * kBlock),
                         apron_max(2) * 16u, stream, s, rg, f, key, o[0], o[1], o[2], n_t, p_mat, ia, ib, oa, ob, odbg,
                         rp_in, rp_out, mt);
        } else {
            if (tu.spatial_xcd_cols == kXcdColsAuto && rg.xcd_rows && ntx >= 24u) {
                // 2-D chunks: 8 tile rows x a third of the tile row (an odd number of chunks per chunk row, so the
                // round-robin XCDs cover every column).  C2: fetch 83 -> 66 B/px at the same time (profiles/r4/r4g,
                // r4h): the window rows a chunk's consecutive tile rows share stay in the XCD's L2.
                if (tu.spatial_xcd_rows == kXcdRowsAuto) rg.xcd_rows = 8u;
                rg.xcd_cols = (ntx + 2u) / 3u;
                grid = xcd_grid(rg, ntx, nty);
            }
            ROMIS_LAUNCH(odbg ? k_spatial1_ntl_dbg : k_spatial1_ntl, dim3(grid), dim3(kBlock),
                         kApronMax * 16u, stream,
                         s, rg, f, key, o[0], o[1], o[2], n_t, p_mat, ia, ib, oa, ob, odbg, rp_in, rp_out, mt);
        }
        if (rp_written) *rp_written = rp_out != nullptr;
        return hipGetLastError();
    }
    if (hin.w) return hipErrorInvalidValue;   // handles without a handle pass: the producer skipped the reservoirs
    auto k = f.unbiased ? (f.N == 1 ? k_spatial_n1_unbiased : (f.N == 2 ? k_spatial_n2_unbiased : k_spatial_n0_unbiased))
                        : (f.N == 1 ? k_spatial_n1_biased : (f.N == 2 ? k_spatial_n2_biased : k_spatial_n0_biased));
    const uint32_t bvh_lds = (f.unbiased && f.spatial_vis && bvh_bytes <= kLdsBudget) ? 1u : 0u;
    ROMIS_LAUNCH(k, dim3(grid), dim3(kBlock), bvh_lds ? bvh_bytes : 0, stream, s, rg, f, key, o[0], o[1], o[2], n_t, p_mat,
                       ia, ib, oa, ob, odbg, bvh_lds);
    return hipGetLastError();
}

hipError_t launch_final(const SceneDev& s, const Region& rg0, const FeaturesDev& f, const float* o, const float4* n_t,
                        const float4* p_mat, const float4* ra, const float4* rb, float* rgb, const Tuning& tu,
                        hipStream_t stream, const uint8_t* vis_in, MissTiles mt) {
    if (rg0.rw == 0 || rg0.rh == 0) return hipSuccess;
    const Region rg = with_map(rg0, 1u);
    const size_t lds = bvh_lds_bytes(s);
    const bool use_lds = tu.final_lds && lds <= kLdsBudget;
    auto k = use_lds ? (f.N == 1 ? k_final_n1_lds : (f.N == 2 ? k_final_n2_lds : k_final_n0_lds))
                     : (f.N == 1 ? k_final_n1 : (f.N == 2 ? k_final_n2 : k_final_n0));
    if (tu.final_sort && use_lds && (f.N == 1 || f.N == 2) && rg.map2d) {   // one tile per block
        SceneDev sf = s;
        if (!tu.final_miss) sf.miss_shade_zero = 0u;   // final.miss = 0: no miss shortcut (A/B runs)
        if ((tu.final_qbvh == 1u || (tu.final_qbvh == 2u && f.N == 2)) && s.nodes_q_ok) {   // 16-byte nodes (occluded_q)
            const size_t lq = ((size_t)s.num_nodes + (size_t)3 * s.num_tris) * 16;
            if (f.N == 1)
                ROMIS_LAUNCH(k_final_n1_sorted_q, dim3(items_of(rg)), dim3(kBlock), lq, stream, sf, rg, f, o[0], o[1], o[2],
                             n_t, p_mat, ra, rb, rgb, vis_in, rg.map2d ? mt : MissTiles{nullptr, 0u, 0u});
            else
                ROMIS_LAUNCH(k_final_n2_sorted_q, dim3(items_of(rg)), dim3(kBlock), lq, stream, sf, rg, f, o[0], o[1], o[2],
                             n_t, p_mat, ra, rb, rgb, rg.map2d ? mt : MissTiles{nullptr, 0u, 0u});
            return hipGetLastError();
        }
        if (f.N == 1)
            ROMIS_LAUNCH(k_final_n1_sorted, dim3(items_of(rg)), dim3(kBlock), lds, stream, sf, rg, f, o[0], o[1], o[2], n_t,
                         p_mat, ra, rb, rgb, vis_in, rg.map2d ? mt : MissTiles{nullptr, 0u, 0u});
        else
            ROMIS_LAUNCH(k_final_n2_sorted, dim3(items_of(rg)), dim3(kBlock), lds, stream, sf, rg, f, o[0], o[1], o[2], n_t,
                         p_mat, ra, rb, rgb, rg.map2d ? mt : MissTiles{nullptr, 0u, 0u});
        return hipGetLastError();
    }
    ROMIS_LAUNCH(k, dim3(items_of(rg)), dim3(kBlock), use_lds ? lds : 0, stream, s, rg, f,
                       o[0], o[1], o[2], n_t, p_mat, ra, rb, rgb);
    return hipGetLastError();
}

hipError_t launch_halo_pack(const Region& rg, const HaloSegs& hs, uint32_t N, const float4* ra, const float4* rb, float4* out,
                            hipStream_t stream) {
    const uint32_t n = hs.px0[hs.n];
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_halo_pack, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, rg, hs, N, ra, rb, out);
    return hipGetLastError();
}

hipError_t launch_halo_unpack(const Region& rg, const HaloSegs& hs, uint32_t N, const float4* in, float4* ra, float4* rb,
                              hipStream_t stream) {
    const uint32_t n = hs.px0[hs.n];
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_halo_unpack, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, rg, hs, N, in, ra, rb);
    return hipGetLastError();
}

hipError_t launch_read_stream(const float4* buf, size_t n4, float* sink, hipStream_t stream) {
    hipLaunchKernelGGL(k_read_stream, dim3(256 * 8), dim3(kBlock), 0, stream, buf, n4, sink);   // 8 blocks per CU, one round
    return hipGetLastError();
}

hipError_t launch_debug_math(const float* x, const float* y, float* pw, float* ex, uint32_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_debug_math, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, x, y, pw, ex, n);
    return hipGetLastError();
}

}  // namespace romis

// mis.hip -- hand-written gfx950 kernels of the repo's namesake estimators, R-MIS and R-OMIS (renderRMIS /
// renderROMIS, render.cpp:64-265): neighbour-selection grid, per-iteration accumulation, the
// per-pixel least-squares solve (Eigen's CompleteOrthogonalDecomposition restated) and the combination to screen.
#include "kernels_common.h"

// ---------------------------------------------------------------------------------------------------------
// R-MIS / R-OMIS (renderRMIS / renderROMIS, render.cpp:64-265).  Whole images: the view is the W x H image and
// pixel index p = y * W + x; reservoir planes [N][pixels], neighbourhoods in MIS_NBR, accumulators in MIS_ACC
// (include/restir_c.h RESTIR_BUF_MIS_*).  One lane per pixel; the per-pixel loops follow the reference's order.

// HitInfo::geometryId: the mesh index (rtcAttachGeometry order, embree_interface.cpp:46-47; one material per mesh);
// a primary miss keeps genPrimaryRayHits' value-initialised HitInfo (render_utils.cpp:15): 0.
__device__ __forceinline__ uint32_t geom_id_of(const SceneDev& s, float4 pm) {
    const uint32_t m = __float_as_uint(pm.w);
    return m + 1u >= s.num_materials ? 0u : m;
}

// areSimilar (neighbour_selection.cpp:7-22), lhs = the canonical pixel; the normal test compares the dot product
// with the radians field, as the reference does (maxDiffCos is computed and unused)
__device__ __forceinline__ bool are_similar(const SceneDev& s, const FeaturesDev& f, float4 ln, uint32_t lg, float4 rn,
                                            float4 rp) {
    if (f.same_geom && lg != geom_id_of(s, rp)) return false;
    const float depthFracDiff = fabsf(1.0f - (ln.w / rn.w));
    if (depthFracDiff > f.depth_frac) return false;
    const float normalsDotProd = vdot(xyz(ln), xyz(rn));
    if (normalsDotProd < f.normal_rad) return false;
    return true;
}

struct MisWin { int x0, y0, x1, y1; };

// indicesSimilarity's window walk (y outer, x inner, the pixel itself skipped) appending one class (similar 1 /
// dissimilar 0): all members, or std::sample's selection sampling of `want` of the class's `len` members (member i
// kept iff U{0..len-1-i}, keyed slot i, < the number still needed)
__device__ uint32_t mis_emit_class(const SceneDev& s, const FeaturesDev& f, const float4* __restrict__ n_t,
                                   const float4* __restrict__ p_mat, uint32_t W, MisWin w, uint32_t p, float4 cn,
                                   uint32_t cg, int cls, uint64_t len, uint64_t want, bool take_all, uint32_t ps,
                                   uint32_t* __restrict__ nbr, size_t npx, uint32_t n) {
    uint64_t needed = take_all ? len : (want < len ? want : len);
    uint64_t i = 0;
    for (int ny = w.y0; ny <= w.y1 && needed; ny++) {
        for (int nx = w.x0; nx <= w.x1 && needed; nx++) {
            const uint32_t q = (uint32_t)ny * W + (uint32_t)nx;
            if (q == p || (int)are_similar(s, f, cn, cg, n_t[q], p_mat[q]) != cls) continue;
            const bool keep = take_all || (uint64_t)uniform_index(draw(ps, (uint32_t)i), (uint32_t)(len - i)) < needed;
            if (keep) { nbr[(size_t)(1u + n) * npx + p] = q; n++; needed--; }
            i++;
        }
    }
    return n;
}

// The same walk over the count pass's similarity bits (window member m = bit m, LDS word m / 32 of the lane, stride
// 256): windows of up to kMisMaskBits members skip re-evaluating areSimilar in the emit passes.
constexpr uint32_t kMisMaskWords = 14, kMisMaskBits = 32u * kMisMaskWords;   // 448 >= (2 * 10 + 1)^2 - 1
__device__ uint32_t mis_emit_class_mask(const uint32_t* __restrict__ mask, uint32_t W, MisWin w, uint32_t p, int cls,
                                        uint64_t len, uint64_t want, bool take_all, uint32_t ps,
                                        uint32_t* __restrict__ nbr, size_t npx, uint32_t n) {
    uint64_t needed = take_all ? len : (want < len ? want : len);
    uint64_t i = 0;
    uint32_t m = 0;
    for (int ny = w.y0; ny <= w.y1 && needed; ny++) {
        for (int nx = w.x0; nx <= w.x1 && needed; nx++) {
            const uint32_t q = (uint32_t)ny * W + (uint32_t)nx;
            if (q == p) continue;
            const int sim = (int)((mask[(m >> 5) * 256u] >> (m & 31u)) & 1u);
            m++;
            if (sim != cls) continue;
            const bool keep = take_all || (uint64_t)uniform_index(draw(ps, (uint32_t)i), (uint32_t)(len - i)) < needed;
            if (keep) { nbr[(size_t)(1u + n) * npx + p] = q; n++; needed--; }
            i++;
        }
    }
    return n;
}

// generateResampleIndicesGrid (neighbour_selection.cpp:107-122): nbr[0][p] = neighbourhood size, nbr[1 + i][p] = its
// i-th pixel (the pixel itself first).  indicesRandom (:24-43) / indicesSimilarity (:45-105) with the reference's
// size arithmetic (Dissimilar: `k - similar.size()` as size_t; EqualSimilarDissimilar in uint32_t).
extern "C" __global__ __launch_bounds__(256) void k_mis_neighbours(SceneDev s, uint32_t W, uint32_t H, FeaturesDev f,
                                                                  uint32_t key_s, uint32_t key_d,
                                                                  const float4* __restrict__ n_t,
                                                                  const float4* __restrict__ p_mat,
                                                                  uint32_t* __restrict__ nbr) {
    __shared__ uint32_t s_mask[kMisMaskWords * 256u];
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= W * H) return;
    const size_t npx = (size_t)W * H;
    const int x = (int)(p % W), y = (int)(p / W), rc = (int)f.R;
    const uint32_t k = f.K;
    const uint32_t ps_s = pix_state(key_s, p), ps_d = pix_state(key_d, p);
    const MisWin w = {max(x - rc, 0), max(y - rc, 0), min(x + rc, (int)W - 1), min(y + rc, (int)H - 1)};
    nbr[npx + p] = p;
    uint32_t n = 1;
    if (f.strategy == RESTIR_NEIGHBOURS_RANDOM) {
        for (uint32_t c = 0; c < k; c++) {
            const uint32_t nx = (uint32_t)w.x0 + uniform_index(draw(ps_s, 2u * c), (uint32_t)(w.x1 - w.x0 + 1));
            const uint32_t ny = (uint32_t)w.y0 + uniform_index(draw(ps_s, 2u * c + 1u), (uint32_t)(w.y1 - w.y0 + 1));
            nbr[(size_t)(1u + n) * npx + p] = ny * W + nx;
            n++;
        }
    } else {
        const float4 cn = n_t[p];
        const uint32_t cg = geom_id_of(s, p_mat[p]);
        uint32_t* mask = s_mask + threadIdx.x;
        const bool use_mask = (uint32_t)((w.x1 - w.x0 + 1) * (w.y1 - w.y0 + 1)) - 1u <= kMisMaskBits;
        uint64_t S = 0, D = 0;
        uint32_t m = 0, word = 0;
        for (int ny = w.y0; ny <= w.y1; ny++)
            for (int nx = w.x0; nx <= w.x1; nx++) {
                const uint32_t q = (uint32_t)ny * W + (uint32_t)nx;
                if (q == p) continue;
                const bool sim = are_similar(s, f, cn, cg, n_t[q], p_mat[q]);
                if (sim) S++; else D++;
                if (use_mask) {
                    word |= (uint32_t)sim << (m & 31u);
                    if ((m & 31u) == 31u) { mask[(m >> 5) * 256u] = word; word = 0; }
                }
                m++;
            }
        if (use_mask && (m & 31u)) mask[(m >> 5) * 256u] = word;
        // emit one class: from the stored bits, or by re-evaluating areSimilar for windows past kMisMaskBits
        auto emit = [&](int cls, uint64_t len, uint64_t want, bool take_all, uint32_t ps, uint32_t n0) {
            return use_mask ? mis_emit_class_mask(mask, W, w, p, cls, len, want, take_all, ps, nbr, npx, n0)
                            : mis_emit_class(s, f, n_t, p_mat, W, w, p, cn, cg, cls, len, want, take_all, ps, nbr, npx, n0);
        };
        if (f.strategy == RESTIR_NEIGHBOURS_SIMILAR) {
            if (S < k) {
                n = emit(1, S, 0, true, ps_s, n);
                n = emit(0, D, (uint64_t)k - S, false, ps_d, n);
            } else {
                n = emit(1, S, k, false, ps_s, n);
            }
        } else if (f.strategy == RESTIR_NEIGHBOURS_DISSIMILAR) {
            if (D < k) {
                n = emit(0, D, 0, true, ps_d, n);
                n = emit(1, S, (uint64_t)k - S, false, ps_s, n);
            } else {
                n = emit(0, D, k, false, ps_d, n);
            }
        } else {   // EqualSimilarDissimilar (uint32_t arithmetic as written, neighbour_selection.cpp:87-95)
            uint32_t sS = min((k / 2u) + 1u, (uint32_t)S);
            const uint32_t desired = k - sS;
            if ((uint64_t)desired > D) sS = (uint32_t)((uint64_t)sS + ((uint64_t)k - D - sS));
            n = emit(1, S, sS, false, ps_s, n);
            n = emit(0, D, (uint32_t)(k - sS), false, ps_d, n);
        }
    }
    nbr[p] = n;
}

// One R-MIS iteration (render.cpp:76-112): acc[3][pixels] += the pixel's estimate over its neighbourhood.
template <bool LDS_BVH>
__device__ __forceinline__ void rmis_body(const SceneDev& s, uint32_t W, uint32_t H, const FeaturesDev& f, v3 origin,
                                          const float4* __restrict__ n_t, const float4* __restrict__ p_mat,
                                          const uint32_t* __restrict__ nbr, const float4* __restrict__ ra,
                                          const float4* __restrict__ rb, float* __restrict__ acc) {
    const Bvh bvh = LDS_BVH ? stage_bvh(s, g_lds) : global_bvh(s);
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= W * H) return;
    const size_t npx = (size_t)W * H;
    const uint32_t N = f.N;
    const Px cur = make_px(s, n_t[p], p_mat[p], origin, p);
    const uint32_t c = nbr[p];
    v3 fc = mk(0.0f, 0.0f, 0.0f);
    for (uint32_t i = 0; i < c; i++) {
        const uint32_t q = nbr[(size_t)(1u + i) * npx + p];
        for (uint32_t j = 0; j < N; j++) {
            const float4 a = ra[(size_t)j * npx + q], b = rb[(size_t)j * npx + q];
            const v3 pos = xyz(a), col = xyz(b);
            float misWeight;
            if (f.mis_weight == RESTIR_MIS_EQUAL) {
                misWeight = 1.0f / (float)c;
            } else {   // generalisedBalanceHeuristic (render_utils.cpp:179-187)
                const float numerator = target_pdf(s, f, cur, pos, col);
                float denominator = ROMIS_FLT_MIN;
                for (uint32_t i2 = 0; i2 < c; i2++) {
                    const uint32_t q2 = nbr[(size_t)(1u + i2) * npx + p];
                    denominator += target_pdf(s, f, make_px(s, n_t[q2], p_mat[q2], origin, q2), pos, col);
                }
                misWeight = numerator / denominator;
            }
            v3 sc = visible(bvh, cur.P, pos) ? shade(s, f, cur, pos, col) : mk(0.0f, 0.0f, 0.0f);
            const v3 t = vscale(vscale(sc, misWeight), a.w);   // misWeight * sampleColor * outputWeight
            fc = vadd(fc, mk(t.x / (float)N, t.y / (float)N, t.z / (float)N));
        }
    }
    acc[p] += fc.x;
    acc[npx + p] += fc.y;
    acc[2 * npx + p] += fc.z;
}

extern "C" __global__ __launch_bounds__(256) void k_rmis_accum(SceneDev s, uint32_t W, uint32_t H, FeaturesDev f, float ox,
                                                              float oy, float oz, const float4* n_t, const float4* p_mat,
                                                              const uint32_t* nbr, const float4* ra, const float4* rb,
                                                              float* acc) {
    rmis_body<false>(s, W, H, f, mk(ox, oy, oz), n_t, p_mat, nbr, ra, rb, acc);
}
extern "C" __global__ __launch_bounds__(256) void k_rmis_accum_lds(SceneDev s, uint32_t W, uint32_t H, FeaturesDev f,
                                                                  float ox, float oy, float oz, const float4* n_t,
                                                                  const float4* p_mat, const uint32_t* nbr,
                                                                  const float4* ra, const float4* rb, float* acc) {
    rmis_body<true>(s, W, H, f, mk(ox, oy, oz), n_t, p_mat, nbr, ra, rb, acc);
}

// ---- Eigen 3 CompleteOrthogonalDecomposition<MatrixXf>::solve (render_utils.h:52) ---------------------------
// ColPivHouseholderQR::computeInPlace (ColPivHouseholderQR.h:482-571), CompleteOrthogonalDecomposition::
// computeInPlace / _solve_impl / applyZAdjointOnTheLeftInPlace (CompleteOrthogonalDecomposition.h:430-560),
// makeHouseholder / applyHouseholderOnTheLeft / OnTheRight (Householder.h), HouseholderSequence::applyThisOnTheLeft
// (HouseholderSequence.h:369-412) and the one-panel upper back substitution, with Eigen's SIMD reduction orders
// (bit-exact with the reference's Eigen on tests/golden/cod_fixtures.json); correctly rounded sqrt / division.
// Eigen's reductions with SSE2 Packet4f arithmetic (the reference's x86-64 build; no FMA), as oracle/restir_oracle.c
// restates them: redux = DenseBase::redux with alignedStart 0 (first packet loaded, a second for 8+ elements, then
// the tail; n < 4 in order), gemv = one row of the row-major general_matrix_vector_product (a zeroed packet over
// the 4-blocks, then the tail); predux(p) = (p0 + p2) + (p1 + p3).
__device__ __forceinline__ float cod_dot_redux(const float* a, const float* b, int n) {
    if (n < 4) {
        float r = a[0] * b[0];
        for (int i = 1; i < n; i++) r = r + a[i] * b[i];
        return r;
    }
    float p[4], q[4];
    const int full = n / 4 * 4, end2 = n / 8 * 8;
    for (int l = 0; l < 4; l++) p[l] = a[l] * b[l];
    if (full > 4) {
        for (int l = 0; l < 4; l++) q[l] = a[4 + l] * b[4 + l];
        for (int i = 8; i < end2; i += 8)
            for (int l = 0; l < 4; l++) {
                p[l] = p[l] + a[i + l] * b[i + l];
                q[l] = q[l] + a[i + 4 + l] * b[i + 4 + l];
            }
        for (int l = 0; l < 4; l++) p[l] = p[l] + q[l];
        if (full > end2)
            for (int l = 0; l < 4; l++) p[l] = p[l] + a[end2 + l] * b[end2 + l];
    }
    float r = (p[0] + p[2]) + (p[1] + p[3]);
    for (int i = full; i < n; i++) r = r + a[i] * b[i];
    return r;
}
__device__ __forceinline__ float cod_dot_gemv(const float* a, const float* b, int n) {
    float c[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    int j = 0;
    for (; j + 4 <= n; j += 4)
        for (int l = 0; l < 4; l++) c[l] = c[l] + a[j + l] * b[j + l];
    float r = (c[0] + c[2]) + (c[1] + c[3]);
    for (; j < n; j++) r = r + a[j] * b[j];
    return r;
}
// squaredNorm: vectorised over a contiguous segment, in index order over a strided row
__device__ __forceinline__ float cod_sqnorm(const float* v, int n, int stride) {
    if (stride == 1) return cod_dot_redux(v, v, n);
    float s = v[0] * v[0];
    for (int i = 1; i < n; i++) s = s + v[i * stride] * v[i * stride];
    return s;
}
__device__ __forceinline__ void cod_make_householder(float* v, int m, int stride, float& tau, float& beta) {
    const float tailSqNorm = m == 1 ? 0.0f : cod_sqnorm(v + stride, m - 1, stride);
    const float c0 = v[0];
    if (tailSqNorm <= ROMIS_FLT_MIN) {
        tau = 0.0f;
        beta = c0;
        for (int i = 1; i < m; i++) v[i * stride] = 0.0f;
    } else {
        float b = sqrtf(c0 * c0 + tailSqNorm);
        if (c0 >= 0.0f) b = -b;
        for (int i = 1; i < m; i++) v[i * stride] = v[i * stride] / (c0 - b);
        tau = (b - c0) / b;
        beta = b;
    }
}
// tmp = essential^* bottom: a row-major GEMV in the QR sweep (COD_HH_GEMV), an inner product when applying Q^* to
// the right-hand side (COD_HH_DOT), in index order for Z^*'s strided essential rows (COD_HH_SEQ)
enum { COD_HH_GEMV = 0, COD_HH_DOT = 1, COD_HH_SEQ = 2 };
__device__ __forceinline__ void cod_householder_left(float* M, int ld, int r0, int c0, int m, int nc, const float* e,
                                                     int estride, float tau, int kind) {
    if (m == 1) {
        for (int j = 0; j < nc; j++) M[r0 + (c0 + j) * ld] *= 1.0f - tau;
        return;
    }
    if (tau == 0.0f) return;
    for (int j = 0; j < nc; j++) {
        float* col = &M[(c0 + j) * ld + r0];
        float t;
        if (kind == COD_HH_GEMV) {
            t = cod_dot_gemv(e, col + 1, m - 1);
        } else if (kind == COD_HH_DOT) {
            t = cod_dot_redux(e, col + 1, m - 1);
        } else {
            t = e[0] * col[1];
            for (int i = 1; i < m - 1; i++) t = t + e[i * estride] * col[1 + i];
        }
        t += col[0];
        col[0] -= tau * t;
        for (int i = 0; i < m - 1; i++) col[1 + i] -= (tau * e[i * estride]) * t;
    }
}
// tmp = right * essential: a column-major GEMV, each row summed in index order onto a zeroed accumulator
__device__ __forceinline__ void cod_householder_right(float* M, int ld, int r0, int c0, int nr, int m, const float* e,
                                                      int estride, float tau) {
    if (m == 1) {
        for (int i = 0; i < nr; i++) M[r0 + i + c0 * ld] *= 1.0f - tau;
        return;
    }
    if (tau == 0.0f) return;
    for (int i = 0; i < nr; i++) {
        float t = 0.0f;
        for (int j = 0; j < m - 1; j++) t = t + M[r0 + i + (c0 + 1 + j) * ld] * e[j * estride];
        t += M[r0 + i + c0 * ld];
        M[r0 + i + c0 * ld] -= tau * t;
        for (int j = 0; j < m - 1; j++) M[r0 + i + (c0 + 1 + j) * ld] -= (tau * t) * e[j * estride];
    }
}

// x = the minimum-norm least-squares solution of A x = b; A column-major NN x NN (copied), NN <= 8
template <int NN>
__device__ void cod_solve_dev(const float* A, const float* b, float* x) {
    constexpr int n = NN;
    float qr[NN * NN], hc[NN], zc[NN], nU[NN], nD[NN], c[NN], y[NN];
    int tr[NN], perm[NN];
    for (int i = 0; i < n * n; i++) qr[i] = A[i];
    for (int k = 0; k < n; k++) { nD[k] = sqrtf(cod_sqnorm(&qr[k * n], n, 1)); nU[k] = nD[k]; }
    float mx = nU[0];
    for (int k = 1; k < n; k++) if (nU[k] > mx) mx = nU[k];
    const float eps = 1.1920928955078125e-07F;
    const float threshold_helper = (mx * eps) * (mx * eps) / (float)n;
    const float norm_downdate_threshold = sqrtf(eps);
    int nonzero = n;
    float maxpivot = 0.0f;
    for (int k = 0; k < n; k++) {
        int bi = k;
        float bv = nU[k];
        for (int j = k + 1; j < n; j++) if (nU[j] > bv) { bv = nU[j]; bi = j; }
        if (nonzero == n && bv * bv < threshold_helper * (float)(n - k)) nonzero = k;
        tr[k] = bi;
        if (k != bi) {
            for (int i = 0; i < n; i++) { const float t = qr[i + k * n]; qr[i + k * n] = qr[i + bi * n]; qr[i + bi * n] = t; }
            float t = nU[k]; nU[k] = nU[bi]; nU[bi] = t;
            t = nD[k]; nD[k] = nD[bi]; nD[bi] = t;
        }
        float beta;
        cod_make_householder(&qr[k + k * n], n - k, 1, hc[k], beta);
        qr[k + k * n] = beta;
        if (fabsf(beta) > maxpivot) maxpivot = fabsf(beta);
        cod_householder_left(qr, n, k, k + 1, n - k, n - k - 1, &qr[k + 1 + k * n], 1, hc[k], COD_HH_GEMV);
        for (int j = k + 1; j < n; j++) {
            if (nU[j] != 0.0f) {
                float temp = fabsf(qr[k + j * n]) / nU[j];
                temp = (1.0f + temp) * (1.0f - temp);
                temp = temp < 0.0f ? 0.0f : temp;
                const float ratio = nU[j] / nD[j];
                const float temp2 = temp * (ratio * ratio);
                if (temp2 <= norm_downdate_threshold) {
                    nD[j] = sqrtf(cod_sqnorm(&qr[k + 1 + j * n], n - k - 1, 1));
                    nU[j] = nD[j];
                } else {
                    nU[j] *= sqrtf(temp);
                }
            }
        }
    }
    for (int k = 0; k < n; k++) perm[k] = k;
    for (int k = 0; k < n; k++) { const int t = perm[k]; perm[k] = perm[tr[k]]; perm[tr[k]] = t; }
    const float pre = fabsf(maxpivot) * (eps * (float)n);
    int rank = 0;
    for (int i = 0; i < nonzero; i++) rank += fabsf(qr[i + i * n]) > pre;
    if (rank < n) {
        for (int k = rank - 1; k >= 0; k--) {
            if (k != rank - 1)
                for (int i = 0; i <= k; i++) { const float t = qr[i + k * n]; qr[i + k * n] = qr[i + (rank - 1) * n]; qr[i + (rank - 1) * n] = t; }
            float beta;
            cod_make_householder(&qr[k + (rank - 1) * n], n - rank + 1, n, zc[k], beta);
            qr[k + (rank - 1) * n] = beta;
            if (k > 0) cod_householder_right(qr, n, 0, rank - 1, k, n - rank + 1, &qr[k + rank * n], n, zc[k]);
            if (k != rank - 1)
                for (int i = 0; i <= k; i++) { const float t = qr[i + k * n]; qr[i + k * n] = qr[i + (rank - 1) * n]; qr[i + (rank - 1) * n] = t; }
        }
    }
    {   // _solve_impl's rank(), over the decomposition's diagonal
        int r2 = 0;
        for (int i = 0; i < nonzero; i++) r2 += fabsf(qr[i + i * n]) > pre;
        rank = r2;
    }
    if (rank == 0) { for (int i = 0; i < n; i++) x[i] = 0.0f; return; }
    for (int i = 0; i < n; i++) c[i] = b[i];
    for (int k = 0; k < rank; k++) cod_householder_left(c, n, k, 0, n - k, 1, &qr[k + 1 + k * n], 1, hc[k], COD_HH_DOT);
    for (int i = 0; i < n; i++) y[i] = i < rank ? c[i] : 0.0f;
    for (int i = rank - 1; i >= 0; i--) {
        if (y[i] != 0.0f) {
            y[i] /= qr[i + i * n];
            for (int j = 0; j < i; j++) y[j] -= y[i] * qr[j + i * n];
        }
    }
    if (rank < n) {
        for (int k = 0; k < rank; k++) {
            if (k != rank - 1) { const float t = y[k]; y[k] = y[rank - 1]; y[rank - 1] = t; }
            cod_householder_left(y, n, rank - 1, 0, n - rank + 1, 1, &qr[k + rank * n], n, zc[k], COD_HH_SEQ);
            if (k != rank - 1) { const float t = y[k]; y[k] = y[rank - 1]; y[rank - 1] = t; }
        }
    }
    for (int i = 0; i < n; i++) x[perm[i]] = y[i];
}

// arbitraryUnbiasedContributionWeightReciprocal (render_utils.cpp:245-257)
__device__ __forceinline__ float aucw_reciprocal(const SceneDev& s, const FeaturesDev& f, const Px& qpx, float M,
                                                 float wsum, float chosen, v3 pos, v3 col) {
    const float targetPdfValue = target_pdf(s, f, qpx, pos, col);
    if (targetPdfValue == 0.0f) return 0.0f;
    const float mockSampleWeight = targetPdfValue / (1.0f / (float)s.num_lights);
    const float arbitraryWeight = ((1.0f / targetPdfValue) * (1.0f / M)) * ((wsum - chosen) + mockSampleWeight);
    return 1.0f / arbitraryWeight;
}

// One R-OMIS iteration (render.cpp:139-231), split in two launches per chunk of the pixel's T x N samples (the
// one-lane-per-pixel form held A, b and every sample's per-distribution state at once: 251-260 VGPRs = 1-2 waves per
// SIMD, its loads a dependent chain per distribution; 24-44 % VALU busy):
//  - k_romis_samples_t{T}: one lane per (sample, pixel), wave = 64 pixels of one sample slot: the sample's column
//    vector over the T distributions (arbitraryUnbiasedContributionWeightReciprocal at each distribution pixel) and
//    its visibility-tested shaded colour -> smp rows [sample][T + 3][pixels];
//  - k_romis_accum_t{T}[_prog]: one lane per pixel: the progressive colour, scale factor, technique matrix and
//    contribution vector updates of those samples, in the reference's order, reading them back from smp.
// Every value is computed by the same operations as in one pass, so the split is bit-exact.
template <int T, bool LDS_BVH>
__device__ __forceinline__ void romis_samples_body(const SceneDev& s, uint32_t W, uint32_t H, const FeaturesDev& f,
                                                   v3 origin, const float4* __restrict__ n_t,
                                                   const float4* __restrict__ p_mat, const uint32_t* __restrict__ nbr,
                                                   const float4* __restrict__ ra, const float4* __restrict__ rb,
                                                   const float2* __restrict__ rdbg, uint32_t s0, uint32_t ns,
                                                   float* __restrict__ smp) {
    const Bvh bvh = LDS_BVH ? stage_bvh(s, g_lds) : global_bvh(s);
    const uint32_t npx = W * H;   // launcher: ns * npx < 2^31
    const uint32_t N = f.N;
    const uint32_t items = ns * npx;
    for (uint32_t it = blockIdx.x * blockDim.x + threadIdx.x; it < items; it += gridDim.x * blockDim.x) {
        const uint32_t sl = it / npx, p = it - sl * npx;
        const uint32_t sg = s0 + sl, pi = sg / N, si = sg - pi * N;
        const uint32_t q = nbr[(size_t)(1u + pi) * npx + p];
        const float4 a = ra[(size_t)si * npx + q], b4 = rb[(size_t)si * npx + q];
        const v3 pos = xyz(a), col = xyz(b4);
        float* out = smp + (size_t)sl * (T + 3) * npx + p;
        // the T target-pdf evaluations as one rolled loop (one inlined copy of target_pdf)
#pragma unroll 1
        for (int d = 0; d < T; d++) {
            const uint32_t qq = nbr[(size_t)(1 + d) * npx + p];
            const float4 db = rb[(size_t)si * npx + qq];
            const float2 dd = rdbg[(size_t)si * npx + qq];
            out[(size_t)d * npx] = aucw_reciprocal(s, f, make_px(s, n_t[qq], p_mat[qq], origin, qq),
                                                   (float)__float_as_uint(db.w), dd.x, dd.y, pos, col);
        }
        const Px cur = make_px(s, n_t[p], p_mat[p], origin, p);
        const v3 sc = visible(bvh, cur.P, pos) ? shade(s, f, cur, pos, col) : mk(0.0f, 0.0f, 0.0f);
        out[(size_t)T * npx] = sc.x;
        out[(size_t)(T + 1) * npx] = sc.y;
        out[(size_t)(T + 2) * npx] = sc.z;
    }
}

template <int T, bool PROG>
__device__ __forceinline__ void romis_accum_body(uint32_t W, uint32_t H, const FeaturesDev& f, uint32_t s0, uint32_t ns,
                                                 const float* __restrict__ smp, float* __restrict__ acc) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= W * H) return;
    const size_t npx = (size_t)W * H;
    const uint32_t N = f.N;
    const int32_t totalSamples = (int32_t)((uint32_t)T * N);
    const int32_t fractionOfTotalSamples = (int32_t)N / (int32_t)T;
    float* Am = acc;
    float* Bv = acc + (size_t)T * T * npx;
    const float* Al = Bv + (size_t)3 * T * npx;
    float* Col = Bv + (size_t)6 * T * npx;
    float A[T * T], bb[3][T], al[3][T];
#pragma unroll
    for (int e = 0; e < T * T; e++) A[e] = Am[(size_t)e * npx + p];
#pragma unroll
    for (int ch = 0; ch < 3; ch++)
#pragma unroll
        for (int i = 0; i < T; i++) {
            bb[ch][i] = Bv[(size_t)(ch * T + i) * npx + p];
            if (PROG) al[ch][i] = Al[(size_t)(ch * T + i) * npx + p];
        }
    v3 fc = mk(0.0f, 0.0f, 0.0f);
    if (PROG) fc = mk(Col[p], Col[npx + p], Col[2 * npx + p]);
    for (uint32_t sl = 0; sl < ns; sl++) {
        const uint32_t sg = s0 + sl, pi = sg / N, si = sg - pi * N;
        if (PROG && si == 0u)   // the start of neighbourhood entry pi (render.cpp:156-160)
            fc = vadd(fc, mk(Al[(size_t)pi * npx + p], Al[(size_t)(T + pi) * npx + p], Al[(size_t)(2 * T + pi) * npx + p]));
        const float* in = smp + (size_t)sl * (T + 3) * npx + p;
        float v[T];
#pragma unroll
        for (int d = 0; d < T; d++) v[d] = in[(size_t)d * npx];
        const v3 sc = mk(in[(size_t)T * npx], in[(size_t)(T + 1) * npx], in[(size_t)(T + 2) * npx]);
        if (PROG) {
            v3 sa = mk(0.0f, 0.0f, 0.0f);
            float sf = ROMIS_FLT_MIN;
#pragma unroll
            for (int d = 0; d < T; d++) {
                sa = vadd(sa, vscale(mk(al[0][d], al[1][d], al[2][d]), v[d]));
                sf += (float)fractionOfTotalSamples * v[d];
            }
            const v3 term = vsub(mk(sc.x / sf, sc.y / sf, sc.z / sf), mk(sa.x / sf, sa.y / sf, sa.z / sf));
            const float inv = 1.0f / (float)totalSamples;
            fc = vadd(fc, mk(inv * term.x, inv * term.y, inv * term.z));
        }
        float scaleFactor = ROMIS_FLT_MIN;
#pragma unroll
        for (int d = 0; d < T; d++) scaleFactor += (float)N * v[d];
        scaleFactor = 1.0f / scaleFactor;
#pragma unroll
        for (int d = 0; d < T; d++) v[d] *= scaleFactor;
#pragma unroll
        for (int j = 0; j < T; j++)
#pragma unroll
            for (int i = 0; i < T; i++) A[i + j * T] += v[i] * v[j];
#pragma unroll
        for (int row = 0; row < T; row++) {
            const float scaleColVecConst = scaleFactor * v[row];
            bb[0][row] += sc.x * scaleColVecConst;
            bb[1][row] += sc.y * scaleColVecConst;
            bb[2][row] += sc.z * scaleColVecConst;
        }
    }
#pragma unroll
    for (int e = 0; e < T * T; e++) Am[(size_t)e * npx + p] = A[e];
#pragma unroll
    for (int ch = 0; ch < 3; ch++)
#pragma unroll
        for (int i = 0; i < T; i++) Bv[(size_t)(ch * T + i) * npx + p] = bb[ch][i];
    if (PROG) { Col[p] = fc.x; Col[npx + p] = fc.y; Col[2 * npx + p] = fc.z; }
}

// Progressive R-OMIS (render.cpp:148-152): at the start of iteration i >= 1 with i % progressiveUpdateMod == 0, each
// colour's alpha vector = the least-squares solution over the technique matrix and contribution vector so far.
template <int T>
__device__ __forceinline__ void romis_alphas_body(uint32_t W, uint32_t H, float* __restrict__ acc) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= W * H) return;
    const size_t npx = (size_t)W * H;
    float A[T * T], bv[T], xv[T];
    for (int e = 0; e < T * T; e++) A[e] = acc[(size_t)e * npx + p];
    for (int ch = 0; ch < 3; ch++) {
        for (int i = 0; i < T; i++) bv[i] = acc[(size_t)(T * T + ch * T + i) * npx + p];
        cod_solve_dev<T>(A, bv, xv);
        for (int i = 0; i < T; i++) acc[(size_t)(T * T + 3 * T + ch * T + i) * npx + p] = xv[i];
    }
}

// saveAlphasVisualisation (render.cpp:227-229, visualiseAlphas render_utils.cpp:189-243): after an iteration, each
// colour's alpha vector solved from the sums so far (the sums themselves untouched; progressive alphas live in their
// own rows).  Technique i, colour ch -> image 3 i + ch; a pixel is glm::mix(0, (1, .5, 0), a) for a > 0 and
// glm::mix(0, (0, .5, 1), -a) otherwise (x (1 - a) + y a, unfused), stored as Screen::writeBitmapToFile's 8-bit word
// (clamp to [0, 1], x255, truncate; bytes B, G, R, A = 255).  A bitmap's rows run bottom-up, and Screen::setPixel
// flips y, so image pixel order = this grid's order (y = 0 bottom): out[(3 i + ch) npx + p].
__device__ __forceinline__ uint32_t vis_u8(float v) {
    const float m = (v < 0.0f) ? 0.0f : v;   // glm::clamp: a NaN passes through ...
    const float c = (1.0f < m) ? 1.0f : m;
    if (c != c) return 0u;                   // ... and truncates to 0 (screen.cpp's to_u8)
    return (uint32_t)(int)__fmul_rn(c, 255.0f);
}
__device__ __forceinline__ float vis_mix(float y, float a) {
    return __fadd_rn(__fmul_rn(0.0f, __fsub_rn(1.0f, a)), __fmul_rn(y, a));
}
template <int T>
__device__ __forceinline__ void romis_vis_body(uint32_t W, uint32_t H, const float* __restrict__ acc,
                                               uint32_t* __restrict__ out) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= W * H) return;
    const size_t npx = (size_t)W * H;
    float A[T * T], bv[T], xv[T];
    for (int e = 0; e < T * T; e++) A[e] = acc[(size_t)e * npx + p];
    for (int ch = 0; ch < 3; ch++) {
        for (int i = 0; i < T; i++) bv[i] = acc[(size_t)(T * T + ch * T + i) * npx + p];
        cod_solve_dev<T>(A, bv, xv);
        for (int i = 0; i < T; i++) {
            const float a = xv[i];
            const bool pos = a > 0.0f;
            const float m = pos ? a : -a;
            const float r = vis_mix(pos ? 1.0f : 0.0f, m), g = vis_mix(0.5f, m), b = vis_mix(pos ? 0.0f : 1.0f, m);
            out[(size_t)(3 * i + ch) * npx + p] = vis_u8(b) | (vis_u8(g) << 8) | (vis_u8(r) << 16) | 0xFF000000u;
        }
    }
}

#define ROMIS_ROMIS_SAMPLES(T, LDS, NAME)                                                                           \
    extern "C" __global__ __launch_bounds__(256) void NAME(SceneDev s, uint32_t W, uint32_t H, FeaturesDev f, float ox,  \
                                                          float oy, float oz, const float4* n_t, const float4* p_mat,  \
                                                          const uint32_t* nbr, const float4* ra, const float4* rb,      \
                                                          const float2* rdbg, uint32_t s0, uint32_t ns, float* smp) {   \
        romis_samples_body<T, LDS>(s, W, H, f, mk(ox, oy, oz), n_t, p_mat, nbr, ra, rb, rdbg, s0, ns, smp);             \
    }
#define ROMIS_ROMIS_ACCUM(T, PROG, NAME)                                                                             \
    extern "C" __global__ __launch_bounds__(256) void NAME(uint32_t W, uint32_t H, FeaturesDev f, uint32_t s0,           \
                                                          uint32_t ns, const float* smp, float* acc) {                 \
        romis_accum_body<T, PROG>(W, H, f, s0, ns, smp, acc);                                                          \
    }
#define ROMIS_ROMIS_KERNELS(T)                                                                                        \
    ROMIS_ROMIS_SAMPLES(T, false, k_romis_samples_t##T)                                                               \
    ROMIS_ROMIS_SAMPLES(T, true, k_romis_samples_lds_t##T)                                                            \
    ROMIS_ROMIS_ACCUM(T, false, k_romis_accum_t##T)                                                                   \
    ROMIS_ROMIS_ACCUM(T, true, k_romis_accum_prog_t##T)                                                               \
    extern "C" __global__ __launch_bounds__(256) void k_romis_alphas_t##T(uint32_t W, uint32_t H, float* acc) {         \
        romis_alphas_body<T>(W, H, acc);                                                                              \
    }                                                                                                                 \
    extern "C" __global__ __launch_bounds__(256) void k_romis_vis_t##T(uint32_t W, uint32_t H, const float* acc,        \
                                                                      uint32_t* out) {                                \
        romis_vis_body<T>(W, H, acc, out);                                                                            \
    }                                                                                                                 \
    extern "C" __global__ __launch_bounds__(256) void k_romis_solve_t##T(uint32_t W, uint32_t H, FeaturesDev f,         \
                                                                        const float* acc, float* rgb) {               \
        romis_solve_body<T>(W, H, f, acc, rgb);                                                                        \
    }                                                                                                                 \
    extern "C" __global__ __launch_bounds__(256) void k_debug_cod_t##T(const float* A, const float* b, float* x,        \
                                                                      uint32_t count) {                               \
        const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;                                                     \
        if (i >= count) return;                                                                                       \
        float a[T * T], bv[T], xv[T];                                                                                 \
        for (int e = 0; e < T * T; e++) a[e] = A[(size_t)i * T * T + e];                                              \
        for (int e = 0; e < T; e++) bv[e] = b[(size_t)i * T + e];                                                     \
        cod_solve_dev<T>(a, bv, xv);                                                                                  \
        for (int e = 0; e < T; e++) x[(size_t)i * T + e] = xv[e];                                                     \
    }

// Direct R-OMIS screen (render.cpp:234-263): three solves per pixel, component sums, tone map, Screen y-flip.
template <int T>
__device__ __forceinline__ void romis_solve_body(uint32_t W, uint32_t H, const FeaturesDev& f, const float* __restrict__ acc,
                                                 float* __restrict__ rgb) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= W * H) return;
    const size_t npx = (size_t)W * H;
    float A[T * T], bv[T], xs[3][T];
    for (int e = 0; e < T * T; e++) A[e] = acc[(size_t)e * npx + p];
    for (int ch = 0; ch < 3; ch++) {
        for (int i = 0; i < T; i++) bv[i] = acc[(size_t)(T * T + ch * T + i) * npx + p];
        cod_solve_dev<T>(A, bv, xs[ch]);
    }
    v3 c = mk(0.0f, 0.0f, 0.0f);
    for (int row = 0; row < T; row++) { c.x += xs[0][row]; c.y += xs[1][row]; c.z += xs[2][row]; }
    if (f.tone_map) {
        const float g = 1.0f / f.gamma;
        v3 e = vscale(mk(-c.x, -c.y, -c.z), f.exposure);
        v3 mapped = mk(1.0f - pm_expf(e.x), 1.0f - pm_expf(e.y), 1.0f - pm_expf(e.z));
        c = mk(pm_powf(mapped.x, g), pm_powf(mapped.y, g), pm_powf(mapped.z, g));
    }
    const uint32_t x = p % W, y = p / W;
    float* o = rgb + 3 * ((size_t)(H - 1u - y) * W + x);
    o[0] = c.x; o[1] = c.y; o[2] = c.z;
}

ROMIS_ROMIS_KERNELS(1)
ROMIS_ROMIS_KERNELS(2)
ROMIS_ROMIS_KERNELS(3)
ROMIS_ROMIS_KERNELS(4)
ROMIS_ROMIS_KERNELS(5)
ROMIS_ROMIS_KERNELS(6)
ROMIS_ROMIS_KERNELS(7)
ROMIS_ROMIS_KERNELS(8)

// combineToScreen (render_utils.cpp:68-85): R-MIS and progressive R-OMIS colour sums / iterations, tone map, y-flip.
extern "C" __global__ __launch_bounds__(256) void k_mis_combine(uint32_t W, uint32_t H, FeaturesDev f, const float* col,
                                                               float* rgb) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= W * H) return;
    const size_t npx = (size_t)W * H;
    const float it = (float)f.iterations;
    v3 c = mk(col[p] / it, col[npx + p] / it, col[2 * npx + p] / it);
    if (f.tone_map) {
        const float g = 1.0f / f.gamma;
        v3 e = vscale(mk(-c.x, -c.y, -c.z), f.exposure);
        v3 mapped = mk(1.0f - pm_expf(e.x), 1.0f - pm_expf(e.y), 1.0f - pm_expf(e.z));
        c = mk(pm_powf(mapped.x, g), pm_powf(mapped.y, g), pm_powf(mapped.z, g));
    }
    const uint32_t x = p % W, y = p / W;
    float* o = rgb + 3 * ((size_t)(H - 1u - y) * W + x);
    o[0] = c.x; o[1] = c.y; o[2] = c.z;
}

// ---------------------------------------------------------------------------------------------------------
// Host launchers (launch.h)
#include "launch.h"
#include "launch_events.h"

namespace romis {

// ---- R-MIS / R-OMIS ---------------------------------------------------------------------------------------
namespace {
typedef void (*RomisSamplesFn)(SceneDev, uint32_t, uint32_t, FeaturesDev, float, float, float, const float4*, const float4*,
                               const uint32_t*, const float4*, const float4*, const float2*, uint32_t, uint32_t, float*);
typedef void (*RomisAccumFn)(uint32_t, uint32_t, FeaturesDev, uint32_t, uint32_t, const float*, float*);
typedef void (*RomisAlphasFn)(uint32_t, uint32_t, float*);
typedef void (*RomisSolveFn)(uint32_t, uint32_t, FeaturesDev, const float*, float*);
typedef void (*RomisVisFn)(uint32_t, uint32_t, const float*, uint32_t*);
typedef void (*DebugCodFn)(const float*, const float*, float*, uint32_t);
#define ROMIS_T_TABLE(PFX) {PFX##1, PFX##2, PFX##3, PFX##4, PFX##5, PFX##6, PFX##7, PFX##8}
const RomisSamplesFn kRomisSamples[8] = ROMIS_T_TABLE(k_romis_samples_t);
const RomisSamplesFn kRomisSamplesLds[8] = ROMIS_T_TABLE(k_romis_samples_lds_t);
const RomisAccumFn kRomisAccum[8] = ROMIS_T_TABLE(k_romis_accum_t);
const RomisAccumFn kRomisAccumProg[8] = ROMIS_T_TABLE(k_romis_accum_prog_t);
const RomisAlphasFn kRomisAlphas[8] = ROMIS_T_TABLE(k_romis_alphas_t);
const RomisSolveFn kRomisSolve[8] = ROMIS_T_TABLE(k_romis_solve_t);
const RomisVisFn kRomisVis[8] = ROMIS_T_TABLE(k_romis_vis_t);
const DebugCodFn kDebugCod[8] = ROMIS_T_TABLE(k_debug_cod_t);
inline dim3 px_grid(size_t npx) { return dim3((uint32_t)((npx + kBlock - 1) / kBlock)); }
}  // namespace

hipError_t launch_mis_neighbours(const SceneDev& s, uint32_t W, uint32_t H, const FeaturesDev& f, uint32_t key_s, uint32_t key_d,
                                 const float4* n_t, const float4* p_mat, uint32_t* nbr, hipStream_t stream) {
    ROMIS_LAUNCH(k_mis_neighbours, px_grid((size_t)W * H), dim3(kBlock), 0, stream, s, W, H, f, key_s, key_d, n_t, p_mat, nbr);
    return hipGetLastError();
}

hipError_t launch_mis_accumulate(const SceneDev& s, uint32_t W, uint32_t H, const FeaturesDev& f, const float* o,
                                 const float4* n_t, const float4* p_mat, const uint32_t* nbr, const float4* ra,
                                 const float4* rb, const float2* rdbg, uint32_t iteration, float* acc, float* smp,
                                 uint32_t smp_samples, const Tuning& tu, hipStream_t stream) {
    const size_t lds = bvh_lds_bytes(s);
    const bool use_lds = tu.final_lds && lds <= kLdsBudget;   // shadow rays: the BVH staged like k_final's
    const dim3 grid = px_grid((size_t)W * H);
    if (f.mode == RESTIR_MODE_RMIS) {
        ROMIS_LAUNCH(use_lds ? k_rmis_accum_lds : k_rmis_accum, grid, dim3(kBlock), use_lds ? lds : 0, stream, s, W, H, f,
                     o[0], o[1], o[2], n_t, p_mat, nbr, ra, rb, acc);
    } else {
        const uint32_t T = f.K + 1u;
        if (T < 1u || T > 8u) return hipErrorInvalidValue;
        if (f.progressive && iteration >= 1u && iteration % f.prog_mod == 0u)   // alphas from the sums so far
            ROMIS_LAUNCH(kRomisAlphas[T - 1], grid, dim3(kBlock), 0, stream, W, H, acc);
        // the T x N samples in chunks of smp_samples (the scratch rows ensure_mis sized), in the reference's order
        const RomisSamplesFn ks = use_lds ? kRomisSamplesLds[T - 1] : kRomisSamples[T - 1];
        const RomisAccumFn ka = f.progressive ? kRomisAccumProg[T - 1] : kRomisAccum[T - 1];
        const uint32_t npx = W * H, S = T * f.N;
        if (smp_samples == 0u || (uint64_t)smp_samples * npx >= (1ull << 31)) return hipErrorInvalidValue;
        for (uint32_t s0 = 0; s0 < S; s0 += smp_samples) {
            const uint32_t ns = std::min(smp_samples, S - s0);
            const uint32_t blocks = std::min<uint32_t>((ns * npx + kBlock - 1u) / kBlock, 8192u);
            ROMIS_LAUNCH(ks, dim3(blocks), dim3(kBlock), use_lds ? lds : 0, stream, s, W, H, f, o[0], o[1], o[2], n_t,
                         p_mat, nbr, ra, rb, rdbg, s0, ns, smp);
            ROMIS_LAUNCH(ka, grid, dim3(kBlock), 0, stream, W, H, f, s0, ns, smp, acc);
        }
    }
    return hipGetLastError();
}

hipError_t launch_mis_finish(uint32_t W, uint32_t H, const FeaturesDev& f, const float* acc, float* rgb, hipStream_t stream) {
    const dim3 grid = px_grid((size_t)W * H);
    const uint32_t T = f.K + 1u;
    if (f.mode == RESTIR_MODE_ROMIS && !f.progressive) {
        if (T < 1u || T > 8u) return hipErrorInvalidValue;
        ROMIS_LAUNCH(kRomisSolve[T - 1], grid, dim3(kBlock), 0, stream, W, H, f, acc, rgb);
    } else {
        const float* col = f.mode == RESTIR_MODE_ROMIS ? acc + (size_t)(T * T + 6u * T) * W * H : acc;
        ROMIS_LAUNCH(k_mis_combine, grid, dim3(kBlock), 0, stream, W, H, f, col, rgb);
    }
    return hipGetLastError();
}

hipError_t launch_romis_vis(uint32_t W, uint32_t H, uint32_t T, const float* acc, uint32_t* out, hipStream_t stream) {
    if (T < 1u || T > 8u) return hipErrorInvalidValue;
    ROMIS_LAUNCH(kRomisVis[T - 1], px_grid((size_t)W * H), dim3(kBlock), 0, stream, W, H, acc, out);
    return hipGetLastError();
}

hipError_t launch_debug_cod(uint32_t n, const float* A, const float* b, float* x, uint32_t count, hipStream_t stream) {
    if (count == 0) return hipSuccess;
    if (n < 1u || n > 8u) return hipErrorInvalidValue;
    hipLaunchKernelGGL(kDebugCod[n - 1], px_grid(count), dim3(kBlock), 0, stream, A, b, x, count);
    return hipGetLastError();
}

}  // namespace romis


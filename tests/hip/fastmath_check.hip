// fastmath_check.hip -- GPU check that the exact fast forms in romis_amd/csrc/device_math.h equal the IEEE
// operations bit for bit: sqrt_rn_core and rcp_rn_core on EVERY float inside their guards, div_by_rcp_d on
// 2^32 hashed operand pairs plus edge cases.  Built by romis_amd/build.py; run by tests/test_gpu_fastmath.py.
// Prints one JSON line; exit status 0 iff no mismatch.
#include "device_math.h"

#include <cstdio>
#include <cstdlib>

using namespace romis;

struct Counters {
    unsigned long long checked[3];
    unsigned long long bad[3];
    unsigned int first[3][2];
};

__global__ void k_unary(unsigned long long base, Counters* c) {
    const unsigned long long i = base + blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    if (i > 0xFFFFFFFFull) return;
    const float x = __uint_as_float((uint32_t)i);
    unsigned int ns = 0, bs = 0, nr = 0, br = 0;
    if (sqrt_fast_ok(x)) {
        ns = 1;
        if (__float_as_uint(sqrt_rn_core(x)) != __float_as_uint(sqrtf(x))) { bs = 1; c->first[0][0] = (uint32_t)i; }
    }
    if (rcp_fast_ok(x)) {
        nr = 1;
        if (__float_as_uint(rcp_rn_core(x)) != __float_as_uint(1.0f / x)) { br = 1; c->first[1][0] = (uint32_t)i; }
    }
    // wave-aggregated counts
    unsigned long long m;
    m = __ballot(ns); if (threadIdx.x % 64 == 0 && m) atomicAdd(&c->checked[0], (unsigned long long)__popcll(m));
    m = __ballot(bs); if (threadIdx.x % 64 == 0 && m) atomicAdd(&c->bad[0], (unsigned long long)__popcll(m));
    m = __ballot(nr); if (threadIdx.x % 64 == 0 && m) atomicAdd(&c->checked[1], (unsigned long long)__popcll(m));
    m = __ballot(br); if (threadIdx.x % 64 == 0 && m) atomicAdd(&c->bad[1], (unsigned long long)__popcll(m));
}

__device__ __forceinline__ float pick(uint32_t h, uint32_t mode) {
    // mode 0: any finite float; 1: moderate magnitudes [2^-40, 2^40]; 2: mantissa-adversarial (all-ones / near
    // powers of two significands)
    uint32_t sign = h & 0x80000000u;
    uint32_t e, m = (h >> 1) & 0x7FFFFFu;
    uint32_t h2 = mix32(h);
    if (mode == 0) e = h2 % 254u + 1u;
    else if (mode == 1) e = 127u - 40u + h2 % 81u;
    else { e = 127u - 20u + h2 % 41u; m = (h2 & 64u) ? (0x7FFFFFu ^ (h2 & 0xFu)) : (h2 & 0xFu); }
    return __uint_as_float(sign | (e << 23) | m);
}

__global__ void k_div(unsigned long long base, Counters* c) {
    const unsigned long long i = base + blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    const uint32_t h = mix32((uint32_t)i ^ 0x2545F491u) ^ (uint32_t)(i >> 32);
    const uint32_t mode = (uint32_t)(i % 3u);
    const float a = pick(mix32(h + 1u), mode), b = pick(mix32(h + 2u), mode);
    unsigned int n = 0, bad = 0;
    if (div_fast_ok(b)) {
        n = 1;
        const float q = div_by_rcp_d(a, rcp_d(b));
        if (__float_as_uint(q) != __float_as_uint(a / b)) {
            bad = 1; c->first[2][0] = __float_as_uint(a); c->first[2][1] = __float_as_uint(b);
        }
    }
    unsigned long long m;
    m = __ballot(n); if (threadIdx.x % 64 == 0 && m) atomicAdd(&c->checked[2], (unsigned long long)__popcll(m));
    m = __ballot(bad); if (threadIdx.x % 64 == 0 && m) atomicAdd(&c->bad[2], (unsigned long long)__popcll(m));
}

// edge operands for the division: exact quotients, denominators at the guard, subnormal / overflowing results
__global__ void k_div_edges(Counters* c) {
    const float as[] = {0.0f, -0.0f, 1.0f, 3.0f, 1e-38f, 1.5e-45f, 3.4e38f, -7.0f, 0x1.fffffep0f, 0x1p-126f,
                        __builtin_inff(), 6.0f, 1e30f, 0x1.000002p0f, __uint_as_float(0x7FC00000u),
                        __uint_as_float(0xFFC12345u), __uint_as_float(0x7FA00001u), -__builtin_inff()};
    const float bs[] = {1.0f, 3.0f, 0x1p-120f, 0x1p120f, 0x1.fffffep0f, 7.0f, 1e-30f, -2.0f, 0x1.000002p0f, 1e20f,
                        1e-20f, 0x1.8p0f};
    const int t = threadIdx.x;
    const int na = sizeof(as) / sizeof(as[0]), nb = sizeof(bs) / sizeof(bs[0]);
    if (t >= na * nb) return;
    const float a = as[t / nb], b = bs[t % nb];
    const float q = div_by_rcp_d(a, rcp_d(b)), r = a / b;
    if (t == 0) {   // sqrt_rn_core(+0) == +0: target_pdf takes the core form for q == 0 as well
        atomicAdd(&c->checked[0], 1ull);
        if (__float_as_uint(sqrt_rn_core(0.0f)) != 0u) atomicAdd(&c->bad[0], 1ull);
    }
    atomicAdd(&c->checked[2], 1ull);
    if (__float_as_uint(q) != __float_as_uint(r)) {
        atomicAdd(&c->bad[2], 1ull); c->first[2][0] = __float_as_uint(a); c->first[2][1] = __float_as_uint(b);
    }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 3; } } while (0)

int main(int argc, char** argv) {
    const unsigned long long div_pairs = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : (1ull << 32);
    Counters* d = nullptr;
    CK(hipMalloc(&d, sizeof(Counters)));
    CK(hipMemset(d, 0, sizeof(Counters)));
    const unsigned long long chunk = 1ull << 28;
    for (unsigned long long b = 0; b < (1ull << 32); b += chunk)
        hipLaunchKernelGGL(k_unary, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, b, d);
    for (unsigned long long b = 0; b < div_pairs; b += chunk)
        hipLaunchKernelGGL(k_div, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, b, d);
    hipLaunchKernelGGL(k_div_edges, dim3(1), dim3(256), 0, 0, d);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    Counters h;
    CK(hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost));
    CK(hipFree(d));
    std::printf("{\"sqrt\": {\"checked\": %llu, \"bad\": %llu, \"first_bad\": %u}, "
                "\"rcp\": {\"checked\": %llu, \"bad\": %llu, \"first_bad\": %u}, "
                "\"div\": {\"checked\": %llu, \"bad\": %llu, \"first_bad\": [%u, %u]}}\n",
                h.checked[0], h.bad[0], h.first[0][0], h.checked[1], h.bad[1], h.first[1][0], h.checked[2], h.bad[2],
                h.first[2][0], h.first[2][1]);
    return (h.bad[0] || h.bad[1] || h.bad[2]) ? 1 : 0;
}

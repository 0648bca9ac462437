// rcpd_probe.hip -- relative error of v_rcp_f64 and of one / two Newton steps over every float b in
// div_fast_ok's range (|b| in [2^-120, 2^120]): max |1 - b y| (fma residual, exact for y near 1/b).
// Decides whether rcp_d (device_math.h) can drop its second Newton step (needs <= 2^-50).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k(unsigned long long base, unsigned long long* mx) {
    const unsigned long long i = base + blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    if (i > 0xFFFFFFFFull) return;
    const float b = __uint_as_float((uint32_t)i);
    const float ab = fabsf(b);
    const double d = (ab >= 0x1p-120f && ab <= 0x1p120f) ? (double)b : 1.0;   // outside: a harmless 1
    const double y0 = __builtin_amdgcn_rcp(d);
    const double e0 = fabs(__builtin_fma(-d, y0, 1.0));
    const double y1 = __builtin_fma(__builtin_fma(-d, y0, 1.0), y0, y0);
    const double e1 = fabs(__builtin_fma(-d, y1, 1.0));
    const double y2 = __builtin_fma(__builtin_fma(-d, y1, 1.0), y1, y1);
    const double e2 = fabs(__builtin_fma(-d, y2, 1.0));
    unsigned long long v[3] = {(unsigned long long)__double_as_longlong(e0), (unsigned long long)__double_as_longlong(e1),
                               (unsigned long long)__double_as_longlong(e2)};
    for (int j = 0; j < 3; j++) {   // wave max (positive doubles order as their bits), one atomic per wave
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned long long w = __shfl_xor(v[j], o);
            v[j] = w > v[j] ? w : v[j];
        }
        if ((threadIdx.x & 63u) == 0u && v[j] > __atomic_load_n(&mx[j], __ATOMIC_RELAXED)) atomicMax(&mx[j], v[j]);
    }
}

int main() {
    unsigned long long* d = nullptr;
    if (hipMalloc(&d, 24) != hipSuccess) return 3;
    (void)hipMemset(d, 0, 24);
    const unsigned long long chunk = 1ull << 28;
    for (unsigned long long b = 0; b < (1ull << 32); b += chunk)
        hipLaunchKernelGGL(k, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, b, d);
    if (hipDeviceSynchronize() != hipSuccess) return 4;
    unsigned long long h[3];
    (void)hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
    double e[3];
    for (int j = 0; j < 3; j++) { union { unsigned long long u; double f; } c; c.u = h[j]; e[j] = c.f; }
    std::printf("{\"max_e0\": %.6e, \"max_e1\": %.6e, \"max_e2\": %.6e, \"log2\": [%.3f, %.3f, %.3f]}\n", e[0], e[1], e[2],
                __builtin_log2(e[0]), __builtin_log2(e[1]), __builtin_log2(e[2]));
    return 0;
}

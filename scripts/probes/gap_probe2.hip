// gap_probe2.hip -- the idle time between dependent kernels on one stream as a function of what the kernels store.
// The frame's kernels (RIS, spatial, final) show 6-8 us between one kernel's end and the next one's start in rocprof
// traces (profiles/r4/gap), while back-to-back VALU spin kernels show none (gap_probe.hip).  Here three kernels per
// iteration each (a) spin, (b) store 64 MiB with plain 16-byte stores, (c) store 64 MiB with nontemporal stores, or
// (d) read 64 MiB; run under `rocprofv3 --kernel-trace` and compare the start(k+1) - end(k) gaps per variant.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void spin(float* out, int iters) {
    float x = (float)threadIdx.x;
    for (int i = 0; i < iters; i++) x = __builtin_fmaf(x, 0.999f, 0.5f);
    if (x == -1.0f) out[blockIdx.x] = x;
}
__global__ void store_plain(float4* buf, size_t n4, float v) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        buf[i] = make_float4(v, v, v, v);
}
__global__ void store_nt(float4* buf, size_t n4, float v) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        float* p = reinterpret_cast<float*>(buf + i);
        __builtin_nontemporal_store(v, p);
        __builtin_nontemporal_store(v, p + 1);
        __builtin_nontemporal_store(v, p + 2);
        __builtin_nontemporal_store(v, p + 3);
    }
}
__global__ void load_sum(const float4* buf, size_t n4, float* out) {
    float acc = 0.0f;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = buf[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == -1.0f) out[blockIdx.x] = acc;
}

#define CK(e) do { hipError_t r_ = (e); if (r_ != hipSuccess) { std::printf("%s: %s\n", #e, hipGetErrorString(r_)); return 1; } } while (0)

int main() {
    const size_t bytes = 64ull << 20, n4 = bytes / 16;
    float4 *a, *b, *c;
    float* o;
    CK(hipMalloc(&a, bytes)); CK(hipMalloc(&b, bytes)); CK(hipMalloc(&c, bytes)); CK(hipMalloc(&o, 1 << 20));
    CK(hipMemset(a, 0, bytes)); CK(hipMemset(b, 0, bytes)); CK(hipMemset(c, 0, bytes));
    hipStream_t s; CK(hipStreamCreate(&s));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int reps = 30;
    const char* names[4] = {"spin", "store_plain", "store_nt", "load"};
    for (int v = 0; v < 4; v++) {
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < reps; r++) {
            float4* bufs[3] = {a, b, c};
            for (int k = 0; k < 3; k++) {
                if (v == 0) hipLaunchKernelGGL(spin, dim3(2048), dim3(256), 0, s, o, 3000);
                if (v == 1) hipLaunchKernelGGL(store_plain, dim3(4096), dim3(256), 0, s, bufs[k], n4, (float)r);
                if (v == 2) hipLaunchKernelGGL(store_nt, dim3(4096), dim3(256), 0, s, bufs[k], n4, (float)r);
                if (v == 3) hipLaunchKernelGGL(load_sum, dim3(4096), dim3(256), 0, s, bufs[k], n4, o);
            }
        }
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("{\"variant\": \"%s\", \"us_per_kernel\": %.2f}\n", names[v], 1000.0 * ms / (3 * reps));
    }
    return 0;
}

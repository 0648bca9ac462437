// gap_probe.hip -- the idle time between dependent kernels on one stream: three back-to-back kernels of a fixed
// length (a VALU spin of ~40 us each, 2048 blocks), launched plainly vs replayed from a captured hipGraph.
// Prints us per iteration for both and the implied per-kernel gap against the kernels' own (event-timed) length.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void spin(float* out, int iters) {
    float x = (float)threadIdx.x;
    for (int i = 0; i < iters; i++) x = __builtin_fmaf(x, 0.999f, 0.5f);
    if (x == -1.0f) out[blockIdx.x] = x;   // never true; keeps the loop
}

#define CK(e) do { hipError_t r_ = (e); if (r_ != hipSuccess) { std::printf("%s: %s\n", #e, hipGetErrorString(r_)); return 1; } } while (0)

int main() {
    float* d; CK(hipMalloc(&d, 4096 * 4));
    hipStream_t s; CK(hipStreamCreate(&s));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const int iters = 4000, reps = 200;
    // one kernel alone
    for (int w = 0; w < 5; w++) hipLaunchKernelGGL(spin, dim3(2048), dim3(256), 0, s, d, iters);
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(spin, dim3(2048), dim3(256), 0, s, d, iters);
    CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
    float ms1; CK(hipEventElapsedTime(&ms1, a, b));
    // plain: 3 kernels per iteration
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; r++)
        for (int k = 0; k < 3; k++) hipLaunchKernelGGL(spin, dim3(2048), dim3(256), 0, s, d, iters);
    CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
    float ms3; CK(hipEventElapsedTime(&ms3, a, b));
    // graph of the 3 kernels
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int k = 0; k < 3; k++) hipLaunchKernelGGL(spin, dim3(2048), dim3(256), 0, s, d, iters);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int w = 0; w < 5; w++) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; r++) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
    float msg; CK(hipEventElapsedTime(&msg, a, b));
    const double k1 = 1000.0 * ms1 / reps, p3 = 1000.0 * ms3 / reps, g3 = 1000.0 * msg / reps;
    std::printf("{\"kernel_us\": %.2f, \"plain3_us\": %.2f, \"graph3_us\": %.2f, \"plain_gap_us\": %.2f, \"graph_gap_us\": %.2f}\n",
                k1, p3, g3, (p3 - 3 * k1) / 3, (g3 - 3 * k1) / 3);
    return 0;
}

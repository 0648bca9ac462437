// fetch_probe.hip -- calibrates rocprofv3's FETCH_SIZE for the access shapes of the spatial pass (DESIGN.md §6,
// "Traffic").  MI355X_MICROARCH.md states FETCH_SIZE = 1/2 of the bytes of a wide coalesced streaming read and leaves
// other widths uncalibrated; the spatial pass's traffic figure doubles FETCH for all of its reads, including the
// accepted neighbours' 16-byte reservoir gathers.  Each kernel below reads a known set of 128-byte lines, once each,
// from a 2 GiB buffer (8x the 256 MiB Infinity Cache, so the lines come from HBM):
//   stream    : 16 B per lane, coalesced (the calibration the guide gives: FETCH = 1/2 of the bytes)
//   g16       : one 16-byte gather per lane at the start of a distinct, randomly placed 128-byte line
//   g32       : two lanes read 32 consecutive bytes of one line (a res_a + res_b pair is two such gathers)
//   g64       : four lanes read the first 64 bytes of one line
//   g128      : eight lanes read the whole line
// The line permutation is multiplicative (odd constant mod 2^24 lines), so no line is read twice.  Run once under
// `rocprofv3 --pmc FETCH_SIZE` and once under `--kernel-trace --stats`; bytes per line = FETCH_SIZE / lines.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr uint64_t kLines = 1ull << 24;          // 2 GiB of 128-byte lines
constexpr uint32_t kGathered = 1u << 21;         // lines touched per gather kernel (256 MiB of lines, 1/8 of them)

__device__ __forceinline__ uint64_t line_of(uint32_t i) { return ((uint64_t)i * 0x9E3779B1ull) & (kLines - 1); }

__global__ void k_stream(const float4* __restrict__ buf, uint64_t n4, float* out) {
    float acc = 0.0f;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x) {
        const float4 v = buf[i];   // plain loads, as the spatial pass issues
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == -1.0f) out[blockIdx.x] = acc;   // never true (the buffer holds zeros); keeps the loads
}

template <uint32_t LANES>   // lanes per line: 1 (16 B), 2 (32 B), 4 (64 B), 8 (128 B)
__global__ void k_gather(const float4* __restrict__ buf, uint32_t set, float* out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t i = t / LANES, part = t % LANES;
    if (i >= kGathered) return;
    const float4 v = buf[line_of(set * kGathered + i) * 8u + part];   // line sets are disjoint
    const float acc = v.x + v.y + v.z + v.w;
    if (acc == -1.0f) out[t & 1023u] = acc;
}

#define CK(e) do { hipError_t r_ = (e); if (r_ != hipSuccess) { std::printf("%s: %s\n", #e, hipGetErrorString(r_)); return 1; } } while (0)

template <uint32_t L>
static int run_gather(const char* name, uint32_t set, const float4* buf, float* out, hipStream_t s, hipEvent_t a,
                      hipEvent_t b) {
    const uint32_t threads = kGathered * L, grid = (threads + 255u) / 256u;
    hipLaunchKernelGGL(k_gather<L>, dim3(grid), dim3(256), 0, s, buf, set, out);   // untimed warm-up, its own lines
    CK(hipEventRecord(a, s));
    hipLaunchKernelGGL(k_gather<L>, dim3(grid), dim3(256), 0, s, buf, set + 1u, out);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    std::printf("{\"kernel\": \"%s\", \"lines\": %u, \"bytes_read_by_lanes\": %llu, \"us\": %.2f}\n", name, kGathered,
                (unsigned long long)kGathered * 16ull * L, ms * 1e3);
    return 0;
}

int main() {
    float4* buf; float* out;
    CK(hipMalloc(&buf, kLines * 128ull));
    CK(hipMemset(buf, 0, kLines * 128ull));
    CK(hipMalloc(&out, 4096 * sizeof(float)));
    hipStream_t s; CK(hipStreamCreate(&s));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipDeviceSynchronize());
    // the gathers first (8 disjoint sets of 2^21 lines: warm-up and timed launch per kernel), then stream 1 GiB twice
    if (run_gather<1>("g16", 0, buf, out, s, a, b) || run_gather<2>("g32", 2, buf, out, s, a, b) ||
        run_gather<4>("g64", 4, buf, out, s, a, b) || run_gather<8>("g128", 6, buf, out, s, a, b))
        return 1;
    const uint64_t n4 = (kLines * 128ull / 2ull) / 16ull;
    hipLaunchKernelGGL(k_stream, dim3(2048), dim3(256), 0, s, buf, n4, out);
    CK(hipEventRecord(a, s));
    hipLaunchKernelGGL(k_stream, dim3(2048), dim3(256), 0, s, buf + n4, n4, out);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    std::printf("{\"kernel\": \"stream\", \"bytes\": %llu, \"us\": %.2f}\n", (unsigned long long)(n4 * 16ull), ms * 1e3);
    CK(hipFree(buf)); CK(hipFree(out));
    return 0;
}

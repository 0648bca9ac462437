// valu_rates.hip -- issue-rate microbenchmark of the VALU instructions the ReSTIR kernels are made of.
// Each kernel runs ITERS x 8 independent instances of one instruction per lane (8 dependency chains), with
// 8 waves per SIMD (2048 threads per CU), so the measured time is the pipe's throughput, not latency.
// Prints cycles per wave-instruction per SIMD, calibrated against s_memtime (shader clock ticks).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 2048

#define BODY8(INS) \
    asm volatile(INS : "+v"(a0) : "v"(b) : "s0", "s1", "vcc"); asm volatile(INS : "+v"(a1) : "v"(b) : "s0", "s1", "vcc"); \
    asm volatile(INS : "+v"(a2) : "v"(b) : "s0", "s1", "vcc"); asm volatile(INS : "+v"(a3) : "v"(b) : "s0", "s1", "vcc"); \
    asm volatile(INS : "+v"(a4) : "v"(b) : "s0", "s1", "vcc"); asm volatile(INS : "+v"(a5) : "v"(b) : "s0", "s1", "vcc"); \
    asm volatile(INS : "+v"(a6) : "v"(b) : "s0", "s1", "vcc"); asm volatile(INS : "+v"(a7) : "v"(b) : "s0", "s1", "vcc");

#define KERNEL32(NAME, INS)                                                                         \
    __global__ __launch_bounds__(256) void NAME(float* out, uint64_t* clk, float seed) {           \
        float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
              a6 = a0 + 6, a7 = a0 + 7, b = seed * 0.5f + 1.0f;                                    \
        uint64_t t0 = __builtin_amdgcn_s_memtime();                                                 \
        for (int i = 0; i < ITERS; i++) { BODY8(INS) }                                              \
        uint64_t t1 = __builtin_amdgcn_s_memtime();                                                 \
        if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;                                            \
        out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;               \
    }

#define BODY8D(INS) \
    asm volatile(INS : "+v"(a0) : "v"(b) : "s0", "s1", "vcc"); asm volatile(INS : "+v"(a1) : "v"(b) : "s0", "s1", "vcc"); \
    asm volatile(INS : "+v"(a2) : "v"(b) : "s0", "s1", "vcc"); asm volatile(INS : "+v"(a3) : "v"(b) : "s0", "s1", "vcc"); \
    asm volatile(INS : "+v"(a4) : "v"(b) : "s0", "s1", "vcc"); asm volatile(INS : "+v"(a5) : "v"(b) : "s0", "s1", "vcc"); \
    asm volatile(INS : "+v"(a6) : "v"(b) : "s0", "s1", "vcc"); asm volatile(INS : "+v"(a7) : "v"(b) : "s0", "s1", "vcc");

#define KERNEL64(NAME, INS)                                                                         \
    __global__ __launch_bounds__(256) void NAME(float* out, uint64_t* clk, float seed) {           \
        double a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
               a6 = a0 + 6, a7 = a0 + 7, b = seed * 0.5 + 1.0;                                     \
        uint64_t t0 = __builtin_amdgcn_s_memtime();                                                 \
        for (int i = 0; i < ITERS; i++) { BODY8D(INS) }                                             \
        uint64_t t1 = __builtin_amdgcn_s_memtime();                                                 \
        if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;                                            \
        out[blockIdx.x * 256 + threadIdx.x] = (float)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);      \
    }

KERNEL32(k_add_f32, "v_add_f32 %0, %0, %1")
KERNEL32(k_fma_f32, "v_fma_f32 %0, %0, %1, %1")
KERNEL32(k_sqrt_f32, "v_sqrt_f32 %0, %0")
KERNEL32(k_rcp_f32, "v_rcp_f32 %0, %0")
KERNEL32(k_mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
KERNEL32(k_mul_hi_u32, "v_mul_hi_u32 %0, %0, %1")
KERNEL32(k_xor_b32, "v_xor_b32 %0, %0, %1")
KERNEL32(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
KERNEL32(k_cmp_f32, "v_cmp_lt_f32 vcc, %0, %1")
KERNEL32(k_div_scale, "v_div_scale_f32 %0, vcc, %0, %1, %0")
KERNEL32(k_div_fixup, "v_div_fixup_f32 %0, %0, %1, %0")
KERNEL32(k_cvt_f32_u32, "v_cvt_f32_u32 %0, %0")
KERNEL32(k_max3_f32, "v_max3_f32 %0, %0, %1, %1")
KERNEL32(k_mov_b32, "v_mov_b32 %0, %1")
KERNEL32(k_readlane, "v_readlane_b32 s0, %0, 3\n v_add_f32 %0, s0, %1")
KERNEL64(k_mul_f64, "v_mul_f64 %0, %0, %1")
KERNEL64(k_fma_f64, "v_fma_f64 %0, %0, %1, %1")
KERNEL64(k_rcp_f64, "v_rcp_f64 %0, %0")
KERNEL64(k_pk_fma_f32, "v_pk_fma_f32 %0, %0, %1, %1")
KERNEL64(k_pk_add_f32, "v_pk_add_f32 %0, %0, %1")
KERNEL64(k_lshl_add_u64, "v_lshl_add_u64 %0, %0, 4, %1")
KERNEL64(k_mov_b64, "v_mov_b64 %0, %1")

// 64-bit accumulators with a 32-bit source operand
#define BODY8M(INS) \
    asm volatile(INS : "+v"(a0) : "v"(b) : "s0", "s1", "vcc"); asm volatile(INS : "+v"(a1) : "v"(b) : "s0", "s1", "vcc"); \
    asm volatile(INS : "+v"(a2) : "v"(b) : "s0", "s1", "vcc"); asm volatile(INS : "+v"(a3) : "v"(b) : "s0", "s1", "vcc"); \
    asm volatile(INS : "+v"(a4) : "v"(b) : "s0", "s1", "vcc"); asm volatile(INS : "+v"(a5) : "v"(b) : "s0", "s1", "vcc"); \
    asm volatile(INS : "+v"(a6) : "v"(b) : "s0", "s1", "vcc"); asm volatile(INS : "+v"(a7) : "v"(b) : "s0", "s1", "vcc");
#define KERNEL6432(NAME, INS)                                                                       \
    __global__ __launch_bounds__(256) void NAME(float* out, uint64_t* clk, float seed) {           \
        double a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
               a6 = a0 + 6, a7 = a0 + 7;                                                             \
        float b = seed * 0.5f + 1.0f;                                                               \
        uint64_t t0 = __builtin_amdgcn_s_memtime();                                                 \
        for (int i = 0; i < ITERS; i++) { BODY8M(INS) }                                             \
        uint64_t t1 = __builtin_amdgcn_s_memtime();                                                 \
        if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;                                            \
        out[blockIdx.x * 256 + threadIdx.x] = (float)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);      \
    }
KERNEL6432(k_mad_u64_u32, "v_mad_u64_u32 %0, s[0:1], %1, %1, %0")
KERNEL6432(k_cvt_f64_f32, "v_cvt_f64_f32 %0, %1")
KERNEL32(k_cvt_f32_f64, "v_cvt_f32_f64 %0, v[0:1]")

KERNEL32(k_mul_f32, "v_mul_f32 %0, %0, %1")
KERNEL32(k_sub_f32, "v_sub_f32 %0, %0, %1")
KERNEL32(k_fmac_f32, "v_fmac_f32 %0, %1, %1")
KERNEL32(k_and_b32, "v_and_b32 %0, %0, %1")
KERNEL32(k_lshrrev_b32, "v_lshrrev_b32 %0, 13, %0")
KERNEL32(k_add_u32, "v_add_u32 %0, %0, %1")
KERNEL32(k_min_i32, "v_min_i32 %0, %0, %1")
KERNEL32(k_mul_u32_u24, "v_mul_u32_u24 %0, %0, %1")
KERNEL32(k_bfi_b32, "v_bfi_b32 %0, %0, %1, %1")
KERNEL32(k_cmp_class, "v_cmp_class_f32 vcc, %0, %1")
KERNEL32(k_cmp_cnd, "v_cmp_lt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc")
KERNEL32(k_cnd_e64, "v_cndmask_b32_e64 %0, %0, %1, s[0:1]")
KERNEL32(k_cmp_e64_cnd, "v_cmp_lt_f32_e64 s[0:1], %0, %1\n v_cndmask_b32_e64 %0, %0, %1, s[0:1]")
KERNEL32(k_xor_sdwa, "v_xor_b32_sdwa %0, %0, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD")
KERNEL32(k_readfirstlane, "v_readfirstlane_b32 s0, %0\n v_add_f32 %0, s0, %1")
KERNEL64(k_pk_mul_f32, "v_pk_mul_f32 %0, %0, %1")
KERNEL64(k_add_f64, "v_add_f64 %0, %0, %1")
// latency: one dependency chain per wave (ILP 1), 8 waves per SIMD
#define KERNEL32L(NAME, INS)                                                                        \
    __global__ __launch_bounds__(256) void NAME(float* out, uint64_t* clk, float seed) {           \
        float a0 = seed + threadIdx.x, b = seed * 0.5f + 1.0f;                                      \
        uint64_t t0 = __builtin_amdgcn_s_memtime();                                                 \
        for (int i = 0; i < ITERS * 8; i++) { asm volatile(INS : "+v"(a0) : "v"(b) : "s0", "s1", "vcc"); } \
        uint64_t t1 = __builtin_amdgcn_s_memtime();                                                 \
        if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;                                            \
        out[blockIdx.x * 256 + threadIdx.x] = a0;                                                   \
    }
KERNEL32L(kl_add_f32, "v_add_f32 %0, %0, %1")
KERNEL32L(kl_fma_f32, "v_fma_f32 %0, %0, %1, %1")
KERNEL32L(kl_sqrt_f32, "v_sqrt_f32 %0, %0")
KERNEL32L(kl_cmp_cnd, "v_cmp_lt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc")

typedef void (*kfn)(float*, uint64_t*, float);
struct K { const char* name; kfn f; int per_body; };

int main() {
    K ks[] = {
        {"v_add_f32", k_add_f32, 1}, {"v_fma_f32", k_fma_f32, 1}, {"v_sqrt_f32", k_sqrt_f32, 1},
        {"v_rcp_f32", k_rcp_f32, 1}, {"v_mul_lo_u32", k_mul_lo_u32, 1}, {"v_mul_hi_u32", k_mul_hi_u32, 1},
        {"v_xor_b32", k_xor_b32, 1}, {"v_cndmask_b32", k_cndmask, 1}, {"v_cmp_lt_f32(vcc)", k_cmp_f32, 1},
        {"v_div_scale_f32", k_div_scale, 1}, {"v_div_fixup_f32", k_div_fixup, 1},
        {"v_cvt_f32_u32", k_cvt_f32_u32, 1}, {"v_max3_f32", k_max3_f32, 1}, {"v_mov_b32", k_mov_b32, 1},
        {"v_readlane+v_add", k_readlane, 2},
        {"v_mul_f64", k_mul_f64, 1}, {"v_fma_f64", k_fma_f64, 1}, {"v_rcp_f64", k_rcp_f64, 1},
        {"v_pk_fma_f32", k_pk_fma_f32, 1}, {"v_pk_add_f32", k_pk_add_f32, 1},
        {"v_mad_u64_u32", k_mad_u64_u32, 1}, {"v_lshl_add_u64", k_lshl_add_u64, 1},
        {"v_mul_f32", k_mul_f32, 1}, {"v_sub_f32", k_sub_f32, 1}, {"v_fmac_f32", k_fmac_f32, 1},
        {"v_and_b32", k_and_b32, 1}, {"v_lshrrev_b32", k_lshrrev_b32, 1}, {"v_add_u32", k_add_u32, 1},
        {"v_min_i32", k_min_i32, 1}, {"v_mul_u32_u24", k_mul_u32_u24, 1}, {"v_bfi_b32", k_bfi_b32, 1},
        {"v_cmp_class_f32", k_cmp_class, 1}, {"v_cmp+v_cndmask(vcc)", k_cmp_cnd, 2},
        {"v_cndmask_e64(s01)", k_cnd_e64, 1}, {"v_cmp_e64+cndmask_e64", k_cmp_e64_cnd, 2},
        {"v_xor_b32_sdwa", k_xor_sdwa, 1}, {"v_readfirstlane+add", k_readfirstlane, 2},
        {"v_pk_mul_f32", k_pk_mul_f32, 1}, {"v_add_f64", k_add_f64, 1},
        {"LAT ILP1 v_add_f32", kl_add_f32, 1}, {"LAT ILP1 v_fma_f32", kl_fma_f32, 1},
        {"LAT ILP1 v_sqrt_f32", kl_sqrt_f32, 1}, {"LAT ILP1 cmp+cndmask", kl_cmp_cnd, 2},
        {"v_mov_b64", k_mov_b64, 1}, {"v_cvt_f64_f32", k_cvt_f64_f32, 1}, {"v_cvt_f32_f64", k_cvt_f32_f64, 1},
    };
    const int blocks = 256 * 8;   // 8 blocks of 256 per CU = 8 waves per SIMD
    float* out; uint64_t* clk;
    hipMalloc(&out, blocks * 256 * sizeof(float));
    hipMalloc(&clk, blocks * sizeof(uint64_t));
    uint64_t* h = (uint64_t*)malloc(blocks * sizeof(uint64_t));
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, clk, 1.0f);   // warm
        hipEventRecord(e0);
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, clk, 1.0f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(h, clk, blocks * sizeof(uint64_t), hipMemcpyDeviceToHost);
        double avg = 0; for (int i = 0; i < blocks; i++) avg += (double)h[i]; avg /= blocks;
        // per SIMD: 8 waves x ITERS x 8 bodies instructions; s_memtime runs at a fixed 100 MHz on gfx9? report both
        const double instr_per_simd = 8.0 * ITERS * 8 * k.per_body;
        const double ns_per = ms * 1e6 / instr_per_simd;
        printf("%-26s %8.3f ms  %7.3f ns/wave-instr/SIMD  (%5.2f cycles @2.4GHz)  memtime/block %.0f\n", k.name, ms,
               ns_per, ns_per * 2.4, avg);
    }
    return 0;
}

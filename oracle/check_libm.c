/*
 * check_libm.c -- TEST INFRASTRUCTURE: exhaustive comparison of oracle/portable_math.h with the image's libm.
 *
 *   make -C oracle check_libm && oracle/_build/check_libm [threads] [stride]
 *
 * stride > 1 checks every stride-th bit pattern (the CPU test suite's quick form); the default is exhaustive.
 *
 * powf(x, y) for every 32-bit pattern x (all 2^32 bases: cosTheta is negative for half the hemisphere, and NaN /
 * inf / subnormal patterns are included) and every exponent the path evaluates with the shipped scenes -- the
 * shininess values 1, 4, 10, 250 (computeShading, shading.cpp:26) and the tone-map exponents 1/gamma for gamma
 * 1 (the Features default, common.h:134), 2.2 and 2.4 (tone_mapping.cpp:10) -- plus expf for every 32-bit x
 * (tone_mapping.cpp:9).  Prints one JSON line per function; exit status 1 on any bit mismatch.
 */
#include "portable_math.h"

#include <omp.h>
#include <stdio.h>
#include <stdlib.h>

static int64_t g_stride = 1;

static uint64_t check_pow(float y, uint64_t* first_bad) {
    uint64_t bad = 0, first = ~0ull;
#pragma omp parallel for schedule(static, 1 << 20) reduction(+ : bad) reduction(min : first)
    for (int64_t i = 0; i < (int64_t)1 << 32; i += g_stride) {
        float x = pm_ffrom((uint32_t)i);
        volatile float yy = y;
        uint32_t want = pm_fbits(powf(x, yy));
        uint32_t got = pm_fbits(pm_powf(x, y));
        if (want != got) { bad++; if ((uint64_t)i < first) first = (uint64_t)i; }
    }
    *first_bad = first;
    return bad;
}

static uint64_t check_exp(uint64_t* first_bad) {
    uint64_t bad = 0, first = ~0ull;
#pragma omp parallel for schedule(static, 1 << 20) reduction(+ : bad) reduction(min : first)
    for (int64_t i = 0; i < (int64_t)1 << 32; i += g_stride) {
        volatile float x = pm_ffrom((uint32_t)i);
        uint32_t want = pm_fbits(expf(x));
        uint32_t got = pm_fbits(pm_expf(x));
        if (want != got) { bad++; if ((uint64_t)i < first) first = (uint64_t)i; }
    }
    *first_bad = first;
    return bad;
}

int main(int argc, char** argv) {
    if (argc > 1) omp_set_num_threads(atoi(argv[1]));
    if (argc > 2) g_stride = atoll(argv[2]);
    const unsigned long long n_inputs = (((1ull << 32) - 1) / (unsigned long long)g_stride) + 1;
    const float ys[] = {1.0f, 4.0f, 10.0f, 250.0f, 1.0f / 2.2f, 1.0f / 2.4f};
    int fail = 0;
    for (unsigned k = 0; k < sizeof(ys) / sizeof(ys[0]); k++) {
        uint64_t first;
        uint64_t bad = check_pow(ys[k], &first);
        printf("{\"fn\": \"powf\", \"y\": \"%a\", \"inputs\": %llu, \"mismatches\": %llu", (double)ys[k],
               n_inputs, (unsigned long long)bad);
        if (bad) printf(", \"first_x_bits\": \"0x%08llx\"", (unsigned long long)first);
        printf("}\n");
        fflush(stdout);
        fail |= bad != 0;
    }
    uint64_t first;
    uint64_t bad = check_exp(&first);
    printf("{\"fn\": \"expf\", \"inputs\": %llu, \"mismatches\": %llu", n_inputs, (unsigned long long)bad);
    if (bad) printf(", \"first_x_bits\": \"0x%08llx\"", (unsigned long long)first);
    printf("}\n");
    fail |= bad != 0;
    return fail;
}

// ref_rng.cpp -- TEST INFRASTRUCTURE (the CPU baseline's timing mode; never shipped, never checked for parity).
//
// The reference's own random-number machinery, driven by the oracle's arithmetic when or_set_rng_mode(1) is
// set, so that bench.py can time the CPU path the way the reference runs it:
//   - every genCanonicalSamples call (light.cpp:49-51) constructs a std::random_device, seeds a std::mt19937
//     from it and draws the light indices through a std::uniform_int_distribution<>;
//   - spatialReuse (render_utils.cpp:89-91) seeds ONE std::mt19937 per call and every OpenMP thread draws its
//     neighbour offsets from it without synchronisation (a data race); here each thread draws from its own
//     generator, seeded once per pass -- no shared state, so this side is if anything faster than the reference;
//   - every reservoir update (reservoir.cpp:24) and light-sample fraction (light.cpp:20, 28-29) calls the C
//     library's rand() (one process-wide generator behind glibc's lock), mapped by linearMap (utils.cpp:26-31).
// Results in this mode are not reproducible (that is the reference's behaviour, and why the product uses the
// keyed counter RNG instead -- DESIGN.md §3); only its speed is reported.
#include <cstdint>
#include <cstdlib>
#include <atomic>
#include <random>

namespace {
thread_local std::mt19937 t_gen;
thread_local std::mt19937 t_pass_gen;
thread_local unsigned t_pass_epoch = 0;
std::atomic<unsigned> g_pass_epoch{0};
}

extern "C" {

// per-pixel generator: std::random_device rd; std::mt19937 gen(rd());
void or_refrng_pixel_seed(void) {
    std::random_device rd;
    t_gen.seed(rd());
}

// std::uniform_int_distribution<> distr(lo, hi); distr(gen)
int or_refrng_uniform(int lo, int hi) {
    std::uniform_int_distribution<> distr(lo, hi);
    return distr(t_gen);
}

// spatialReuse's generator: a new pass (epoch) makes every thread re-seed its own generator on first use
void or_refrng_shared_seed(void) { g_pass_epoch.fetch_add(1, std::memory_order_relaxed); }

int or_refrng_shared_uniform(int lo, int hi) {
    const unsigned e = g_pass_epoch.load(std::memory_order_relaxed);
    if (t_pass_epoch != e) {
        std::random_device rd;
        t_pass_gen.seed(rd());
        t_pass_epoch = e;
    }
    std::uniform_int_distribution<> distr(lo, hi);
    return distr(t_pass_gen);
}

// linearMap(static_cast<float>(rand()), 0.0f, RAND_MAX, 0.0f, 1.0f)
float or_refrng_rand01(void) {
    const float val = static_cast<float>(rand());
    const float ratio = (val - 0.0f) / (static_cast<float>(RAND_MAX) - 0.0f);
    return ratio * (1.0f - 0.0f) + 0.0f;
}

}  // extern "C"

// screen.cpp -- host output of a rendered frame: the reference's 8-bit bitmap (Screen::writeBitmapToFile,
// screen.cpp:45-56, through stb_image_write's BMP writer) and its per-render configuration record
// (render.cpp:281-287: struct Features serialised by cereal's JSONOutputArchive).  Byte-for-byte what the
// reference writes for the same frame / features (tests/test_screen_output.py pins both against the
// reference's own stb / cereal / glm compiled from /root/reference: tests/golden/screen_fixtures.json).
#include "restir_c.h"
#include "pow10_table.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

using namespace romis;

// glm::clamp(x, 0, 1) = min(max(x, 0), 1) with glm's (y < x ? y : x) / (x < y ? y : x): a NaN passes through
inline float glm_clamp01(float x) {
    const float m = (x < 0.0f) ? 0.0f : x;
    return (1.0f < m) ? 1.0f : m;
}

// glm::u8vec4(glm::vec4(c, 1) * 255.0f): float -> uint8 conversion truncates toward zero.  The values are in
// [0, 255] after the clamp; a NaN (undefined in C++) converts as x86-64's cvttss2si does: 0x80000000, low byte 0.
inline uint8_t to_u8(float v) {
    if (std::isnan(v)) return 0;
    return static_cast<uint8_t>(static_cast<int>(v));
}

inline void put16(std::vector<uint8_t>& o, uint32_t v) { o.push_back(v & 0xFF); o.push_back((v >> 8) & 0xFF); }
inline void put32(std::vector<uint8_t>& o, uint32_t v) { put16(o, v & 0xFFFF); put16(o, v >> 16); }

// ---- doubles as the reference's JSON writer prints them ----------------------------------------------------
// cereal's JSONOutputArchive hands floats to RapidJSON's Writer::Double, which prints Grisu2 digits (Loitsch,
// PLDI 2010: shortest within the rounding boundaries shrunk by one unit of the 64-bit products -- NOT always the
// shortest round-trip string, e.g. 6.0e25f prints ...085e25 where the shortest is ...083e25) laid out by its own
// rules.  Restated here on 64-bit "do-it-yourself" floats (f * 2^e) with the cached powers of ten of
// pow10_table.h; tests/test_screen_output.py pins the bytes against the reference's own writer.
struct Fp {
    uint64_t f;
    int e;
};
inline Fp fp_mul(Fp a, Fp b) {   // 64 x 64 -> the high 64 bits, rounded half up
    const unsigned __int128 p = (unsigned __int128)a.f * b.f;
    uint64_t h = (uint64_t)(p >> 64);
    if ((uint64_t)p & (1ull << 63)) h++;
    return Fp{h, a.e + b.e + 64};
}
inline Fp fp_normalize(Fp a) {
    const int s = __builtin_clzll(a.f);
    return Fp{a.f << s, a.e - s};
}

constexpr uint64_t kHidden = 1ull << 52;

// the digits of d > 0 (finite) into buf, *len digits, value = digits * 10^*K
void grisu2(double d, char* buf, int* len, int* K) {
    uint64_t bits;
    std::memcpy(&bits, &d, 8);
    const int be = (int)((bits >> 52) & 0x7FF);
    Fp v = be ? Fp{(bits & (kHidden - 1)) + kHidden, be - 1075} : Fp{bits & (kHidden - 1), -1074};
    // boundaries m+ / m- of v's rounding interval, on m+'s normalised exponent
    Fp plus{(v.f << 1) + 1, v.e - 1};
    while (!(plus.f & (kHidden << 1))) { plus.f <<= 1; plus.e--; }
    plus.f <<= 64 - 52 - 2;
    plus.e -= 64 - 52 - 2;
    Fp minus = (v.f == kHidden) ? Fp{(v.f << 2) - 1, v.e - 2} : Fp{(v.f << 1) - 1, v.e - 1};
    minus.f <<= minus.e - plus.e;
    minus.e = plus.e;
    // a cached power c_k = 10^-K bringing the product's exponent into [-60, -32]
    const double dk = (-61 - plus.e) * 0.30102999566398114 + 347;
    int k = (int)dk;
    if (dk - k > 0.0) k++;
    const int idx = (k >> 3) + 1;
    *K = -(-348 + idx * 8);
    const Fp c{kPow10F[idx], kPow10E[idx]};
    const Fp w = fp_mul(fp_normalize(v), c);
    Fp hi = fp_mul(plus, c), lo = fp_mul(minus, c);
    lo.f++;
    hi.f--;
    // digit generation: integral part, then fractional digits, stopping inside [lo, hi]; then nudge the last digit
    // toward w while that stays inside the interval and gets closer
    static const uint32_t p10[] = {1, 10, 100, 1000, 10000, 100000, 1000000, 10000000, 100000000, 1000000000};
    const int sh = -hi.e;
    const uint64_t one = 1ull << sh;
    const uint64_t wp_w = hi.f - w.f;
    uint64_t delta = hi.f - lo.f;
    uint32_t p1 = (uint32_t)(hi.f >> sh);
    uint64_t p2 = hi.f & (one - 1);
    int kappa = 1;
    while (kappa < 9 && p1 >= p10[kappa]) kappa++;
    *len = 0;
    auto round_last = [&](uint64_t rest, uint64_t ten_kappa, uint64_t dist) {
        while (rest < dist && delta - rest >= ten_kappa && (rest + ten_kappa < dist || dist - rest > rest + ten_kappa - dist)) {
            buf[*len - 1]--;
            rest += ten_kappa;
        }
    };
    while (kappa > 0) {
        const uint32_t q = p1 / p10[kappa - 1];
        p1 %= p10[kappa - 1];
        if (q || *len) buf[(*len)++] = (char)('0' + q);
        kappa--;
        const uint64_t rest = ((uint64_t)p1 << sh) + p2;
        if (rest <= delta) {
            *K += kappa;
            round_last(rest, (uint64_t)p10[kappa] << sh, wp_w);
            return;
        }
    }
    for (;;) {
        p2 *= 10;
        delta *= 10;
        const char q = (char)(p2 >> sh);
        if (q || *len) buf[(*len)++] = (char)('0' + q);
        p2 &= one - 1;
        kappa--;
        if (p2 < delta) {
            *K += kappa;
            round_last(p2, one, wp_w * (-kappa < 9 ? p10[-kappa] : 0));
            return;
        }
    }
}

// RapidJSON's layout of digits * 10^k: integers as "5.0", decimals for 10^-6 <= |v| < 10^21, else "1.5e30" / "1e-7"
bool json_double(double d, std::string& out) {
    if (!std::isfinite(d)) return false;
    if (d == 0.0) { out += std::signbit(d) ? "-0.0" : "0.0"; return true; }
    if (d < 0) { out += '-'; d = -d; }
    char buf[32];
    int length = 0, k = 0;
    grisu2(d, buf, &length, &k);
    const std::string digits(buf, (size_t)length);
    const int kk = length + k;
    if (k >= 0 && kk <= 21) {
        out += digits;
        out.append((size_t)k, '0');
        out += ".0";
    } else if (0 < kk && kk <= 21) {
        out += digits.substr(0, (size_t)kk);
        out += '.';
        out += digits.substr((size_t)kk);
    } else if (-6 < kk && kk <= 0) {
        out += "0.";
        out.append((size_t)(-kk), '0');
        out += digits;
    } else {
        out += digits[0];
        if (length > 1) { out += '.'; out += digits.substr(1); }
        out += 'e';
        int K = kk - 1;
        if (K < 0) { out += '-'; K = -K; }
        out += std::to_string(K);
    }
    return true;
}

// stbi_write_bmp's header with 4 components: BITMAPFILEHEADER + BITMAPV4HEADER (BI_BITFIELDS, 32 bpp, alpha mask)
void bmp_header(std::vector<uint8_t>& o, uint32_t width, uint32_t height) {
    const size_t bytes = 14 + 108 + (size_t)width * height * 4;
    o.push_back('B'); o.push_back('M');
    put32(o, (uint32_t)bytes); put16(o, 0); put16(o, 0); put32(o, 14 + 108);
    put32(o, 108); put32(o, width); put32(o, height); put16(o, 1); put16(o, 32);
    put32(o, 3); put32(o, 0); put32(o, 0); put32(o, 0); put32(o, 0); put32(o, 0);
    put32(o, 0xff0000u); put32(o, 0xff00u); put32(o, 0xffu); put32(o, 0xff000000u);
    put32(o, 0);
    for (int i = 0; i < 12; i++) put32(o, 0);   // CIEXYZ endpoints (9) + gamma (3)
}

}  // namespace

namespace romis {
// A bitmap whose pixels are already stb's 32-bit words (bytes B, G, R, A) in file order, rows bottom-up
// (the R-OMIS alpha visualisation, k_romis_vis_t{T}).
bool write_bmp_words(const char* path, uint32_t width, uint32_t height, const uint32_t* words) {
    const size_t px = (size_t)width * height;
    if (!path || (!words && px) || 14 + 108 + px * 4 > 0xFFFFFFFFull) return false;
    std::vector<uint8_t> o;
    o.reserve(14 + 108);
    bmp_header(o, width, height);
    FILE* f = std::fopen(path, "wb");
    if (!f) return false;
    bool ok = std::fwrite(o.data(), 1, o.size(), f) == o.size();
    if (px) ok = std::fwrite(words, 4, px, f) == px && ok;   // little-endian words = the B, G, R, A bytes
    return std::fclose(f) == 0 && ok;
}
}  // namespace romis

extern "C" {

restir_status restir_rgb_to_rgba8(const float* rgb, size_t pixels, uint8_t* rgba) {
    if ((!rgb || !rgba) && pixels) return RESTIR_ERR_INVALID;
    for (size_t i = 0; i < pixels; i++) {
        for (int c = 0; c < 3; c++) rgba[4 * i + c] = to_u8(glm_clamp01(rgb[3 * i + c]) * 255.0f);
        rgba[4 * i + 3] = to_u8(1.0f * 255.0f);
    }
    return RESTIR_OK;
}

restir_status restir_encode_bmp(const float* rgb, uint32_t width, uint32_t height, uint8_t* out, size_t capacity,
                                size_t* length) {
    const size_t px = (size_t)width * height;
    const size_t bytes = 14 + 108 + px * 4;
    if (length) *length = bytes;
    if (!out) return RESTIR_OK;   // size query
    if ((!rgb && px) || capacity < bytes || bytes > 0xFFFFFFFFull) return RESTIR_ERR_INVALID;
    std::vector<uint8_t> rgba(px * 4);
    restir_rgb_to_rgba8(rgb, px, rgba.data());
    // stbi_write_bmp with 4 components: a BITMAPV4 header (BI_BITFIELDS, 32 bpp, alpha mask), rows bottom-up,
    // pixels B, G, R, A (stb_image_write.h stbi_write_bmp_core / stbiw__write_pixels)
    std::vector<uint8_t> o;
    o.reserve(bytes);
    bmp_header(o, width, height);
    for (uint32_t j = height; j-- > 0;) {
        const uint8_t* row = rgba.data() + (size_t)j * width * 4;
        for (uint32_t i = 0; i < width; i++) {
            const uint8_t* d = row + 4 * (size_t)i;
            o.push_back(d[2]); o.push_back(d[1]); o.push_back(d[0]); o.push_back(d[3]);
        }
    }
    std::memcpy(out, o.data(), bytes);
    return RESTIR_OK;
}

restir_status restir_write_bmp(const char* path, const float* rgb, uint32_t width, uint32_t height) {
    if (!path) return RESTIR_ERR_INVALID;
    size_t n = 0;
    restir_encode_bmp(rgb, width, height, nullptr, 0, &n);
    std::vector<uint8_t> buf(n);
    const restir_status st = restir_encode_bmp(rgb, width, height, buf.data(), n, &n);
    if (st != RESTIR_OK) return st;
    FILE* f = std::fopen(path, "wb");
    if (!f) return RESTIR_ERR_INVALID;
    const bool ok = std::fwrite(buf.data(), 1, n, f) == n;
    return (std::fclose(f) == 0 && ok) ? RESTIR_OK : RESTIR_ERR_INVALID;
}

restir_status restir_features_json(const restir_features* f, const restir_features_record_extra* extra, char* out,
                                   size_t capacity, size_t* length) {
    if (!f) return RESTIR_ERR_INVALID;
    restir_features_record_extra x{};
    if (extra) {
        x = *extra;
    } else {   // struct Features' defaults for the fields the ReSTIR path does not read (common.h:91-97)
        x.enable_recursive = 0; x.enable_hard_shadow = 1; x.enable_soft_shadow = 1; x.enable_normal_interp = 1;
        x.enable_accel_structure = 1; x.max_reflection_recursion = 5;
    }
    std::string s = "{";
    bool first = true;
    auto key = [&](const char* k) {
        s += first ? "\n    \"" : ",\n    \"";
        first = false;
        s += k;
        s += "\": ";
    };
    auto b = [&](const char* k, unsigned v) { key(k); s += v ? "true" : "false"; };
    auto u = [&](const char* k, uint32_t v) { key(k); s += std::to_string(v); };
    bool ok = true;
    auto d = [&](const char* k, float v) { key(k); ok = json_double((double)v, s) && ok; };
    // Features::serialize order (common.h:140-145)
    b("enableShading", f->enable_shading);
    b("enableRecursive", x.enable_recursive);
    b("enableHardShadow", x.enable_hard_shadow);
    b("enableSoftShadow", x.enable_soft_shadow);
    b("enableNormalInterp", x.enable_normal_interp);
    b("enableTextureMapping", f->enable_texture_mapping);
    b("enableAccelStructure", x.enable_accel_structure);
    u("maxReflectionRecursion", x.max_reflection_recursion);
    u("rayTraceMode", f->ray_trace_mode);
    b("initialSamplesVisibilityCheck", f->initial_samples_visibility_check);
    u("numSamplesInReservoir", f->num_samples_in_reservoir);
    u("initialLightSamples", f->initial_light_samples);
    u("numNeighboursToSample", f->num_neighbours_to_sample);
    u("spatialResampleRadius", f->spatial_resample_radius);
    u("maxIterationsMIS", f->max_iterations_mis);
    u("neighbourSelectionStrategy", f->neighbour_selection_strategy);
    u("misWeightRMIS", f->mis_weight_rmis);
    b("useProgressiveROMIS", f->use_progressive_romis);
    u("progressiveUpdateMod", f->progressive_update_mod);
    b("saveAlphasVisualisation", f->save_alphas_visualisation);
    b("unbiasedCombination", f->unbiased_combination);
    b("spatialReuse", f->spatial_reuse);
    b("spatialReuseVisibilityCheck", f->spatial_reuse_visibility_check);
    b("temporalReuse", f->temporal_reuse);
    u("spatialResamplingPasses", f->spatial_resampling_passes);
    u("temporalClampM", f->temporal_clamp_m);
    b("enableToneMapping", f->enable_tone_mapping);
    d("gamma", f->gamma);
    d("exposure", f->exposure);
    s += "\n}";
    if (!ok) return RESTIR_ERR_INVALID;   // cereal / RapidJSON refuse a non-finite double
    if (length) *length = s.size();
    if (!out) return RESTIR_OK;           // size query
    if (capacity < s.size() + 1) return RESTIR_ERR_INVALID;
    std::memcpy(out, s.c_str(), s.size() + 1);
    return RESTIR_OK;
}

}  // extern "C"

#!/usr/bin/env python3
"""Instruction-budget variants of the spatial pass (k_spatial1_ntl): copies of kernels.hip with one piece of the
per-pixel work replaced by a cheap stand-in that keeps its data dependences (results change; only instruction
counts and time are compared), built into romis_amd/_build/variants/<name>/libromis_amd.so.  The product source is
never modified.  Run scripts/pmc_kbench.sh / kbench_libs.sh against the variants on the GPU.

    python scripts/budget_variants.py            # builds every variant
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from romis_amd import build  # noqa: E402

SRC = os.path.join(build.CSRC, "kernels.hip")


SPANS = {   # the function each variant patches: (first line, the text that follows the function)
    "spatial": ("__device__ __forceinline__ void spatial1_ntl_body(", "#ifndef ROMIS_SPATIAL1_NTL_WPE"),
    "ris": ("__device__ __forceinline__ void ris_pixel(", "// k_ris: genCanonicalSamples per pixel."),
    "spatialu": ("__device__ __forceinline__ void spatial1u_body(", "#define ROMIS_SPATIAL1U_KERNEL"),
    "spatialn": ("__device__ __forceinline__ void spatialn_ntl_body(", "#ifndef ROMIS_SPATIAL2_NTL_WPE"),
    "final": ("__device__ __forceinline__ void final_sorted_body(", "extern \"C\" __global__ __launch_bounds__(256) void k_final_n1_sorted("),
}


def body_span(src, which):
    a = src.index(SPANS[which][0])
    b = src.index(SPANS[which][1], a)
    return a, b


# name -> list of (regex, replacement) applied inside spatial1_ntl_body only
VARIANTS = {
    # the K neighbour target pdfs (the combine's p-hat chains) -> a 2-op stand-in on the same inputs
    "no_phat": [(r"target_pdf(?:_lean)?\(s, f, cur, p, c, tb\)", "fabsf(p.x + c.y)")],
    # the neighbour offset draws (2 mix32 + umulhi + clamp each) -> a multiply-add of the pixel state
    "no_rng": [(r"__umulhi\(draw\(ps, 2u \* n\), span\)", "((ps + 2u * n) % span)"),
               (r"__umulhi\(draw\(ps, 2u \* n \+ 1u\), span\)", "((ps >> 8) + n) % span")],
    # the accepted neighbours' reservoir gathers read the pixel's own records instead (same instructions, coalesced
    # addresses): what the scattered addresses cost in the memory pipeline
    "coalesced": [(r"ld_at\(ia, qo\[(n \+ 1|0)\]\)", "ld_at(ia, pofs)"), (r"ld_at\(ib, qo\[(n \+ 1|0)\]\)", "ld_at(ib, pofs)")],
    # no neighbour reservoir loads at all (the pixel's own records stand in): gather latency and traffic removed
    "no_gather": [(r"na\[(n \+ 1|0)\] = ld_at\(ia, qo\[(n \+ 1|0)\]\);", r"na[\1] = ca;"),
                  (r"nb\[(n \+ 1|0)\] = ld_at\(ib, qo\[(n \+ 1|0)\]\);", r"nb[\1] = cb;")],
    # round 5 (C4f): only the position / W half of each accepted neighbour's reservoir gathered (colour / M from the
    # pixel's own): the upper bound of a 16-byte sample record for the light-grid scenes
    "half_gather": [(r"nb\[(n \+ 1|0)\] = ld_at\(ib, qo\[(n \+ 1|0)\]\);", r"nb[\1] = cb;")],
    # round 5 (C2 at N = 2, k_spatial2_ntl): no neighbour reservoir gathers (the pixel's own sub-reservoirs stand in)
    "n2_no_gather": [(r"na\[j\] = ld_at\(ia, qo\[n\] \+ \(uint32_t\)j \* jofs\); nb\[j\] = ld_at\(ib, qo\[n\] \+ \(uint32_t\)j \* jofs\);",
                      "na[j] = ca[j]; nb[j] = cb[j];")],
    # round 5: final shading (k_final_n1_sorted at C2) -- the shadow rays, the shading, the tone map, the binning
    "fin_no_trace": [(r"s_vis\[__float_as_uint\(a\.w\)\] = visible\(bvh, xyz\(a\), xyz\(b\)\) \? 1u : 0u;",
                      "s_vis[__float_as_uint(a.w)] = (a.x < b.x) ? 1u : 0u;")],
    "fin_no_shade": [(r"sc\[j\] = shade\(s, f, px, r\[j\]\.pos, r\[j\]\.col, tb\);",
                      "sc[j] = vadd(vscale(r[j].col, px.N.x), vscale(r[j].pos, px.P.y));")],
    "fin_no_tonemap": [(r"color = tone_map_rgb\(f, vdivs\(color, \(float\)NT\), tb\);", "color = vscale(color, 0.5f);")],
    "fin_no_sort": [(r"bin\[j\] = need\[j\] \? target_bin\(bvh, r\[j\]\.pos\) : 0u;", "bin[j] = 0u;")],
    # everything after the window barrier replaced by a copy of the pixel's own records (the skeleton: own loads,
    # window DMA, barrier, stores), and the same without the window DMA
    "skeleton": [(r"    const float4 cn = l_nt\[\(uint32_t\)\(y - ay0\) \* AW \+ \(uint32_t\)\(x - ax0\)\];",
                  "    st_at(oa, pofs, ca); st_at(ob, pofs, make_float4(cb.x, cb.y, cb.z, __uint_as_float(qi[0] + qo[1]))); return;\n"
                  "    const float4 cn = l_nt[(uint32_t)(y - ay0) * AW + (uint32_t)(x - ax0)];")],
    "skeleton_nodma": [(r"    const float4 cn = l_nt\[\(uint32_t\)\(y - ay0\) \* AW \+ \(uint32_t\)\(x - ax0\)\];",
                        "    st_at(oa, pofs, ca); st_at(ob, pofs, make_float4(cb.x, cb.y, cb.z, __uint_as_float(qi[0] + qo[1]))); return;\n"
                        "    const float4 cn = l_nt[(uint32_t)(y - ay0) * AW + (uint32_t)(x - ax0)];"),
                       (r"    ntl_stage_window\(rg, n_t, l_nt, ax0, ay0, AW, n_apron\);", "")],
    # RIS (ris_pixel): the candidates' target pdfs, light-index draws + accept draws, reservoir updates
    "ris_no_phat": [(r"target_pdf(?:_lean)?\(s, f, px, pos, col, tb\);", "fabsf(pos.x + col.y);")],
    "ris_no_rng": [(r"uniform_index\(draw\(ps, 4u \* c\), L\)", "min(c, L - 1u)"),
                   (r"rand01\(draw\(ps, 4u \* c \+ 3u\)\)", "0.5f")],
    "ris_no_update": [(r"res_update<NT>\(r, N, pos, col, weight\(pd\), rand01\(draw\(ps, 4u \* c \+ 3u\)\), pd\);",
                       "r[0].wsum += weight(pd); r[0].pos = vadd(r[0].pos, pos);")],
    # round 4: what the keyed hash itself costs with the light fetch still random per lane --
    # the draws as the bare Weyl sequence ps + slot * G (no mixing), as a one-multiply xorshift-multiply-xorshift,
    # and the light index by shift (umulhi(d, L) == d >> 25 exactly for L = 128, C2's point lights)
    "ris_rng_weyl": [(r"uniform_index\(draw\(ps, 4u \* c\), L\)", "uniform_index(ps + 4u * c * 0x9E3779B9u, L)"),
                     (r"rand01\(draw\(ps, 4u \* c \+ 3u\)\)", "rand01(ps + (4u * c + 3u) * 0x9E3779B9u)")],
    "ris_rng_1mul": [(r"uniform_index\(draw\(ps, 4u \* c\), L\)", "uniform_index(draw1(ps, 4u * c), L)"),
                     (r"rand01\(draw\(ps, 4u \* c \+ 3u\)\)", "rand01(draw1(ps, 4u * c + 3u))"),
                     (r"const uint32_t ps = pix_state\(key, y \* rg\.W \+ x\);",
                      "const uint32_t ps = pix_state(key, y * rg.W + x);\n"
                      "            auto draw1 = [](uint32_t ps_, uint32_t slot) { uint32_t h = ps_ + slot * 0x9E3779B9u; "
                      "h ^= h >> 16; h *= 0x7feb352du; return h ^ (h >> 15); };")],
    "ris_lidx_shift": [(r"uniform_index\(draw\(ps, 4u \* c\), L\)", "(draw(ps, 4u * c) >> 25)")],
    # light grids (C4 / C5): no light-table read at all -- the drawn light's corner from its index by arithmetic
    # (the upper bound of a closed-form regularLightGrid corner), its colour a constant
    "ris_grid_noload": [(r"pos = vadd\(vadd\(xyz\(lt\[0\]\), vscale\(shared_row\(1\), a\)\), vscale\(shared_row\(2\), b\)\);\n"
                         r"(\s+)const v3 gc = xyz\(lt\[1\]\);",
                         "const uint32_t li_ = (uint32_t)(lt - lights) >> 1; "
                         "pos = vadd(vadd(mk((float)(li_ >> 6) * 0.01f, 0.9f, (float)(li_ & 63u) * 0.01f), "
                         "vscale(shared_row(1), a)), vscale(shared_row(2), b));\n\\1const v3 gc = mk(0.5f, 0.5f, 0.5f);")],
    # kLtRegular (C4 / C5): the drawn light's colour gather replaced by a value of its index (no memory access)
    "ris_reg_noload": [(r"const v3 gc = xyz\(lights\[i\]\);",
                        "const v3 gc = mk(0.5f + (float)(i & 7u) * 0.01f, 0.5f, 0.5f);")],
    # no candidate loop at all (every pixel takes the miss path): primary rays + stores, the kernel's floor
    "ris_no_cand": [(r"\? 0u : f\.M;", "? 0u : 0u;")],
    # k_spatial1u (C5's unbiased + visibility pass): the Z loop's shadow rays, its sign-only target pdfs, its
    # G-buffer gathers, and the combine's K target pdfs, each replaced by a data-dependent stand-in
    "u_no_vis": [(r"\(!VIS \|\| visible\(bvh, rp\.P, cmb\.pos\)\)", "(!VIS || rp.P.x != cmb.pos.x)"),
                 (r"const bool v = !VIS \|\| visible\(bvh, cur\.P, cmb\.pos\);", "const bool v = !VIS || cur.P.x != cmb.pos.x;")],
    "u_no_zphat": [(r": target_pdf_positive\(s, f, rp, cmb\.pos, cmb\.col, tb\);", ": rp.P.y != cmb.pos.y;")],
    "u_no_zload": [(r"const float4 qn = ld_at\(n_t, qo\[n\]\), qp = ld_at\(p_mat, qo\[n\]\);",
                    "const float4 qn = cn, qp = make_float4(cpm.x + (float)n, cpm.y, cpm.z, cpm.w);")],
    "u_no_comb": [(r"cmb\.take\(target_pdf\(s, f, cur, p, c, tb\), na\[n\]\.w",
                   "cmb.take(p.x * c.y + cur.P.z, na[n].w")],
    # pieces of the target pdf itself (shared device functions: every kernel changes, RIS is the one timed)
    "risg_no_pow": [(r"return pow_pre\(x, px, pw, job\) \? pw : pow_core\(tb, job, px\.kd_sh\.w\);",
                     "return x * px.kd_sh.w;")],
    "risg_no_div": [(r"return vdivs\(vadd\(diffuse, specular\), d \* d\);", "return vscale(vadd(diffuse, specular), d * d);")],
    "risg_no_norm": [(r"v3 L = vnormalize_len\(vsub\(lpos, px\.P\), r\.d\);", "v3 L = vsub(lpos, px.P); r.d = L.x + L.y;"),
                     (r"v3 R = vnormalize\(vsub\(vscale\(px\.N, 2\.0f \* r\.dotNL\), L\)\);",
                      "v3 R = vsub(vscale(px.N, 2.0f * r.dotNL), L);")],
    "risg_no_len": [(r"return vlength\(shade_ref\(s, f, px, lpos, lcol, tb\)\);",
                     "const v3 sh_ = shade_ref(s, f, px, lpos, lcol, tb); return sh_.x + sh_.y + sh_.z;")],
    # round 5: every block reads the SAME tile's records and window (the image's middle tile: geometry, L2-resident after
    # the first blocks) and stores to its own tile -- the pass's compute with its load phase reduced to L2 hits.  If this
    # runs far below the shipped time, the pass's time is load phase + compute in series, not either alone.
    "l2res": [(r"    const int tx0 = \(int\)\(rg\.rx0 \+ \(tile % ntx\) \* kTileW\), ty0 = \(int\)\(rg\.ry0 \+ \(tile / ntx\) \* kTH\);",
               "    const int stx0 = (int)(rg.rx0 + (tile % ntx) * kTileW), sty0 = (int)(rg.ry0 + (tile / ntx) * kTH);\n"
               "    const uint32_t ftile = ((rg.rh + kTH - 1) / kTH) / 2u * ntx + ntx / 2u;\n"
               "    const int tx0 = (int)(rg.rx0 + (ftile % ntx) * kTileW), ty0 = (int)(rg.ry0 + (ftile / ntx) * kTH);"),
              (r"(    const uint32_t pofs = \(\(uint32_t\)\(y - \(int\)rg\.vy0\) \* rg\.vw \+ \(uint32_t\)\(x - \(int\)rg\.vx0\)\) << 4;)",
               "\\1\n    const uint32_t pofs_s = pofs + ((((uint32_t)(sty0 - ty0)) * rg.vw + (uint32_t)(stx0 - tx0)) << 4);"),
              (r"st_at\((oa|ob|odbg|rp_out), pofs", r"st_at(\1, pofs_s")],
    # the whole combine (takes) -> sums
    "no_take": [(r"cmb\.take\(target_pdf(?:_lean)?\(s, f, cur, p, c, tb\), na\[n\]\.w, __float_as_uint\(nb\[n\]\.w\), p, c\);",
                 "cmb.wsum += target_pdf(s, f, cur, p, c, tb) * na[n].w; cmb.macc += __float_as_uint(nb[n].w);")],
}

VARIANTS["l2res_no_phat"] = VARIANTS["l2res"] + VARIANTS["no_phat"]
VARIANTS["l2res_no_gather"] = VARIANTS["l2res"] + VARIANTS["no_gather"]


def main():
    src = open(SRC).read()
    only = set(sys.argv[1:])
    for name, subs in VARIANTS.items():
        if only and name not in only:
            continue
        if name.startswith("risg_"):
            a, b = 0, len(src)
        else:
            a, b = body_span(src, "ris" if name.startswith("ris_") else "spatialu" if name.startswith("u_")
                             else "spatialn" if name.startswith("n2_") else "final" if name.startswith("fin_") else "spatial")
        body = src[a:b]
        for pat, rep in subs:
            body, n = re.subn(pat, rep, body)
            if n == 0:
                raise SystemExit(f"{name}: pattern not found: {pat}")
        vdir = os.path.join(build.OUT, "variants", name)
        os.makedirs(vdir, exist_ok=True)
        path = os.path.join(vdir, "kernels.hip")
        with open(path, "w") as fh:
            fh.write(src[:a] + body + src[b:])
        obj = os.path.join(vdir, "kernels.hip.o")
        subprocess.check_call([build.HIPCC] + build.COMMON + build.SOURCES[0][1] + ["-c", path, "-o", obj])
        objs = [obj] + [os.path.join(build.OUT, s + ".o") for s, _ in build.SOURCES[1:]]
        subprocess.check_call([build.HIPCC, "-shared", f"--offload-arch={build.ARCH}", "-fno-gpu-rdc", "-o",
                               os.path.join(vdir, "libromis_amd.so")] + objs)
        print(name, "built")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Ablation study: price each part of the per-candidate arithmetic by building kernel variants that replace it
with a cheap stand-in (device_math.h / kernels.hip ROMIS_ABL_* hooks), then timing every variant with
scripts/kbench.py.  Variants change results -- they exist only to measure; the shipped library defines none.

    python scripts/ablate.py build            # here (cross-compiles gfx950)
    python scripts/ablate.py run [--rounds 3]  # on the GPU box: one kbench process per variant, JSON to stdout
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

VARIANTS = {
    "rng": ["ROMIS_ABL_RNG"],                 # cheap hash instead of the keyed mix32 draws
    "pow": ["ROMIS_ABL_POW"],                 # pow(cos, n) -> cos * n
    "shade": ["ROMIS_ABL_SHADE"],             # target pdf -> one dot product
    "light0": ["ROMIS_ABL_LIGHT0"],           # every candidate reads light 0 (no LDS bank conflicts)
    "spatial_self": ["ROMIS_ABL_SPATIAL_SELF"],  # spatial neighbours = the pixel itself (no gathers)
    "spatial_copy": ["ROMIS_ABL_SPATIAL_COPY"],  # spatial = copy own reservoir (memory floor)
    "pdcur": ["ROMIS_ABL_PDCUR"],             # k_spatial1: the pixel's own target pdf not evaluated (W stand-in)
}


def lib_path(name):
    from romis_amd import build
    return os.path.join(build.OUT, "variants", name, "libromis_amd.so")


def main():
    cmd = sys.argv[1] if len(sys.argv) > 1 else "run"
    if cmd == "build":
        from romis_amd import build
        for name, defs in VARIANTS.items():
            print(build.build_variant(name, defs))
        return
    extra = sys.argv[2:]
    out = {}
    for name in ["exact"] + list(VARIANTS):
        env = dict(os.environ)
        if name != "exact":
            env["ROMIS_AMD_LIB"] = lib_path(name)
        r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "kbench.py"), "--only", "default"] + extra,
                           env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(r.stderr, file=sys.stderr)
            raise SystemExit(f"variant {name} failed")
        out[name] = json.loads(r.stdout)["default"]
        print(name, out[name], file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

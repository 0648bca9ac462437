"""Build libromis_amd.so in-tree (romis_amd/_build/) with hipcc for gfx950.

    python -m romis_amd.build [--force]

Flags that matter for parity (DESIGN.md "Floating point"): -ffp-contract=off (no FMA contraction, host and
device), correctly rounded f32 division / sqrt, no fast-math.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_build")
LIB = os.path.join(OUT, "libromis_amd.so")
ARCH = os.environ.get("ROMIS_AMD_ARCH", "gfx950")

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", f"-I{os.path.join(ROOT, 'include')}",
          f"-I{CSRC}"]
DEVICE = [f"--offload-arch={ARCH}", "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-rdc"]

# -fno-slp-vectorize: the SLP pass packs independent f32 multiplies / adds into v_pk_* ops, which issue at the
# cost of an FMA (≈4.5 cycles per wave instruction on gfx950) instead of ≈2.4 for each scalar op, and need
# v_mov shuffles to assemble their operand pairs; without it: RIS 354 -> 340 us, spatial 85 -> 81, final 104 -> 92
# (kbench, profiles/r2/noslp), fewer VGPRs and no RIS scratch spill.  Results are identical (no contraction).
KERNEL_FLAGS = ["-fno-slp-vectorize"]

SOURCES = [
    ("kernels.hip", ["-x", "hip"] + DEVICE + KERNEL_FLAGS),
    ("restir.cpp", ["-x", "hip"] + DEVICE),
    ("mis.hip", ["-x", "hip"] + DEVICE + KERNEL_FLAGS),
    ("bvh.cpp", ["-x", "c++"]),
    ("screen.cpp", ["-x", "c++"]),
]
HEADERS = ["device_math.h", "restir_types.h", "launch.h", "bvh.h", "pow10_table.h", "kernels_common.h", "launch_events.h"]


def source_hash() -> str:
    """sha256 over the device sources, the launcher (restir.cpp decides which buffers a pass reads and writes) and
    the flags: identifies the kernels a profile was measured on (bench.py reports a committed PMC traffic figure
    only when it matches)."""
    import hashlib
    h = hashlib.sha256()
    for f in [SOURCES[0][0], SOURCES[1][0]] + HEADERS:
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    h.update(" ".join([c for c in COMMON + DEVICE + KERNEL_FLAGS if not c.startswith("-I")]).encode())   # flags, not paths
    return h.hexdigest()[:16]


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src: str, extra: list[str], force: bool) -> str:
    obj = os.path.join(OUT, os.path.basename(src) + ".o")
    deps = [os.path.join(CSRC, src)] + [os.path.join(CSRC, h) for h in HEADERS] + \
        [os.path.join(ROOT, "include", "restir_c.h"), __file__]
    if force or _stale(obj, deps):
        cmd = [HIPCC] + COMMON + extra + ["-c", os.path.join(CSRC, src), "-o", obj]
        subprocess.check_call(cmd)
    return obj


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OUT, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(lambda s: _compile(s[0], s[1], force), SOURCES))
    if force or _stale(LIB, objs):
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-fno-gpu-rdc", "-o", LIB] + objs
        subprocess.check_call(cmd)
    tool = os.path.join(OUT, "tools", "fastmath_check")
    src = os.path.join(ROOT, "tests", "hip", "fastmath_check.hip")
    if os.path.exists(src) and (force or _stale(tool, [src, os.path.join(CSRC, "device_math.h"), __file__])):
        os.makedirs(os.path.dirname(tool), exist_ok=True)
        subprocess.check_call([HIPCC] + COMMON + DEVICE + ["-x", "hip", src, "-o", tool])
    if verbose:
        print(LIB)
    return LIB


def build_variant(name: str, defines: list[str], flags: list[str] | None = None) -> str:
    """Build _build/variants/<name>/libromis_amd.so with kernels.hip compiled under extra -D defines (launch-bound
    knobs such as ROMIS_SPATIAL_WPE) and compiler flags.  The host objects are the shipped ones."""
    build()
    vdir = os.path.join(OUT, "variants", name)
    os.makedirs(vdir, exist_ok=True)
    obj = os.path.join(vdir, "kernels.hip.o")
    subprocess.check_call([HIPCC] + COMMON + SOURCES[0][1] + [f"-D{d}" for d in defines] + list(flags or []) +
                          ["-c", os.path.join(CSRC, "kernels.hip"), "-o", obj])
    lib = os.path.join(vdir, "libromis_amd.so")
    objs = [obj] + [os.path.join(OUT, s + ".o") for s, _ in SOURCES[1:]]
    subprocess.check_call([HIPCC, "-shared", f"--offload-arch={ARCH}", "-fno-gpu-rdc", "-o", lib] + objs)
    return lib


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    args = ap.parse_args(argv)
    build(force=args.force, verbose=True)
    return 0



# C++ programs over the C++ binding (include/romis_amd/restir.hpp): the reference-side callers the C++ wrapper tests
# drive (tests/test_cpp_wrapper.py).  Built on the build host next to the library; the GPU box runs the prebuilt ones.
CPP_PROGRAMS = [("render_scene.cpp", "render_scene"), ("render_threads.cpp", "render_threads"),
                ("write_outputs.cpp", "write_outputs")]
CPP_DIR = os.path.join(ROOT, "tests", "cpp")


def build_cpp_program(src: str, out: str) -> str:
    """g++ one program against libromis_amd.so (rpath to the in-tree build) when it is older than its sources."""
    lib = LIB if os.path.exists(LIB) else build()
    libdir = os.path.dirname(lib)
    deps = [src, os.path.join(CPP_DIR, "scene_io.h"), os.path.join(ROOT, "include", "restir_c.h"),
            os.path.join(ROOT, "include", "romis_amd", "restir.hpp")]
    if _stale(out, deps):
        subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-pthread", f"-I{os.path.join(ROOT, 'include')}",
                               src, "-o", out, f"-L{libdir}", "-lromis_amd", f"-Wl,-rpath,{libdir}"])
    return out


def build_cpp_programs() -> list[str]:
    return [build_cpp_program(os.path.join(CPP_DIR, src), os.path.join(OUT, out)) for src, out in CPP_PROGRAMS]

if __name__ == "__main__":
    sys.exit(main())

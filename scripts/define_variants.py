#!/usr/bin/env python3
"""Exact build variants of the kernels: the product's kernels.hip compiled with extra -D defines (launch-shape and
register-cap macros that never change results), each into romis_amd/_build/variants/<name>/libromis_amd.so for
scripts/kbench_libs.sh A/B runs on the GPU.

    python scripts/define_variants.py ris_w6:ROMIS_RIS_WPE=6 ris_w4:ROMIS_RIS_WPE=4
"""
import concurrent.futures as cf
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from romis_amd import build  # noqa: E402


def build_one(spec):
    name, _, defs = spec.partition(":")
    vdir = os.path.join(build.OUT, "variants", name)
    os.makedirs(vdir, exist_ok=True)
    obj = os.path.join(vdir, "kernels.hip.o")
    flags = ["-D" + d for d in defs.split(",") if d]
    subprocess.check_call([build.HIPCC] + build.COMMON + build.SOURCES[0][1] + flags +
                          ["-c", os.path.join(build.CSRC, "kernels.hip"), "-o", obj])
    objs = [obj] + [os.path.join(build.OUT, s + ".o") for s, _ in build.SOURCES[1:]]
    subprocess.check_call([build.HIPCC, "-shared", f"--offload-arch={build.ARCH}", "-fno-gpu-rdc", "-o",
                           os.path.join(vdir, "libromis_amd.so")] + objs)
    return name + " " + " ".join(flags)


def main():
    build.build()
    # the variants compile side by side (one kernels.hip each, ~2 min; 4 at a time fit the container's memory)
    with cf.ThreadPoolExecutor(max_workers=4) as ex:
        for line in ex.map(build_one, sys.argv[1:]):
            print(line)


if __name__ == "__main__":
    main()

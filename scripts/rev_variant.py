#!/usr/bin/env python3
"""Build romis_amd/_build/variants/<name>/libromis_amd.so from kernels.hip + restir.cpp as committed at a git revision
(device headers too), for A/B runs against the working tree with scripts/kbench_libs.sh.

    python scripts/rev_variant.py <name> <rev>
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from romis_amd import build  # noqa: E402


def main():
    name, rev = sys.argv[1], sys.argv[2]
    vdir = os.path.join(build.OUT, "variants", name)
    os.makedirs(vdir, exist_ok=True)
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "csrc")
        os.makedirs(src)
        for f in [s for s, _ in build.SOURCES] + build.HEADERS:
            with open(os.path.join(src, f), "wb") as fh:
                fh.write(subprocess.check_output(["git", "-C", ROOT, "show", f"{rev}:romis_amd/csrc/{f}"]))
        objs = []
        for s, extra in build.SOURCES:
            obj = os.path.join(vdir, s + ".o")
            flags = [c if not c.startswith("-I" + build.CSRC) else "-I" + src for c in build.COMMON]
            subprocess.check_call([build.HIPCC] + flags + extra + ["-c", os.path.join(src, s), "-o", obj])
            objs.append(obj)
    subprocess.check_call([build.HIPCC, "-shared", f"--offload-arch={build.ARCH}", "-fno-gpu-rdc", "-o",
                           os.path.join(vdir, "libromis_amd.so")] + objs)
    print(name, rev)


if __name__ == "__main__":
    main()

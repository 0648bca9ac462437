#!/bin/bash
# Round 5 probe 27: the N = 2 pass over point-light handles (k_spatial2h_t2, RIS N = 2 writing both sub-reservoirs'
# handles) -- the handle / N = 2 parity tests, then C2 at N = 2 against the committed library ("head") and with
# spatial.handles = 0.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p27
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu \
    -k "handles or N2 or n2 or miss_tiles or full_size_c2" > gpurun_out/r5p27/tests.log 2>&1 \
    || { tail -30 gpurun_out/r5p27/tests.log; exit 40; }
tail -2 gpurun_out/r5p27/tests.log
bash scripts/ab_libs_cfg.sh r5p27 c2 "--N 2 --rounds 5 --frames 10 --variants handles: ntl:spatial.handles=0" head || exit 41
bash scripts/ab_libs_cfg.sh r5p27b c2 "--N 2 --rounds 5 --frames 10 --variants handles: ntl:spatial.handles=0" head || exit 42

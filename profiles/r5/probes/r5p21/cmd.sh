#!/bin/bash
# Round 5 probe 21: the reservoir update's acceptance decided from one fma residual outside a 2^-24 band (accept_u,
# device_math.h) instead of the correctly rounded division -- the whole GPU suite, then kbench / cfg_kbench against the
# committed library (variant "head", scripts/rev_variant.py), interleaved.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p21
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5p21/tests.log 2>&1 \
    || { tail -30 gpurun_out/r5p21/tests.log; exit 40; }
tail -2 gpurun_out/r5p21/tests.log
bash scripts/kbench_libs.sh r5p21/times "--only default --rounds 9 --frames 10" head || exit 41
bash scripts/kbench_libs.sh r5p21/times2 "--only default --rounds 9 --frames 10" head || exit 42
bash scripts/ab_libs_cfg.sh r5p21 c4f "--rounds 3 --frames 3" head || exit 43

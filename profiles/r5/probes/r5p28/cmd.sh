#!/bin/bash
# Round 5 probe 28: the acceptance rule also settling w = 0 (back-facing lights, wSum still at its FLT_MIN seed) without the
# division -- the whole GPU suite, then kbench / cfg_kbench against the
# committed library (variant "head", scripts/rev_variant.py), interleaved.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p28
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5p28/tests.log 2>&1 \
    || { tail -30 gpurun_out/r5p28/tests.log; exit 40; }
tail -2 gpurun_out/r5p28/tests.log
bash scripts/kbench_libs.sh r5p28/times "--only default --rounds 9 --frames 10" head || exit 41
bash scripts/kbench_libs.sh r5p28/times2 "--only default --rounds 9 --frames 10" head || exit 42
bash scripts/ab_libs_cfg.sh r5p28 c4f "--rounds 3 --frames 3" head || exit 43

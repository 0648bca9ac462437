#!/bin/bash
# Round 5 probe 26: N = 2 RIS keeping each sub-reservoir's accepted candidate index (the N = 1 loop's form) instead of
# its sample -- the N = 2 / general parity tests, then C2 at N = 2 against the committed library ("head").
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p26
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu \
    -k "N2 or n2 or odd_sizes or c3 or miss_tiles or ris or stage" > gpurun_out/r5p26/tests.log 2>&1 \
    || { tail -30 gpurun_out/r5p26/tests.log; exit 40; }
tail -2 gpurun_out/r5p26/tests.log
bash scripts/ab_libs_cfg.sh r5p26 c2 "--N 2 --rounds 5 --frames 10" head || exit 41
bash scripts/ab_libs_cfg.sh r5p26b c2 "--N 2 --rounds 5 --frames 10" head || exit 42

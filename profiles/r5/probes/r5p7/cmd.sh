#!/bin/bash
# Round 5 probe 7: k_spatial1h_t2 with the material table in LDS (batched window reads reverted) against the committed
# handle kernel (h1); handle parity first.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p7
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "handles or render_frame" > gpurun_out/r5p7/tests.log 2>&1 || { tail -40 gpurun_out/r5p7/tests.log; exit 40; }
tail -2 gpurun_out/r5p7/tests.log
bash scripts/kbench_libs.sh r5p7/times "--only default handles_off --rounds 9 --frames 10" h1 || exit 41
bash scripts/kbench_libs.sh r5p7/times2 "--only default handles_off --rounds 9 --frames 10" h1 || exit 42

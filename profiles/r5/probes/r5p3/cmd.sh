#!/bin/bash
# Round 5 probe 3: the spatial pass's load phase without its two early waits (powf tables by LDS-DMA behind the own
# loads; the block's background-tile flag through the scalar cache).  Parity of the spatial / background-tile tests,
# then kbench A/B against the previous load phase (variants old / tabonly / flagonly).
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p3
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "spatial or miss_tiles or full_size" > gpurun_out/r5p3/tests.log 2>&1 || { tail -30 gpurun_out/r5p3/tests.log; exit 40; }
tail -3 gpurun_out/r5p3/tests.log
bash scripts/kbench_libs.sh r5p3/times "--only default --rounds 7 --frames 10" old tabonly flagonly || exit 41

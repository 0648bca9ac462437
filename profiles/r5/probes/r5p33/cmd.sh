#!/bin/bash
# Round 5 probe 33: the handle parity tests with the 4,096-light grid case (the host's fallback to the reservoir form).
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p33
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu \
    -k "handles" > gpurun_out/r5p33/tests.log 2>&1 || { tail -30 gpurun_out/r5p33/tests.log; exit 40; }
tail -2 gpurun_out/r5p33/tests.log

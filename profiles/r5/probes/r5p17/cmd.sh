#!/bin/bash
# Round 5 probe 17 / 18: light-grid sample handles (k_spatial1g_t2; p17: W, M | i, a, b staged in LDS beside the n_t window and
# the light colours; p18: gathered by the n_t-window pass, one 16-byte gather per neighbour) -- the handle parity tests, then cfg_kbench C4f / C4 / C2 against spatial.handles = 0.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p17
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
    -k "handles or c4_c5 or miss_tiles" -m gpu > gpurun_out/r5p17/tests.log 2>&1 || { tail -30 gpurun_out/r5p17/tests.log; exit 40; }
tail -3 gpurun_out/r5p17/tests.log
for C in c4f c4 c2; do
    FR=3; [ $C = c2 ] && FR=10
    timeout -k 10 300 python3 scripts/cfg_kbench.py --config $C --rounds 5 --frames $FR \
        --variants "handles:" "ntl:spatial.handles=0" > gpurun_out/r5p17/$C.json 2> gpurun_out/r5p17/$C.err || { tail -5 gpurun_out/r5p17/$C.err; exit 41; }
    cat gpurun_out/r5p17/$C.json
done

#!/bin/bash
# Round 5 probe 34: temporal reuse fused into the primary + RIS kernel (k_primary_ris_n{1,2}_lds_pt_temporal,
# fuse.temporal) -- the whole GPU suite, then C3 (N = 1 and 2) with fuse.temporal 1 against 0.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p34
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5p34/tests.log 2>&1 \
    || { tail -30 gpurun_out/r5p34/tests.log; exit 40; }
tail -2 gpurun_out/r5p34/tests.log
for rep in 1 2; do
    timeout -k 10 300 python3 scripts/cfg_kbench.py --config c3 --rounds 5 --frames 10 \
        --variants "fused:fuse.temporal=1" "separate:fuse.temporal=0" > gpurun_out/r5p34/c3_$rep.json || exit 41
    cat gpurun_out/r5p34/c3_$rep.json
done
timeout -k 10 300 python3 scripts/cfg_kbench.py --config c3 --N 2 --rounds 5 --frames 10 \
    --variants "fused:fuse.temporal=1" "separate:fuse.temporal=0" > gpurun_out/r5p34/c3_n2.json || exit 42
cat gpurun_out/r5p34/c3_n2.json

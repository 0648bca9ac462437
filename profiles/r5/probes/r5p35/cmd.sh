#!/bin/bash
# Round 5 probe 35: temporal frames on sample handles -- the fused temporal kernel rebuilds the predecessor from the
# frame handles its last pass wrote, and the spatial passes read handles (k_spatial1h) -- the whole GPU suite, then C3
# with spatial.handles 1 against 0 (N = 1).
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p35
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5p35/tests.log 2>&1 \
    || { tail -30 gpurun_out/r5p35/tests.log; exit 40; }
tail -2 gpurun_out/r5p35/tests.log
for rep in 1 2; do
    timeout -k 10 300 python3 scripts/cfg_kbench.py --config c3 --rounds 5 --frames 10 \
        --variants "handles:spatial.handles=1" "planes:spatial.handles=0" > gpurun_out/r5p35/c3_$rep.json || exit 41
    cat gpurun_out/r5p35/c3_$rep.json
done
timeout -k 10 240 python3 bench.py --config c3 --steps 200 --warmup 20 > gpurun_out/r5p35/bench_c3.json 2> gpurun_out/r5p35/bench_c3.err \
    || { tail -5 gpurun_out/r5p35/bench_c3.err; exit 43; }
python3 -c "import json;d=json.loads(open('gpurun_out/r5p35/bench_c3.json').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['value'],d['kernels'])"

#!/bin/bash
# Round 4: the driver's bench command with longer GEMM clock pre-warms (now right before the warm-up frames).
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4j
mkdir -p $OUT
for rep in 1 2 3; do
    for ms in 500 1500 3000 0; do
        timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --prewarm-gemm-ms $ms \
            > $OUT/g${ms}_$rep.json 2> $OUT/g${ms}_$rep.err || { tail -5 $OUT/g${ms}_$rep.err; exit 21; }
        python3 -c "import json; d=json.load(open('$OUT/g${ms}_$rep.json')); print('gemm$ms', d['ms_per_step'], d['value'], d['roofline']['avg_launch_us'])"
    done
done

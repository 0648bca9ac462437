#!/bin/bash
# Every BASELINE.json config on one GPU (bench.py --config cN), plus the reference-default N = 2 for c2 / c3.
#   scripts/all_configs.sh <tag>
set -o pipefail
TAG=${1:-configs}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO" || exit 1
export TMPDIR=/tmp
for C in c1 c2 c3 c4 c5 c4f c5f; do
    STEPS=200; WARM=20; case $C in c5|c5f) STEPS=30; WARM=5;; c4f) STEPS=100;; esac
    timeout -k 10 300 python3 bench.py --config $C --steps $STEPS --warmup $WARM > "$OUT/bench_$C.json" 2> "$OUT/bench_$C.err" || { tail -5 "$OUT/bench_$C.err"; exit 60; }
    echo "$C $(python3 -c "import json,sys; d=json.load(open('$OUT/bench_$C.json')); r=d.get('roofline') or {}; print(d['ms_per_step'], d['value'], r.get('avg_launch_us'), r.get('frac'), (d.get('roofline_ris') or {}).get('frac'))")"
done
for C in c2 c3; do
    timeout -k 10 300 python3 bench.py --config $C --N 2 --steps 200 --warmup 20 > "$OUT/bench_${C}_N2.json" 2> "$OUT/bench_${C}_N2.err" || exit 61
    echo "${C}_N2 $(python3 -c "import json; d=json.load(open('$OUT/bench_${C}_N2.json')); print(d['ms_per_step'], d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])")"
done

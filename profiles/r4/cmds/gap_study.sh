#!/bin/bash
# Round 4: where the driver's 29 us per frame outside kernels goes (bench.py --steps 20 --warmup 5, the driver's
# command).  Plain runs with / without the pre-warm and the fenced timing events, then a kernel trace of each.
#   scripts/r4/gap_study.sh <tag>
set -o pipefail
TAG=${1:-gap}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$REPO" || exit 1
B="python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
run() {   # name, extra args
    echo "[gap] $1" >&2
    timeout -k 10 240 $B $2 > "$OUT/$1.json" 2> "$OUT/$1.err" || { tail -5 "$OUT/$1.err"; exit 11; }
}
run fence_noprewarm "--prewarm 0 --tune timing.fence=1"
run nofence_noprewarm "--prewarm 0"
run nofence_prewarm40 "--prewarm 40"
run fence_prewarm40 "--prewarm 40 --tune timing.fence=1"
run nofence_prewarm160 "--prewarm 160"
run nofence_noprewarm_b "--prewarm 0"
run nofence_prewarm40_b "--prewarm 40"
for v in "fence_noprewarm:--prewarm 0 --tune timing.fence=1" "nofence_prewarm40:--prewarm 40" "nofence_noprewarm100:--prewarm 0 --steps 100"; do
    name=${v%%:*}; extra=${v#*:}
    echo "[gap] trace $name" >&2
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr_$name" -o run -- \
        $B $extra > "$OUT/tr_$name.json" 2> "$OUT/tr_$name.err" || { tail -5 "$OUT/tr_$name.err"; exit 12; }
done
echo "[gap] done" >&2

#!/bin/bash
# Round 5 probe 36: rocprofv3 kernel trace + stats of the C3 bench line (N = 1 and 2): temporal frames' kernels.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
OUT=$REPO/gpurun_out/r5p36
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c3" -o run -- \
    python3 bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c3_bench.json" 2> "$OUT/c3.err" || exit 11
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c3_n2" -o run -- \
    python3 bench.py --config c3 --N 2 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c3_n2_bench.json" 2> "$OUT/c3_n2.err" || exit 12
find "$OUT" -name '*.csv' | sort

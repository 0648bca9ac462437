#!/bin/bash
# PC sampling (rocprofv3 host-trap, beta) of the headline frame's kernels: where the waves sit.
#   scripts/pc_sample.sh <tag> [interval_us]
set -o pipefail
TAG=${1:-pcs}
IV=${2:-1}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO" || exit 1
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
    --pc-sampling-interval "$IV" --output-format csv -d "$OUT/pcs" -o run -- \
    python3 scripts/kbench.py --only default --rounds 1 --frames 40 > "$OUT/kbench.json" 2> "$OUT/pcs.err"
rc=$?
tail -5 "$OUT/pcs.err"
find "$OUT" -name '*.csv' | head
for f in $(find "$OUT" -name '*.csv'); do head -3 "$f"; wc -l "$f"; done
exit $rc

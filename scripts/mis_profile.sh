#!/bin/bash
# Kernel trace + one SQ counter pass over scripts/mis_bench.py (GPU only, no CPU timing).
#   scripts/mis_profile.sh <tag> ["<mis_bench args>"]
set -o pipefail
TAG=${1:-mis}
MARGS=${2:-"--no-cpu --reps 1"}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd "$REPO" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python3 scripts/mis_bench.py $MARGS > "$OUT/mis_bench.jsonl" 2> "$OUT/mis_bench.err" || exit 11
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 scripts/mis_bench.py $MARGS > "$OUT/trace.jsonl" 2> "$OUT/trace.err" || exit 12
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d "$OUT/pmc0" -o run -- python3 scripts/mis_bench.py $MARGS > "$OUT/pmc0.jsonl" 2> "$OUT/pmc0.err" || exit 13

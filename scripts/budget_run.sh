#!/bin/bash
# Instruction budget of the spatial pass: SQ counters (one --pmc pass) and kbench times for the shipped library and
# each scripts/budget_variants.py variant.   scripts/budget_run.sh <tag> <variant> ...
set -o pipefail
TAG=${1:-budget}; shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO" || exit 1
export TMPDIR=/tmp
CTRS="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for V in shipped "$@"; do
    LIB=$REPO/romis_amd/_build/libromis_amd.so
    [ "$V" != shipped ] && LIB=$REPO/romis_amd/_build/variants/$V/libromis_amd.so
    ROMIS_AMD_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d "$OUT/sq_$V" -o run -- \
        python3 scripts/kbench.py --only default --rounds 1 --frames 3 > "$OUT/sq_$V.json" 2> "$OUT/sq_$V.err" || exit 50
done
bash scripts/kbench_libs.sh "$TAG/times" "--only default --rounds 5 --frames 10" "$@" || exit 51

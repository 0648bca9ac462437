#!/bin/bash
# HBM traffic of the spatial pass (FETCH_SIZE / WRITE_SIZE, separate --pmc passes) and its kernel time, per config:
# C2 (1080p headline: k_spatial1h_t2 over sample handles; "ntl": the n_t-window pass with reservoir gathers,
# spatial.handles = 0), C4 (4K, TOML camera: 87 % background), C4f / C5f (4K / 8K looking into the box: the passes on
# geometry, past the Infinity Cache; C4f's default k_spatial1g_t2 over light-grid handles, "ntl" its reservoir form).   scripts/traffic_study.sh <tag>
set -o pipefail
TAG=${1:-traffic}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO" || exit 1
export TMPDIR=/tmp
for CFG in c2 c4 c4f c5f; do
    VARS=("chunks:spatial.xcd_rows=255")
    [ $CFG = c2 ] || [ $CFG = c4f ] && VARS+=("ntl:spatial.xcd_rows=255,spatial.handles=0")
    FR=3; [ $CFG = c5f ] && FR=1
    for V in "${VARS[@]}"; do
        NAME=${V%%:*}
        for C in FETCH_SIZE WRITE_SIZE; do
            timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$OUT/${CFG}_${NAME}_$C" -o run -- \
                python3 scripts/cfg_kbench.py --config $CFG --rounds 1 --frames $FR --variants "$V" \
                > "$OUT/${CFG}_${NAME}_$C.json" 2> "$OUT/${CFG}_${NAME}_$C.err" || exit 40
        done
    done
    timeout -k 10 300 python3 scripts/cfg_kbench.py --config $CFG --rounds 5 --frames $FR \
        --variants "${VARS[@]}" > "$OUT/${CFG}_times.json" 2> "$OUT/${CFG}_times.err" || exit 41
    cat "$OUT/${CFG}_times.json"
done

#!/bin/bash
# HBM traffic of the spatial pass (FETCH_SIZE / WRITE_SIZE, separate --pmc passes) at C2 (1080p) and C4 (4K) for
# the XCD chunk order (default), one contiguous band per XCD (spatial.xcd_rows = 0) and the background-tile flags off
# (miss.tiles = 0), plus the kernel times of
# the same variants; at C4 also 32x8 tiles (spatial.th = 1) beside the default 32x16.   scripts/traffic_study.sh <tag>
set -o pipefail
TAG=${1:-traffic}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO" || exit 1
export TMPDIR=/tmp
for CFG in c2 c4; do
    VARS=("chunks:spatial.xcd_rows=255" "rows:spatial.xcd_rows=255,spatial.xcd_cols=0" "bands:spatial.xcd_rows=0"
          "tiles0:spatial.xcd_rows=255,miss.tiles=0")
    # C4: the default 32x16 tiles (k_spatial1_ntl_t2) against 32x8 ones
    [ $CFG = c4 ] && VARS+=("chunks_th1:spatial.xcd_rows=255,spatial.th=1")
    for V in "${VARS[@]}"; do
        NAME=${V%%:*}
        for C in FETCH_SIZE WRITE_SIZE; do
            timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/${CFG}_${NAME}_$C" -o run -- \
                python3 scripts/cfg_kbench.py --config $CFG --rounds 1 --frames 3 --variants "$V" \
                > "$OUT/${CFG}_${NAME}_$C.json" 2> "$OUT/${CFG}_${NAME}_$C.err" || exit 40
        done
    done
    timeout -k 10 200 python3 scripts/cfg_kbench.py --config $CFG --rounds 5 --frames 5 \
        --variants "${VARS[@]}" > "$OUT/${CFG}_times.json" 2> "$OUT/${CFG}_times.err" || exit 41
    cat "$OUT/${CFG}_times.json"
done

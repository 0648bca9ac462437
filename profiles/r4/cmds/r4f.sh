#!/bin/bash
# Round 4, 2-D XCD chunks for the spatial pass (spatial.xcd_cols) at C4 / C2: parity of the new order, kernel times and
# FETCH_SIZE per variant; then the FETCH_SIZE calibration of 16 / 32 / 64 / 128-byte gathers (scripts/probes/fetch_probe).
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4f
mkdir -p $OUT
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "ntl_2d or ntl_t2_2d or compact_light or render_frame_matches or c4_c5 or full_size_c2 or final or extreme" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 21; }
tail -1 $OUT/tests.log
# C4: spatial.xcd_rows counts 32 x 16 tile rows (k_spatial1_ntl_t2); 30 tiles = 960 px
C4=("chunks:spatial.xcd_rows=255" "r2c30:spatial.xcd_rows=2,spatial.xcd_cols=30" "r4c30:spatial.xcd_rows=4,spatial.xcd_cols=30"
    "r4c15:spatial.xcd_rows=4,spatial.xcd_cols=15" "r8c15:spatial.xcd_rows=8,spatial.xcd_cols=15"
    "r4c60:spatial.xcd_rows=4,spatial.xcd_cols=60" "r8c30:spatial.xcd_rows=8,spatial.xcd_cols=30")
# C2: 32 x 8 tiles; 4 rows of full width is the default
C2=("chunks:spatial.xcd_rows=255" "r8c30:spatial.xcd_rows=8,spatial.xcd_cols=30" "r4c30:spatial.xcd_rows=4,spatial.xcd_cols=30"
    "r8c20:spatial.xcd_rows=8,spatial.xcd_cols=20" "r16c15:spatial.xcd_rows=16,spatial.xcd_cols=15")
for CFG in c4 c2; do
    if [ $CFG = c4 ]; then VARS=("${C4[@]}"); else VARS=("${C2[@]}"); fi
    timeout -k 10 300 python3 scripts/cfg_kbench.py --config $CFG --rounds 5 --frames 5 --variants "${VARS[@]}" \
        > $OUT/${CFG}_times.json 2> $OUT/${CFG}_times.err || { tail -5 $OUT/${CFG}_times.err; exit 22; }
    cat $OUT/${CFG}_times.json
    for V in "${VARS[@]}"; do
        NAME=${V%%:*}
        timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/${CFG}_${NAME}_FETCH_SIZE" -o run -- \
            python3 scripts/cfg_kbench.py --config $CFG --rounds 1 --frames 3 --variants "$V" \
            > "$OUT/${CFG}_${NAME}_FETCH_SIZE.json" 2> "$OUT/${CFG}_${NAME}_FETCH_SIZE.err" || exit 23
    done
    echo "[r4f] $CFG done"
done
# the light table staged after the primary rays, only for tiles with a hit (ris.late = 1, default) vs every tile
for c in c4 c5 c2; do
    timeout -k 10 300 python3 scripts/cfg_kbench.py --config $c --rounds 4 --frames $([ $c = c5 ] && echo 3 || echo 8) \
        --variants late:ris.late=1 early:ris.late=0,final.miss=0 > $OUT/late_$c.json 2> $OUT/late_$c.err || { tail -5 $OUT/late_$c.err; exit 27; }
    cat $OUT/late_$c.json
done
# RIS ablations at C5 / C4 (scripts/budget_variants.py): the colour gather of kLtRegular, the candidate loop
bash scripts/ab_libs_cfg.sh r4f/ab c5 "--rounds 3 --frames 3" ris_reg_noload ris_no_cand ris_pf || exit 28
bash scripts/ab_libs_cfg.sh r4f/ab c4 "--rounds 3 --frames 8" ris_reg_noload ris_no_cand || exit 29
# C5's unbiased + visibility pass: Z-loop rays / sign-only p-hats / G-buffer gathers, combine p-hats
bash scripts/ab_libs_cfg.sh r4f/abu c5 "--rounds 3 --frames 3" u_no_vis u_no_zphat u_no_zload u_no_comb || exit 30
timeout -k 10 60 scripts/probes/_bin/fetch_probe > $OUT/fetch_probe.jsonl 2>&1 || { cat $OUT/fetch_probe.jsonl; exit 24; }
cat $OUT/fetch_probe.jsonl
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/probe_FETCH_SIZE -o run -- \
    scripts/probes/_bin/fetch_probe > $OUT/probe_fetch.log 2>&1 || exit 25
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $OUT/probe_RDREQ -o run -- \
    scripts/probes/_bin/fetch_probe > $OUT/probe_rdreq.log 2>&1 || exit 26
echo "[r4f] done"

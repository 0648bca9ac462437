#!/bin/bash
# Round 4: background-tile flags (MissTiles) -- the GPU suite, then kernel times with the flags and the late light
# staging on / off; 2-D XCD chunks with an odd number of chunks per chunk row (the XCDs then cover every column);
# the plain-vs-graph launch gap probe; the driver's bench command and C4 / C5 bench lines.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4g
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
    timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 \
        || { tail -40 $OUT/tests.log; exit 21; }
    tail -1 $OUT/tests.log
fi
for c in c5 c4 c2; do
    timeout -k 10 300 python3 scripts/cfg_kbench.py --config $c --rounds 4 --frames $([ $c = c5 ] && echo 3 || echo 8) \
        --variants default: tiles0:miss.tiles=0 late0:ris.late=0 both0:miss.tiles=0,ris.late=0 \
        > $OUT/mt_$c.json 2> $OUT/mt_$c.err || { tail -5 $OUT/mt_$c.err; exit 22; }
    cat $OUT/mt_$c.json
done
C2=("chunks:spatial.xcd_rows=255" "r8c20:spatial.xcd_rows=8,spatial.xcd_cols=20" "r4c20:spatial.xcd_rows=4,spatial.xcd_cols=20"
    "r16c20:spatial.xcd_rows=16,spatial.xcd_cols=20" "r8c12:spatial.xcd_rows=8,spatial.xcd_cols=12")
C4=("chunks:spatial.xcd_rows=255" "r4c24:spatial.xcd_rows=4,spatial.xcd_cols=24" "r8c24:spatial.xcd_rows=8,spatial.xcd_cols=24"
    "r4c40:spatial.xcd_rows=4,spatial.xcd_cols=40" "r8c40:spatial.xcd_rows=8,spatial.xcd_cols=40" "r2c24:spatial.xcd_rows=2,spatial.xcd_cols=24")
C5=("chunks:spatial.xcd_rows=255" "r8c48:spatial.xcd_rows=8,spatial.xcd_cols=48" "r16c48:spatial.xcd_rows=16,spatial.xcd_cols=48"
    "r8c80:spatial.xcd_rows=8,spatial.xcd_cols=80")
for CFG in c2 c4 c5; do
    case $CFG in c2) VARS=("${C2[@]}");; c4) VARS=("${C4[@]}");; c5) VARS=("${C5[@]}");; esac
    timeout -k 10 400 python3 scripts/cfg_kbench.py --config $CFG --rounds $([ $CFG = c5 ] && echo 3 || echo 5) \
        --frames $([ $CFG = c5 ] && echo 3 || echo 5) --variants "${VARS[@]}" \
        > $OUT/${CFG}_times.json 2> $OUT/${CFG}_times.err || { tail -5 $OUT/${CFG}_times.err; exit 23; }
    cat $OUT/${CFG}_times.json
    [ $CFG = c5 ] && continue
    for V in "${VARS[@]}"; do
        NAME=${V%%:*}
        timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/${CFG}_${NAME}_FETCH_SIZE" -o run -- \
            python3 scripts/cfg_kbench.py --config $CFG --rounds 1 --frames 3 --variants "$V" \
            > "$OUT/${CFG}_${NAME}_FETCH_SIZE.json" 2> "$OUT/${CFG}_${NAME}_FETCH_SIZE.err" || exit 24
    done
    echo "[r4g] $CFG done"
done
timeout -k 10 60 scripts/probes/_bin/gap_probe > $OUT/gap_probe.json 2>&1 || { cat $OUT/gap_probe.json; exit 25; }
cat $OUT/gap_probe.json
for rep in 1 2; do
    timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_$rep.json 2> $OUT/bench_$rep.err \
        || { tail -5 $OUT/bench_$rep.err; exit 26; }
    python3 -c "import json; d=json.load(open('$OUT/bench_$rep.json')); print('c2', d['ms_per_step'], d['value'], d['roofline']['avg_launch_us'], {k: v['us_per_launch'] for k, v in d['kernels'].items() if isinstance(v, dict)})"
done
for c in c4 c5; do
    timeout -k 10 240 python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err \
        || { tail -5 $OUT/bench_$c.err; exit 27; }
    python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', d['ms_per_step'], d['value'], d['roofline']['avg_launch_us'], {k: v['us_per_launch'] for k, v in d['kernels'].items() if isinstance(v, dict)})"
done
echo "[r4g] done"

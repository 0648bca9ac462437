#!/bin/bash
# Round 4: background-tile G-buffer skip (single unbiased pass) -- parity, C5 / C4 kernel times, C5 bench line.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4k
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_halo.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "miss_tiles or render_frame_matches or c4_c5 or full_size or stitch or in_flight or spatial_pass_bit_exact or final or halo_frames or unbiased" \
    > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 20; }
tail -1 $OUT/tests.log
for c in c5 c4; do
    timeout -k 10 300 python3 scripts/cfg_kbench.py --config $c --rounds 4 --frames $([ $c = c5 ] && echo 3 || echo 8) \
        --variants default: tiles0:miss.tiles=0 > $OUT/$c.json 2> $OUT/$c.err || { tail -5 $OUT/$c.err; exit 19; }
    cat $OUT/$c.json
done
timeout -k 10 240 python3 bench.py --config c5 --steps 30 --warmup 5 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err \
    || { tail -5 $OUT/bench_c5.err; exit 21; }
python3 -c "import json; d=json.load(open('$OUT/bench_c5.json')); print('c5', d['ms_per_step'], d['value'], {k: v['us_per_launch'] for k, v in d['kernels'].items() if isinstance(v, dict)})"

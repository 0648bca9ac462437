#!/bin/bash
# Round 4: C2's XCD order A/B with the background-tile flags on -- row chunks (default) against 2-D chunks, kernel
# times in two orders and the driver's bench command with each.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4h
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_halo.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "miss_tiles or render_frame_matches or c4_c5 or full_size or stitch or in_flight or spatial_pass_bit_exact or final or halo_frames" \
    > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 20; }
tail -1 $OUT/tests.log
for c in c4 c5; do
    timeout -k 10 300 python3 scripts/cfg_kbench.py --config $c --rounds 4 --frames $([ $c = c5 ] && echo 3 || echo 8) \
        --variants default: tiles0:miss.tiles=0 > $OUT/$c.json 2> $OUT/$c.err || { tail -5 $OUT/$c.err; exit 19; }
    cat $OUT/$c.json
done
V=("chunks:spatial.xcd_rows=255" "r8c20:spatial.xcd_rows=8,spatial.xcd_cols=20" "r8c12:spatial.xcd_rows=8,spatial.xcd_cols=12"
   "r6c20:spatial.xcd_rows=6,spatial.xcd_cols=20")
timeout -k 10 400 python3 scripts/cfg_kbench.py --config c2 --rounds 8 --frames 10 --variants "${V[@]}" > $OUT/ab1.json 2> $OUT/ab1.err \
    || { tail -5 $OUT/ab1.err; exit 21; }
cat $OUT/ab1.json
timeout -k 10 400 python3 scripts/cfg_kbench.py --config c2 --rounds 8 --frames 10 --variants "${V[3]}" "${V[2]}" "${V[1]}" "${V[0]}" \
    > $OUT/ab2.json 2> $OUT/ab2.err || { tail -5 $OUT/ab2.err; exit 22; }
cat $OUT/ab2.json
for rep in 1 2 3; do
    for v in "rows:" "r8c20:--tune spatial.xcd_rows=8 --tune spatial.xcd_cols=20"; do
        name=${v%%:*}; extra=${v#*:}
        timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline $extra > $OUT/b_${name}_$rep.json \
            2> $OUT/b_${name}_$rep.err || { tail -5 $OUT/b_${name}_$rep.err; exit 23; }
        python3 -c "import json; d=json.load(open('$OUT/b_${name}_$rep.json')); print('$name', d['ms_per_step'], d['value'], d['roofline']['avg_launch_us'])"
    done
done

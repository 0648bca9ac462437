#!/bin/bash
# Round 4: auto 2-D XCD chunks at C2 -- parity, kernel times against row chunks (two orders), the driver's command.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4m
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_halo.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "spatial_pass_bit_exact or full_size or miss_tiles or render_frame_matches or stitch or halo_frames" \
    > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 20; }
tail -1 $OUT/tests.log
V=("auto:spatial.xcd_cols=255" "rows:spatial.xcd_cols=0")
timeout -k 10 400 python3 scripts/cfg_kbench.py --config c2 --rounds 8 --frames 10 --variants "${V[@]}" > $OUT/ab1.json 2> $OUT/ab1.err || exit 21
cat $OUT/ab1.json
timeout -k 10 400 python3 scripts/cfg_kbench.py --config c2 --rounds 8 --frames 10 --variants "${V[1]}" "${V[0]}" > $OUT/ab2.json 2> $OUT/ab2.err || exit 22
cat $OUT/ab2.json
for rep in 1 2 3; do
    for v in "auto:" "rows:--tune spatial.xcd_cols=0"; do
        name=${v%%:*}; extra=${v#*:}
        timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline $extra > $OUT/b_${name}_$rep.json \
            2> $OUT/b_${name}_$rep.err || { tail -5 $OUT/b_${name}_$rep.err; exit 23; }
        python3 -c "import json; d=json.load(open('$OUT/b_${name}_$rep.json')); print('$name', d['ms_per_step'], d['value'], d['roofline']['avg_launch_us'])"
    done
done
# RIS at 7 waves per SIMD (72 VGPRs, 20 B of spills) against the shipped 6
bash scripts/ab_libs_cfg.sh r4m/w7 c2 "--rounds 5 --frames 10" ris_w7 || exit 24
bash scripts/ab_libs_cfg.sh r4m/w7 c4 "--rounds 3 --frames 8" ris_w7 || exit 25

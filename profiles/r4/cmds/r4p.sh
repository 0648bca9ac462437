#!/bin/bash
# Round 4: background-tile flags for N = 2 (k_spatial2_ntl, k_final_n2_sorted) -- parity, then C2 / C3 at N = 2 with
# the flags on and off.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4p
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_halo.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "miss_tiles or spatial_pass_bit_exact or final or render_frame_matches or full_size or stitch or halo_frames or in_flight" \
    > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 20; }
tail -1 $OUT/tests.log
for c in c2 c1; do
    timeout -k 10 300 python3 scripts/cfg_kbench.py --config $c --N 2 --rounds 4 --frames 8 --variants default: tiles0:miss.tiles=0 \
        > $OUT/${c}_N2.json 2> $OUT/${c}_N2.err || { tail -5 $OUT/${c}_N2.err; exit 21; }
    cat $OUT/${c}_N2.json
done

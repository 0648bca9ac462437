#!/bin/bash
# Round 6 s20: primary rays over per-tile candidate triangle lists (primary.tl, tile_triangles + closest_list) against
# the BVH walk: parity (the new test, the frame / handle / miss-tile / temporal / stitch tests), then interleaved
# kbench pairs at C2, C3, C4, C4f, C5 and C2 N = 2.
set -o pipefail
O=gpurun_out/s20; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "primary_tile_lists or render_frame or spatial_handles_frames or miss_tiles or tiles_stitch or temporal or full_size" \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 20; }
tail -1 $O/tests.log
for C in c2 c3 c4 c4f c5; do
    timeout -k 10 300 python3 scripts/cfg_kbench.py --config $C --rounds 5 --frames 6 \
        --variants default: tl_off:primary.tl=0 > $O/$C.json || exit 21
    echo "$C $(cat $O/$C.json)"
done
timeout -k 10 300 python3 scripts/cfg_kbench.py --config c2 --N 2 --rounds 5 --frames 6 \
    --variants default: tl_off:primary.tl=0 > $O/c2_n2.json || exit 22
echo "c2 N2 $(cat $O/c2_n2.json)"

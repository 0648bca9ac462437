#!/bin/bash
# Round 6 s22: point-light shadow rays over cone-cell triangle lists (final.cones, visible_cones): parity (the new
# test and the frame / miss-tile / temporal / stitch tests), then interleaved kbench pairs at C2, C3 and C2 N = 2.
set -o pipefail
O=gpurun_out/s22; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "cone_lists or primary_tile_lists or render_frame or miss_tiles or tiles_stitch or temporal" \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 20; }
tail -1 $O/tests.log
for C in c2 c3; do
    timeout -k 10 300 python3 scripts/cfg_kbench.py --config $C --rounds 7 --frames 8 \
        --variants default: cones_off:final.cones=0 > $O/$C.json || exit 21
    echo "$C $(cat $O/$C.json)"
done
timeout -k 10 300 python3 scripts/cfg_kbench.py --config c2 --N 2 --rounds 7 --frames 8 \
    --variants default: cones_off:final.cones=0 > $O/c2_n2.json || exit 22
echo "c2 N2 $(cat $O/c2_n2.json)"

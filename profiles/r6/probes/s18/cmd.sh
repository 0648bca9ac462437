#!/bin/bash
# Round 6 s18: the handle pass with the G-buffer records gathered too (k_spatial1hgg, spatial.gather = 2: no LDS window,
# the light table alone in LDS, 32 x 8 tiles) against the shipped gathered-handle pass (k_spatial1hg_t2), C2; register
# caps 7 (shipped build), 6 and 8 waves per SIMD (build variants hgg_w6 / hgg_w8).
set -o pipefail
O=gpurun_out/s18; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "spatial_handles_frames or miss_tiles" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 20; }
tail -1 $O/tests.log
for V in shipped hgg_w6 hgg_w8; do
    LIB=romis_amd/_build/libromis_amd.so
    [ "$V" != shipped ] && LIB=romis_amd/_build/variants/$V/libromis_amd.so
    ROMIS_AMD_LIB=$PWD/$LIB timeout -k 10 300 python3 scripts/cfg_kbench.py --config c2 --rounds 7 --frames 10 \
        --variants default: gall:spatial.gather=2 > $O/c2_$V.json || exit 21
    echo "$V $(cat $O/c2_$V.json)"
done

#!/bin/bash
# Round 6 s21: powf's core packed over candidate pairs in RIS (ROMIS_POW_PACK, target_pdf_pair / pow_core_pair): parity,
# then the shipped build (packed, 7 waves per SIMD) against nopack (ROMIS_POW_PACK=0) and pack_w6 (6 waves) at C2 / C3 / C4f.
set -o pipefail
O=gpurun_out/s21; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "primary_tile_lists or render_frame or spatial_handles_frames or miss_tiles or temporal or full_size or odd" \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 20; }
tail -1 $O/tests.log
for C in c2 c3 c4f; do
  for V in shipped nopack pack_w6; do
    LIB=romis_amd/_build/libromis_amd.so
    [ "$V" != shipped ] && LIB=romis_amd/_build/variants/$V/libromis_amd.so
    ROMIS_AMD_LIB=$PWD/$LIB timeout -k 10 300 python3 scripts/cfg_kbench.py --config $C --rounds 5 --frames 8 > $O/${C}_$V.json || exit 21
    echo "$C $V $(cat $O/${C}_$V.json)"
  done
done

#!/bin/bash
# Round 6 s17: the gathered-handle pass with every neighbour's handle gathered before the window's LDS-DMA and barrier
# (ROMIS_HG_EARLY=1, profiles/r6/pruned/hg_early_gather.diff; build variant hg_early) against the shipped pass, C2.
set -o pipefail
mkdir -p gpurun_out/hge
ROMIS_AMD_LIB=$PWD/romis_amd/_build/variants/hg_early/libromis_amd.so timeout -k 10 300 python -u -m pytest \
    tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "spatial_handles_frames or miss_tiles or tiles_stitch" > gpurun_out/hge/tests.log 2>&1 \
  && bash scripts/ab_libs_cfg.sh hge c2 "--rounds 7 --frames 10" hg_early > gpurun_out/hge/ab.log 2>&1

#!/bin/bash
# Round 6 s14: glibc powf coefficients through the scalar cache (ROMIS_POW_COEF_SMEM variant: RIS spills 13 -> 1) --
# parity of the variant, then A/B at C2, C2 N = 2, C4f, C3.
set -o pipefail
OUT=gpurun_out/r6s14
mkdir -p $OUT
export TMPDIR=/tmp
ROMIS_AMD_LIB=$PWD/romis_amd/_build/variants/coef_smem/libromis_amd.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "render_frame or c2 or device_math or handles or temporal" > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 21; }
tail -2 $OUT/parity.log
bash scripts/ab_libs_cfg.sh r6s14 c2 "--rounds 7 --frames 10" coef_smem || exit 22
bash scripts/ab_libs_cfg.sh r6s14 c2 "--rounds 7 --frames 10" coef_smem || exit 23
bash scripts/ab_libs_cfg.sh r6s14 c3 "--rounds 5 --frames 8" coef_smem || exit 24
bash scripts/ab_libs_cfg.sh r6s14 c4f "--rounds 3 --frames 3" coef_smem || exit 25

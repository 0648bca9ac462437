#!/bin/bash
# Round 5 probe 30: final shading in blocks of 1024 threads over 2 x 2 groups of 32 x 8 tiles (ROMIS_FINAL_TB=4 build
# variant: one BVH copy per 16 waves, 8 waves per SIMD instead of 6, the group's rays binned together) -- the frame
# tests through the variant, then kbench / cfg_kbench against the shipped library.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p30
ROMIS_AMD_LIB=$REPO/romis_amd/_build/variants/fin_tb4/libromis_amd.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 \
    --timeout-method thread tests -m gpu > gpurun_out/r5p30/tests.log 2>&1 || { tail -30 gpurun_out/r5p30/tests.log; exit 40; }
tail -2 gpurun_out/r5p30/tests.log
bash scripts/kbench_libs.sh r5p30/times "--only default --rounds 7 --frames 10" fin_tb4 || exit 41
bash scripts/kbench_libs.sh r5p30/times2 "--only default --rounds 7 --frames 10" fin_tb4 || exit 42
bash scripts/ab_libs_cfg.sh r5p30 c4f "--rounds 3 --frames 3" fin_tb4 || exit 43

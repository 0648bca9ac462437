#!/bin/bash
# Round 5 probe 24: RIS block order -- the fused primary + RIS kernel's tiles in reverse order (ROMIS_RIS_REV: C2's top
# rows, half geometry, first; its bottom rows, 10 % geometry, last) against the shipped order, C2 and C4f; the C2 frame
# tests through the variant.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p24
ROMIS_AMD_LIB=$REPO/romis_amd/_build/variants/ris_rev/libromis_amd.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests/test_gpu_parity.py -k "handles or full_size_c2 or miss_tiles" -m gpu > gpurun_out/r5p24/tests.log 2>&1 \
    || { tail -30 gpurun_out/r5p24/tests.log; exit 40; }
tail -2 gpurun_out/r5p24/tests.log
bash scripts/kbench_libs.sh r5p24/times "--only default --rounds 7 --frames 10" ris_rev || exit 41
bash scripts/kbench_libs.sh r5p24/times2 "--only default --rounds 7 --frames 10" ris_rev || exit 42
bash scripts/ab_libs_cfg.sh r5p24 c4f "--rounds 3 --frames 3" ris_rev || exit 43

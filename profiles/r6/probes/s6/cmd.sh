#!/bin/bash
# Round 6 s6: shadow-ray traversal with both successors requested before the box test (ROMIS_OCC_PREFETCH variant):
# parity of the variant library, then final-shading A/B at C2, C4f, C5 against the shipped library.
set -o pipefail
OUT=gpurun_out/r6s6
mkdir -p $OUT
export TMPDIR=/tmp
ROMIS_AMD_LIB=$PWD/romis_amd/_build/variants/occ_pf/libromis_amd.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "render_frame or miss_tiles or c1 or c2 or c4_c5 or vis" > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 21; }
tail -2 $OUT/parity.log
bash scripts/ab_libs_cfg.sh r6s6 c2 "--rounds 7 --frames 10" occ_pf || exit 22
bash scripts/ab_libs_cfg.sh r6s6 c4f "--rounds 5 --frames 3" occ_pf || exit 23
bash scripts/ab_libs_cfg.sh r6s6 c5 "--rounds 3 --frames 2" occ_pf || exit 24

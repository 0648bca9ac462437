#!/bin/bash
# Round 5 probe 31: final shading's shadow rays with their leaves tested in rounds (occluded_ww, ROMIS_FINAL_WW=1 build
# variant: lanes step inner nodes to their next hit leaf, then the wave tests all pending leaves at once) -- the GPU
# suite through the variant, then kbench / cfg_kbench against the shipped library.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p31
ROMIS_AMD_LIB=$REPO/romis_amd/_build/variants/fin_ww/libromis_amd.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 \
    --timeout-method thread tests -m gpu > gpurun_out/r5p31/tests.log 2>&1 || { tail -30 gpurun_out/r5p31/tests.log; exit 40; }
tail -2 gpurun_out/r5p31/tests.log
bash scripts/kbench_libs.sh r5p31/times "--only default --rounds 7 --frames 10" fin_ww || exit 41
bash scripts/kbench_libs.sh r5p31/times2 "--only default --rounds 7 --frames 10" fin_ww || exit 42
bash scripts/ab_libs_cfg.sh r5p31 c4f "--rounds 3 --frames 3" fin_ww || exit 43

#!/bin/bash
# Round 5 probe 20: the handle pass's window DMA offsets by steps instead of a division per entry (ROMIS_H_INC build
# variant) -- its handle parity tests, then kbench against the shipped library (interleaved, twice).
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p20
ROMIS_AMD_LIB=$REPO/romis_amd/_build/variants/h_inc/libromis_amd.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests/test_gpu_parity.py -k "handles or full_size_c2" -m gpu > gpurun_out/r5p20/tests.log 2>&1 \
    || { tail -30 gpurun_out/r5p20/tests.log; exit 40; }
tail -2 gpurun_out/r5p20/tests.log
bash scripts/kbench_libs.sh r5p20/times "--only default --rounds 9 --frames 10" h_inc || exit 41
bash scripts/kbench_libs.sh r5p20/times2 "--only default --rounds 9 --frames 10" h_inc || exit 42

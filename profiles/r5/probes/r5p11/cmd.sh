#!/bin/bash
# Round 5 probe 11: XCD chunk tail split evenly over the XCDs (ROMIS_XCD_BAL) -- spatial parity tests, then kbench
# A/B at C2 (handles, ntl) and C4f against the old whole-chunk tail (variant xcdold).
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p11
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py \
    -k "spatial or handles or render_frame or full_size_c2 or miss_tiles or tiles_stitch" > gpurun_out/r5p11/tests.log 2>&1 || { tail -40 gpurun_out/r5p11/tests.log; exit 40; }
tail -2 gpurun_out/r5p11/tests.log
bash scripts/kbench_libs.sh r5p11/times "--only default handles_off --rounds 9 --frames 10" xcdold prev || exit 41
bash scripts/kbench_libs.sh r5p11/times2 "--only default handles_off --rounds 9 --frames 10" xcdold prev || exit 42
for L in shipped xcdold; do
  LIB=$REPO/romis_amd/_build/libromis_amd.so; [ $L != shipped ] && LIB=$REPO/romis_amd/_build/variants/$L/libromis_amd.so
  ROMIS_AMD_LIB=$LIB timeout -k 10 300 python3 scripts/cfg_kbench.py --config c4f --rounds 3 --frames 3 > gpurun_out/r5p11/c4f_$L.json 2> gpurun_out/r5p11/c4f_$L.err || exit 43
  echo "c4f $L $(cat gpurun_out/r5p11/c4f_$L.json | tr -d '\n' | head -c 300)"
done

#!/bin/bash
# Round 5 probe 8: C4 / C5 full-size band parity on geometry bands (c4, c5, c4f, c5f: RGB + grid), the halo GPU tests,
# then bench lines of the framed configs.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p8
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_parity.py \
    -k "c4_c5_band" > gpurun_out/r5p8/tests.log 2>&1 || { tail -40 gpurun_out/r5p8/tests.log; exit 40; }
grep -E "PASS|FAIL" gpurun_out/r5p8/tests.log | tail -5
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_halo.py \
    > gpurun_out/r5p8/halo.log 2>&1 || { tail -40 gpurun_out/r5p8/halo.log; exit 41; }
tail -2 gpurun_out/r5p8/halo.log
for C in c4f c5f; do
  S=200; [ $C = c5f ] && S=30
  timeout -k 10 400 python3 bench.py --config $C --steps $S --warmup 10 --no-cpu-stages > gpurun_out/r5p8/bench_$C.json 2> gpurun_out/r5p8/bench_$C.err || { tail gpurun_out/r5p8/bench_$C.err; exit 42; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r5p8/bench_$C.json')); print('$C', d['ms_per_step'], d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], {k: v['us_per_launch'] for k, v in d['kernels'].items() if k != 'note'})"
done

#!/bin/bash
# Round 5 probe 10: the pruned build with the two-plane point-light table -- the whole GPU suite + smoke, kbench A/B
# against the committed 32-byte-record table (variant aos), then bench lines of the framed configs.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p10
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests -m gpu \
    > gpurun_out/r5p10/tests.log 2>&1 || { tail -40 gpurun_out/r5p10/tests.log; exit 40; }
tail -2 gpurun_out/r5p10/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 41
bash scripts/kbench_libs.sh r5p10/times "--only default --rounds 9 --frames 10" aos || exit 42
bash scripts/kbench_libs.sh r5p10/times2 "--only default --rounds 9 --frames 10" aos || exit 43
for C in c4f c5f; do
  S=200; [ $C = c5f ] && S=30
  timeout -k 10 400 python3 bench.py --config $C --steps $S --warmup 10 --no-cpu-stages > gpurun_out/r5p10/bench_$C.json 2> gpurun_out/r5p10/bench_$C.err || { tail gpurun_out/r5p10/bench_$C.err; exit 44; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r5p10/bench_$C.json')); print('$C', d['ms_per_step'], d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], {k: v['us_per_launch'] for k, v in d['kernels'].items() if k != 'note'})"
done

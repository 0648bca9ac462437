#!/bin/bash
# Round 6 s8: final.qbvh auto (N = 2) -- the GPU parity file and the driver-form C2 N = 2 bench.
set -o pipefail
OUT=gpurun_out/r6s8
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 21; }
tail -2 $OUT/parity.log
for rep in 1 2; do
timeout -k 10 200 python3 bench.py --N 2 --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c2_N2_$rep.json 2> $OUT/bench_c2_N2_$rep.err || { tail -5 $OUT/bench_c2_N2_$rep.err; exit 23; }
python3 -c "import json;d=json.loads(open('$OUT/bench_c2_N2_$rep.json').read().splitlines()[-1]);print('c2 N2',d['ms_per_step'])"
done

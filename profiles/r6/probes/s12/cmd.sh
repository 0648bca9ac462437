#!/bin/bash
# Round 6 s12: N = 2 temporal frames on handle records (C3 N = 2) -- temporal / C3 parity, then the C3 N = 2 bench.
set -o pipefail
OUT=gpurun_out/r6s12
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "temporal or c3 or odd_sizes or n2" > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 21; }
tail -2 $OUT/parity.log
timeout -k 10 300 python3 scripts/cfg_kbench.py --config c3 --N 2 --rounds 5 --frames 8 --variants h:spatial.n2h=1 r:spatial.n2h=0 > $OUT/c3_n2.json 2> $OUT/c3_n2.err || { tail -5 $OUT/c3_n2.err; exit 22; }
cat $OUT/c3_n2.json
for rep in 1 2; do
timeout -k 10 200 python3 bench.py --config c3 --N 2 --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c3_N2_$rep.json 2> $OUT/bench_c3_N2_$rep.err || { tail -5 $OUT/bench_c3_N2_$rep.err; exit 23; }
python3 -c "import json;d=json.loads(open('$OUT/bench_c3_N2_$rep.json').read().splitlines()[-1]);print('c3 N2',d['ms_per_step'])"
done

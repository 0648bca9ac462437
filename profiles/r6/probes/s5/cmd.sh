#!/bin/bash
# Round 6 s5: N = 2 handle records (k_spatial2hg[_t2]) -- parity, then cfg_kbench C2 / C3 at N = 2 and the driver-form C2 N = 2 bench.
set -o pipefail
OUT=gpurun_out/r6s5
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "n2_handles or miss_tiles or render_frame or N2 or n2" > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 21; }
tail -2 $OUT/parity.log
timeout -k 10 300 python3 scripts/cfg_kbench.py --config c2 --N 2 --rounds 7 --frames 10 --variants ntl:spatial.n2h=0 h1:spatial.n2h=1 h2:spatial.n2h=1,spatial.th=2 > $OUT/c2_n2.json 2> $OUT/c2_n2.err || { tail -20 $OUT/c2_n2.err; exit 22; }
cat $OUT/c2_n2.json
for V in 0 1; do
  timeout -k 10 200 python3 bench.py --N 2 --steps 200 --warmup 20 --no-cpu-baseline --tune spatial.n2h=$V > $OUT/bench_c2_N2_h$V.json 2> $OUT/bench_c2_N2_h$V.err || { tail -5 $OUT/bench_c2_N2_h$V.err; exit 23; }
  python3 -c "import json;d=json.loads(open('$OUT/bench_c2_N2_h$V.json').read().splitlines()[-1]);print('n2h$V',d['ms_per_step'],d['roofline']['achieved'])"
done

#!/bin/bash
# Round 6 s1: the sweeping handle pass (k_spatial1h_sw) -- its parity tests, then cfg_kbench C2 / C3 against k_spatial1h_t2.
set -o pipefail
OUT=gpurun_out/r6s1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k "handles" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 21; }
tail -2 $OUT/tests.log
V="t2:spatial.sweep=0 sw1:spatial.sweep=1 sw2:spatial.sweep=2 sw3:spatial.sweep=3 sw4:spatial.sweep=4 sw6:spatial.sweep=6 sw8:spatial.sweep=8"
timeout -k 10 300 python3 scripts/cfg_kbench.py --config c2 --rounds 5 --frames 10 --variants $V > $OUT/c2.json 2> $OUT/c2.err || { tail -20 $OUT/c2.err; exit 22; }
cat $OUT/c2.json
timeout -k 10 300 python3 scripts/cfg_kbench.py --config c3 --rounds 3 --frames 8 --variants t2:spatial.sweep=0 sw2:spatial.sweep=2 sw4:spatial.sweep=4 > $OUT/c3.json 2> $OUT/c3.err || { tail -20 $OUT/c3.err; exit 23; }
cat $OUT/c3.json

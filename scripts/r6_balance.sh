#!/bin/bash
# Round 6: uneven-layout halo tests on the GPU + the per-rank layout timing (profiles/r6/balance.json)
set -o pipefail
OUT=gpurun_out/r6_balance
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_halo.py -x -q --timeout 300 --timeout-method thread > $OUT/halo_tests.log 2>&1 || { tail -30 $OUT/halo_tests.log; exit 21; }
tail -2 $OUT/halo_tests.log
timeout -k 10 600 python3 scripts/balance_measure.py > $OUT/balance.json 2> $OUT/balance.err || { tail -20 $OUT/balance.err; exit 22; }
cat $OUT/balance.err

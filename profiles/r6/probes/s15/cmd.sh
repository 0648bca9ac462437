#!/bin/bash
# Round 6 s15: the fused primary + RIS kernel over a tile queue of persistent blocks (ris.queue) -- parity, then A/B.
set -o pipefail
OUT=gpurun_out/r6s15
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "ris_queue" > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 21; }
tail -2 $OUT/parity.log
for C in c2 c4 c4f; do
  R=7; F=10; [ $C = c4f ] && R=3 && F=3
  timeout -k 10 300 python3 scripts/cfg_kbench.py --config $C --rounds $R --frames $F --variants tile:ris.queue=0 queue:ris.queue=1 > $OUT/$C.json 2> $OUT/$C.err || { tail -5 $OUT/$C.err; exit 22; }
  cat $OUT/$C.json
done
timeout -k 10 300 python3 scripts/cfg_kbench.py --config c2 --N 2 --rounds 5 --frames 10 --variants tile:ris.queue=0 queue:ris.queue=1 > $OUT/c2_n2.json 2> $OUT/c2_n2.err || { tail -5 $OUT/c2_n2.err; exit 23; }
cat $OUT/c2_n2.json
timeout -k 10 300 python3 scripts/cfg_kbench.py --config c5 --rounds 3 --frames 2 --variants tile:ris.queue=0 queue:ris.queue=1 > $OUT/c5.json 2> $OUT/c5.err || { tail -5 $OUT/c5.err; exit 24; }
cat $OUT/c5.json

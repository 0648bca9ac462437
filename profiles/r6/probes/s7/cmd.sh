#!/bin/bash
# Round 6 s7: final shading's shadow rays over 16-byte quantized BVH nodes (k_final_n*_sorted_q, final.qbvh) -- the GPU
# parity file, then final-shading A/B at C2, C2 N = 2, C4f and C5.
set -o pipefail
OUT=gpurun_out/r6s7
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 21; }
tail -2 $OUT/parity.log
timeout -k 10 300 python3 scripts/cfg_kbench.py --config c2 --rounds 7 --frames 10 --variants q:final.qbvh=1 f:final.qbvh=0 > $OUT/c2.json 2> $OUT/c2.err || { tail -5 $OUT/c2.err; exit 22; }
cat $OUT/c2.json
timeout -k 10 300 python3 scripts/cfg_kbench.py --config c2 --N 2 --rounds 5 --frames 10 --variants q:final.qbvh=1 f:final.qbvh=0 > $OUT/c2_n2.json 2> $OUT/c2_n2.err || { tail -5 $OUT/c2_n2.err; exit 23; }
cat $OUT/c2_n2.json
timeout -k 10 300 python3 scripts/cfg_kbench.py --config c4f --rounds 5 --frames 3 --variants q:final.qbvh=1 f:final.qbvh=0 > $OUT/c4f.json 2> $OUT/c4f.err || { tail -5 $OUT/c4f.err; exit 24; }
cat $OUT/c4f.json

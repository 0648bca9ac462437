#!/bin/bash
# Round 6 s11: the unbiased pass's visibility rays over 16-byte quantized nodes (k_spatial1u_vis_q, spatial.qbvh) --
# miss-tile / frame parity, then C5 and C5f A/B.
set -o pipefail
OUT=gpurun_out/r6s11
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "miss_tiles or c4_c5 or render_frame" > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 21; }
tail -2 $OUT/parity.log
timeout -k 10 400 python3 scripts/cfg_kbench.py --config c5 --rounds 3 --frames 2 --variants f:spatial.qbvh=0 q:spatial.qbvh=1 > $OUT/c5.json 2> $OUT/c5.err || { tail -5 $OUT/c5.err; exit 22; }
cat $OUT/c5.json
timeout -k 10 400 python3 scripts/cfg_kbench.py --config c5f --rounds 2 --frames 1 --variants f:spatial.qbvh=0 q:spatial.qbvh=1 > $OUT/c5f.json 2> $OUT/c5f.err || { tail -5 $OUT/c5f.err; exit 23; }
cat $OUT/c5f.json

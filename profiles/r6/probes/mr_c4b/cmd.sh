#!/bin/bash
# Round 6 (mr_c4b): bench.py --config c4 / c5 at 8 ranks over gloo on one GPU after distributed.balanced_layout keeps
# the best measured of the cost-balanced 4 x 2 layout and its 3 refinements (halo frames over the torch transport, the
# halo self-check) -- the strong-scaling path end to end; mr_c4 is the same run before that change.
set -o pipefail
OUT=gpurun_out/mr_c4b
mkdir -p $OUT
export TMPDIR=/tmp
PORT=29653
for CFG in c4 c5; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
      --master-port $PORT bench.py --config $CFG --gpus 8 --dist-backend gloo --steps 10 --warmup 2 --no-cpu-baseline \
      > $OUT/${CFG}_n8.json 2> $OUT/${CFG}_n8.err || { tail -20 $OUT/${CFG}_n8.err; exit 31; }
  tail -c 1500 $OUT/${CFG}_n8.json
  PORT=$((PORT + 1))
done

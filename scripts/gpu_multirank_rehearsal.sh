#!/bin/bash
# Multi-rank bench rehearsal on one GPU (gloo process group, ranks share the card): bench.py --gpus N prints the
# halo self-check fields.   scripts/gpu_multirank_rehearsal.sh <tag> [N ...]
set -o pipefail
TAG=${1:-rehearsal}; shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO" || exit 1
export TMPDIR=/tmp
PORT=29533
# c2 (ghost zones + the halo self-check) at every N given; c5 (strong scaling: the unbiased + visibility pass over
# reservoir halos) at 2 ranks
RUNS=()
for N in "${@:-2 8}"; do RUNS+=("c2:$N"); done
RUNS+=("c5:2")
for R in "${RUNS[@]}"; do
    CFG=${R%%:*}; N=${R#*:}
    timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
        --master-port $PORT bench.py --config $CFG --gpus "$N" --dist-backend gloo --steps 10 --warmup 2 --no-cpu-baseline \
        > "$OUT/${CFG}_n$N.json" 2> "$OUT/${CFG}_n$N.err" || { tail -20 "$OUT/${CFG}_n$N.err"; exit 31; }
    cat "$OUT/${CFG}_n$N.json"
    PORT=$((PORT + 1))
done

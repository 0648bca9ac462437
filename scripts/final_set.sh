#!/bin/bash
# The end-of-session measurement set on one GPU: parity suite + smoke + default bench, the driver's own bench command
# (twice), every BASELINE config, the headline's rocprof kernel-trace/stats + PMC traffic passes, the spatial traffic
# study (C2, C4), an SQ pass for RIS's VALU count and the gloo multi-rank bench rehearsal.   scripts/final_set.sh <tag>
set -o pipefail
T=${1:-final}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
bash scripts/gpu_check.sh ${T}_check || exit $?
mkdir -p gpurun_out/${T}_driver
for rep in 1 2; do
    timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_driver/bench_$rep.json \
        2> gpurun_out/${T}_driver/bench_$rep.err || { tail -5 gpurun_out/${T}_driver/bench_$rep.err; exit 30; }
    cat gpurun_out/${T}_driver/bench_$rep.json
done
bash scripts/all_configs.sh ${T}_cfg && BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash scripts/gpu_profile.sh ${T}_prof \
    && bash scripts/traffic_study.sh ${T}_traffic \
    && bash scripts/pmc_passes.sh ${T}_valu "SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
    && python3 -c "from romis_amd import build; print(build.source_hash())" > gpurun_out/${T}_valu/source_hash.txt \
    && bash scripts/gpu_multirank_rehearsal.sh ${T}_mr 2 8

#!/bin/bash
# The end-of-session measurement set on one GPU, in two parts (each fits one gpurun call):
#   part a: parity suite + smoke + default bench, the driver's own bench command (twice), every BASELINE config;
#   part b: the headline's rocprof kernel-trace/stats + PMC traffic passes, the spatial traffic study (C2, C4, C4f, C5f),
#           an SQ pass for RIS's VALU count, the memory-pipeline / wait counters of the spatial pass over sample handles
#           against the n_t-window pass with reservoir gathers, and the gloo multi-rank bench rehearsal.
#   scripts/final_set.sh <tag> a|b
set -o pipefail
T=${1:-final}
PART=${2:-a}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
if [ "$PART" = a ]; then
    bash scripts/gpu_check.sh ${T}_check || exit $?
    mkdir -p gpurun_out/${T}_driver
    for rep in 1 2; do
        timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_driver/bench_$rep.json \
            2> gpurun_out/${T}_driver/bench_$rep.err || { tail -5 gpurun_out/${T}_driver/bench_$rep.err; exit 30; }
        cat gpurun_out/${T}_driver/bench_$rep.json
    done
    bash scripts/all_configs.sh ${T}_cfg
else
    BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash scripts/gpu_profile.sh ${T}_prof \
        && bash scripts/traffic_study.sh ${T}_traffic \
        && bash scripts/pmc_passes.sh ${T}_valu "SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
        && python3 -c "from romis_amd import build; print(build.source_hash())" > gpurun_out/${T}_valu/source_hash.txt \
        && bash scripts/pmc_kbench.sh ${T}_mempipe "--only default handles_off --rounds 1 --frames 3" \
            "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
            "TD_TD_BUSY_sum TD_TC_STALL_sum" \
            "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
            "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
            "FETCH_SIZE" \
        && bash scripts/gpu_multirank_rehearsal.sh ${T}_mr 2 8
fi

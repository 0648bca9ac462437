#!/bin/bash
# The end-of-session measurement set on one GPU: parity suite + smoke + default bench, every BASELINE config,
# the headline's rocprof kernel-trace/stats + PMC traffic passes, the spatial traffic study (C2, C4) and the
# gloo multi-rank bench rehearsal.   scripts/final_set.sh <tag>
set -o pipefail
T=${1:-final}
bash scripts/gpu_check.sh ${T}_check && bash scripts/all_configs.sh ${T}_cfg && bash scripts/gpu_profile.sh ${T}_prof \
    && bash scripts/traffic_study.sh ${T}_traffic && bash scripts/gpu_multirank_rehearsal.sh ${T}_mr 2 8

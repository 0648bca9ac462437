#!/bin/bash
# Round 5 probe 2: rocprofv3's PC-sampling configurations on gfx950, then one stochastic (cycles) PC-sampling run
# over the headline frame's kernels (hot spots and stall reasons of k_spatial1_ntl and k_primary_ris_n1_lds_pt).
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p2
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r5p2/list.txt 2>&1 || echo "list rc=$?"
grep -i -B2 -A12 "pc.sampl\|PC Sampling" gpurun_out/r5p2/list.txt | head -60
timeout -k 10 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
    --pc-sampling-interval 65536 --output-format csv -d gpurun_out/r5p2/pcs -o run -- \
    python3 scripts/kbench.py --only default --rounds 1 --frames 3 > gpurun_out/r5p2/pcs.json 2> gpurun_out/r5p2/pcs.err
echo "pcs rc=$?"
find gpurun_out/r5p2/pcs -type f | head; tail -5 gpurun_out/r5p2/pcs.err

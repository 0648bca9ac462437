#!/bin/bash
# Round 4: inter-kernel gaps by store type (scripts/probes/gap_probe2.hip) under a kernel trace.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4i
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- scripts/probes/_bin/gap_probe2 \
    > $OUT/gap_probe2.json 2> $OUT/gap_probe2.err || { tail -5 $OUT/gap_probe2.err; exit 21; }
cat $OUT/gap_probe2.json
python3 scripts/probes/gap2_analyze.py $OUT/trace/run_kernel_trace.csv | tee $OUT/gaps.json

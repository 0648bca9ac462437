#!/bin/bash
# Copy a scripts/final_set.sh run (gpurun_out/<tag>_*) into profiles/<dest>_* and regenerate profiles/traffic.json and
# profiles/valu.json from it (run here, after the GPU call).   scripts/collect_set.sh <tag> <dest, e.g. r4/s2>
set -e
T=$1; D=profiles/$2
G=gpurun_out
mkdir -p ${D}_check ${D}_driver ${D}_cfg ${D}_prof ${D}_mr ${D}_valu ${D}_mempipe
cp $G/${T}_check/{tests.log,smoke.log,bench.json} ${D}_check/
cp $G/${T}_driver/bench_*.json ${D}_driver/
cp $G/${T}_cfg/*.json ${D}_cfg/
cp $G/${T}_prof/{bench.json,trace_bench.json,source_hash.txt} ${D}_prof/
cp $G/${T}_prof/trace/run_kernel_stats.csv ${D}_prof/trace_kernel_stats.csv
cp $G/${T}_prof/pmc_fetch/run_counter_collection.csv ${D}_prof/pmc_fetch.csv
cp $G/${T}_prof/pmc_write/run_counter_collection.csv ${D}_prof/pmc_write.csv
python3 scripts/gap_analysis.py $G/${T}_prof/trace/run_kernel_trace.csv --warmup 5 --steps 20 > ${D}_prof/frames.json
cp $G/${T}_mr/*.json ${D}_mr/ 2>/dev/null || true
cp $G/${T}_valu/pmc0/run_counter_collection.csv ${D}_valu/sq_counter_collection.csv
cp $G/${T}_valu/pmc0.json $G/${T}_valu/source_hash.txt ${D}_valu/
python3 scripts/valu_json.py ${D}_valu > /dev/null
for i in 0 1 2 3 4; do
    cp $G/${T}_mempipe/pmc$i/run_counter_collection.csv ${D}_mempipe/pmc${i}_counter_collection.csv 2>/dev/null || true
done
python3 scripts/traffic_json.py ${T}_traffic --profile ${D}_traffic
echo "source hash now: $(python3 -c 'from romis_amd import build; print(build.source_hash())'), profiled: $(cat ${D}_prof/source_hash.txt)"

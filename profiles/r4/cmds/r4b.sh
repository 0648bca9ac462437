#!/bin/bash
# Round 4, second GPU call: bench start-up (GEMM pre-warm, sampled spatial events), the cross-lane spatial kernel
# study, and the cost of the keyed hash in RIS (variant libraries from scripts/budget_variants.py).
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4b
mkdir -p $OUT
B="python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
for rep in 1 2; do
  for v in "base:" "gemm100:--prewarm-gemm-ms 100" "gemm300:--prewarm-gemm-ms 300" "every4:--tune timing.every=4" \
           "every4_gemm100:--tune timing.every=4 --prewarm-gemm-ms 100"; do
    name=${v%%:*}; extra=${v#*:}
    timeout -k 10 240 $B $extra > "$OUT/${name}_$rep.json" 2> "$OUT/${name}_$rep.err" || { tail -5 "$OUT/${name}_$rep.err"; exit 11; }
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r4b/*.json")):
    d = json.load(open(f)); print(f.split("/")[-1], d["ms_per_step"], d["value"], d["roofline"]["avg_launch_us"], d["roofline"]["frac"])
PY
bash scripts/r4/x2_study.sh r4b_x2 || exit $?
bash scripts/kbench_libs.sh r4b_rng "--only default --rounds 5 --frames 10" ris_rng_weyl ris_rng_1mul ris_lidx_shift ris_no_rng || exit $?

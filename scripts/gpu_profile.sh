#!/bin/bash
# Profile the headline bench on the GPU box (run through gpurun from the repo root).
#   scripts/gpu_profile.sh <tag>
# Writes under gpurun_out/<tag>/: bench.json (plain run), the rocprofv3 kernel-trace + stats of the same
# command, and two separate --pmc passes (FETCH_SIZE, WRITE_SIZE: they do not fit one pass on gfx950).
set -o pipefail
TAG=${1:-prof}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$REPO" || exit 1
BENCH_ARGS=${BENCH_ARGS:-"--steps 50 --warmup 5"}

python3 -c "from romis_amd import build; print(build.source_hash())" > "$OUT/source_hash.txt" || exit 10
echo "[profile] plain bench" >&2
timeout -k 10 300 python3 bench.py $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 11
cat "$OUT/bench.json"

echo "[profile] kernel trace + stats" >&2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py $BENCH_ARGS --no-cpu-baseline > "$OUT/trace_bench.json" 2> "$OUT/trace.err" || exit 12

echo "[profile] pmc FETCH_SIZE" >&2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch_bench.json" 2> "$OUT/pmc_fetch.err" || exit 13

echo "[profile] pmc WRITE_SIZE" >&2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write_bench.json" 2> "$OUT/pmc_write.err" || exit 14

find "$OUT" -name '*.csv' | sort >&2
echo "[profile] done" >&2

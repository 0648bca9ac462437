#!/bin/bash
# GPU parity suite + smoke + default bench on the box (run through gpurun from the repo root).
#   scripts/gpu_check.sh <tag> [pytest -k expression]
# Writes gpurun_out/<tag>/{tests.log,smoke.log,bench.json}.  Stops at the first failing step.
set -o pipefail
TAG=${1:-check}
KEXPR=${2:-}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO" || exit 1
export TMPDIR=/tmp
if [ -n "$KEXPR" ]; then
    timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$KEXPR" > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 21; }
else
    timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 21; }
fi
tail -3 "$OUT/tests.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 22; }
cat "$OUT/smoke.log"
timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 23; }
cat "$OUT/bench.json"

#!/bin/bash
# Separate rocprofv3 --pmc passes over a short headline bench (one counter group per pass; gfx950 cannot
# fit them all at once).  Usage (on the GPU box, from the repo root): scripts/pmc_passes.sh <tag> "<group>" ...
# Writes gpurun_out/<tag>/pmc<i>/ per group.
set -o pipefail
TAG=$1; shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd "$REPO" || exit 1
mkdir -p "gpurun_out/$TAG"
i=0
for G in "$@"; do
    timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d "gpurun_out/$TAG/pmc$i" -o run -- \
        python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > "gpurun_out/$TAG/pmc$i.json" 2> "gpurun_out/$TAG/pmc$i.err" || exit $((20 + i))
    i=$((i + 1))
done

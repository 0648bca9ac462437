#!/bin/bash
# rocprofv3 --pmc passes over scripts/kbench.py (one counter group per pass; each pass its own process).
#   scripts/pmc_kbench.sh <tag> "<kbench args>" "<group>" ["<group>" ...]
# Writes gpurun_out/<tag>/pmc<i>/ per group.
set -o pipefail
TAG=$1; shift
KARGS=$1; shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd "$REPO" || exit 1
mkdir -p "gpurun_out/$TAG"
i=0
for G in "$@"; do
    timeout -s KILL 150 rocprofv3 --pmc $G --output-format csv -d "gpurun_out/$TAG/pmc$i" -o run -- \
        python3 scripts/kbench.py $KARGS > "gpurun_out/$TAG/pmc$i.json" 2> "gpurun_out/$TAG/pmc$i.err" || exit $((20 + i))
    i=$((i + 1))
done

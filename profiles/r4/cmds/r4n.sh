#!/bin/bash
# Round 4: RIS at 7 waves per SIMD (ROMIS_RIS1_WPE=7, 20 B spills) against the shipped 6, alternating libraries.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4n
mkdir -p $OUT
for rep in 1 2 3; do
    for c in c2 c5; do
        bash scripts/ab_libs_cfg.sh r4n/$rep $c "--rounds 3 --frames $([ $c = c5 ] && echo 3 || echo 10)" ris_w7 || exit 21
    done
done

#!/bin/bash
# Round 5 probe 25: what the neighbour reservoir gathers cost the N = 2 pass (C2 at N = 2, the reference default;
# k_spatial2_ntl): budget variant n2_no_gather against the shipped library.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
bash scripts/ab_libs_cfg.sh r5p25 c2 "--N 2 --rounds 5 --frames 10" n2_no_gather || exit 41

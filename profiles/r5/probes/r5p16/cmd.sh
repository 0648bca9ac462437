#!/bin/bash
# Round 5 probe 16: what the accepted neighbours' reservoir gathers cost the 4K pass on geometry (C4f,
# k_spatial1_ntl_t2): budget variants (scripts/budget_variants.py) half_gather (position / W only), no_gather, coalesced
# against the shipped library; C2's n_t-window pass (spatial.handles = 0) alongside.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
bash scripts/ab_libs_cfg.sh r5p16 c4f "--rounds 5 --frames 3" half_gather no_gather coalesced || exit 41
bash scripts/ab_libs_cfg.sh r5p16 c2 "--rounds 5 --frames 10 --variants ntl:spatial.handles=0" half_gather no_gather coalesced || exit 42

#!/bin/bash
# Round 5 probe 29: what final shading's pieces cost at C2 (k_final_n1_sorted) -- budget variants with the shadow rays,
# the shading, the tone map or the ray binning replaced by stand-ins (scripts/budget_variants.py; results change).
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
bash scripts/ab_libs_cfg.sh r5p29 c2 "--rounds 5 --frames 10" fin_no_trace fin_no_shade fin_no_tonemap fin_no_sort || exit 41

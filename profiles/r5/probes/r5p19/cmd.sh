#!/bin/bash
# Round 5 probe 19: RIS waves per SIMD for the light-grid form (k_primary_ris_n1_lds_reg, which now also writes the
# grid handle: 36 B of spills at 7 waves) -- C4f and C4 with the shipped 7 against 6 and 8 (build variants).
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
bash scripts/ab_libs_cfg.sh r5p19 c4f "--rounds 5 --frames 3" ris_w6 ris_w8 || exit 41
bash scripts/ab_libs_cfg.sh r5p19 c4 "--rounds 5 --frames 5" ris_w6 ris_w8 || exit 42

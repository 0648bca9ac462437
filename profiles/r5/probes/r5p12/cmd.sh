#!/bin/bash
# Round 5 probe 12: static wave priority in the handle pass (waves 4-7 or 0-3 at s_setprio 1 after the barrier) and
# RIS at 8 / 6 waves per SIMD -- kbench A/B against the shipped build (results are identical by construction).
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
bash scripts/kbench_libs.sh r5p12/times "--only default --rounds 9 --frames 10" prio_hi prio_lo ris_w8 ris_w6 || exit 41


#!/bin/bash
# Round 5 probe 32: the fused primary + RIS kernel's floor at C2 -- budget variants without the candidate loop
# (ris_no_cand: primary rays + stores) and with the candidates' target pdfs replaced (ris_no_phat).
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
bash scripts/ab_libs_cfg.sh r5p32 c2 "--rounds 5 --frames 10" ris_no_cand ris_no_phat || exit 41

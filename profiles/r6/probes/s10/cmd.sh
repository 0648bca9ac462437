#!/bin/bash
# Round 6 s10: N = 2 RIS register caps (ROMIS_RIS_WPE 4 / 6 against the shipped 5) at C2 N = 2 and C3 N = 2.
set -o pipefail
export TMPDIR=/tmp
bash scripts/ab_libs_cfg.sh r6s10 c2 "--N 2 --rounds 5 --frames 10" ris_w4 ris_w6 || exit 22
bash scripts/ab_libs_cfg.sh r6s10 c3 "--N 2 --rounds 3 --frames 8" ris_w4 ris_w6 || exit 23

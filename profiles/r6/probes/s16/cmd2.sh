#!/bin/bash
# Round 6 s16 (2): the max-ilp scheduling variant across the other configs.
set -o pipefail
export TMPDIR=/tmp
bash scripts/ab_libs_cfg.sh r6s16c c3 "--rounds 5 --frames 8" ilp || exit 22
bash scripts/ab_libs_cfg.sh r6s16c c2 "--N 2 --rounds 5 --frames 10" ilp || exit 23
bash scripts/ab_libs_cfg.sh r6s16c c4f "--rounds 3 --frames 3" ilp || exit 24
bash scripts/ab_libs_cfg.sh r6s16c c5 "--rounds 3 --frames 2" ilp || exit 25
bash scripts/ab_libs_cfg.sh r6s16d c2 "--rounds 7 --frames 10" ilp || exit 26

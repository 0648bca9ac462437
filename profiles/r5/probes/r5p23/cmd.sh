#!/bin/bash
# Round 5 probe 23: XCD balance of the handle pass's chunk order at C2 (68 tile rows of 32 x 16 in chunks of 2 over
# 8 XCDs: two XCDs own 5 chunks, six own 4) -- chunk heights 1 / 2 (default) / 4 and the chunks of odd rounds in
# reverse XCD order (ROMIS_XCD_SNAKE build variant).
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
bash scripts/kbench_libs.sh r5p23/times "--only default spatial_rows1 spatial_rows4 --rounds 7 --frames 10" snake || exit 41
bash scripts/kbench_libs.sh r5p23/times2 "--only default spatial_rows1 spatial_rows4 --rounds 7 --frames 10" snake || exit 42

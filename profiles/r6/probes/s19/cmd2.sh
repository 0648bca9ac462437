#!/bin/bash
# Round 6 s19 (2): k_spatial1hgg's XCD chunk height (spatial.xcd_rows 1 / 2 = auto / 4 / 8 rows of 32 x 8 tiles) at C2,
# and the pass at C3 (temporal frames, two passes over handles), against k_spatial1hg_t2.
set -o pipefail
O=gpurun_out/s19; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/cfg_kbench.py --config c2 --rounds 7 --frames 10 --variants default: \
    gall:spatial.gather=2 gall1:spatial.gather=2,spatial.xcd_rows=1 gall4:spatial.gather=2,spatial.xcd_rows=4 \
    gall8:spatial.gather=2,spatial.xcd_rows=8 > $O/c2_rows.json || exit 21
cat $O/c2_rows.json
timeout -k 10 300 python3 scripts/cfg_kbench.py --config c3 --rounds 5 --frames 8 --variants default: \
    gall:spatial.gather=2 > $O/c3.json || exit 22
cat $O/c3.json

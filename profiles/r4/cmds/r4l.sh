#!/bin/bash
# Round 4: background G-buffer store skip (miss.gbuf) -- parity, then C4 / C5 / C2 kernel times with it on and off.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4l
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "miss_tiles or render_frame_matches or c4_c5" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 20; }
tail -1 $OUT/tests.log
for c in c4 c5 c2; do
    timeout -k 10 300 python3 scripts/cfg_kbench.py --config $c --rounds 5 --frames $([ $c = c5 ] && echo 3 || echo 8) \
        --variants gbuf2:miss.gbuf=2 gbuf0:miss.gbuf=0 gbuf1:miss.gbuf=1 > $OUT/$c.json 2> $OUT/$c.err || { tail -5 $OUT/$c.err; exit 19; }
    cat $OUT/$c.json
done

#!/bin/bash
# Round 4, fourth GPU call: the fused primary + RIS kernel's work order (ris.order: natural = bottom tile row first,
# 1 = reversed) at C2 / C4 / C5, and frames in flight over several contexts (upper bound of frame overlap).
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4d
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "full_size_c2 or compact_light" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 21; }
tail -1 $OUT/tests.log
for c in c2 c4 c5; do
    timeout -k 10 300 python3 scripts/cfg_kbench.py --config $c --rounds 4 --frames $([ $c = c5 ] && echo 3 || echo 10) \
        --variants natural:ris.order=0 reversed:ris.order=1 > $OUT/kb_$c.json 2> $OUT/kb_$c.err || { tail -5 $OUT/kb_$c.err; exit 22; }
    cat $OUT/kb_$c.json
done
timeout -k 10 300 python3 scripts/inflight_probe.py > $OUT/inflight.json 2> $OUT/inflight.err || { tail -5 $OUT/inflight.err; exit 23; }
cat $OUT/inflight.json

#!/bin/bash
# Round 4: RIS N = 1 at 7 waves per SIMD as the default -- parity of the RIS kernels, then A/B against 6 (ris_w6) at
# C1 / C2 / C3 / C4, alternating.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4o
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
    timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
        -k "compact_light or render_frame_matches or full_size or c4_c5 or extreme or miss_tiles or ris" > $OUT/tests.log 2>&1 \
        || { tail -40 $OUT/tests.log; exit 20; }
    tail -1 $OUT/tests.log
fi
for rep in 1 2; do
    for c in c1 c2 c3 c4; do
        bash scripts/ab_libs_cfg.sh r4o/$rep $c "--rounds 3 --frames 10" ris_w6 || exit 21
    done
done

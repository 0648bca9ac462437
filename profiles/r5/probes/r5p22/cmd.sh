#!/bin/bash
# Round 5 probe 22: how the handle pass's time scales with the image (the fixed cost of a launch and its last
# partial round of blocks): kbench at 1920 x 540, 1920 x 1080, 1920 x 2160 and 3840 x 2160 (nightclub, C2 settings).
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p22
for S in 1920x540 1920x1080 1920x2160 3840x2160 1920x1080; do
    W=${S%x*}; H=${S#*x}
    timeout -k 10 200 python3 scripts/kbench.py --only default --rounds 5 --frames 10 --width $W --height $H \
        > gpurun_out/r5p22/k_$S.json 2> gpurun_out/r5p22/k_$S.err || { tail -5 gpurun_out/r5p22/k_$S.err; exit 41; }
    echo "$S $(python3 -c "import json; d=json.load(open('gpurun_out/r5p22/k_$S.json'))['default']; print(d)")"
done

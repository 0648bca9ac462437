#!/bin/bash
# Round 5 probe 5: k_spatial1h at 32 x 8/16/24/32 tiles -- handle parity tests, then kbench of every tile height.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p5
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "handles or render_frame or full_size_c2 or miss_tiles" > gpurun_out/r5p5/tests.log 2>&1 || { tail -40 gpurun_out/r5p5/tests.log; exit 40; }
tail -2 gpurun_out/r5p5/tests.log
timeout -k 10 400 python3 scripts/kbench.py --only default handles_off handles_t1 handles_t3 handles_t4 --rounds 7 --frames 10 \
    > gpurun_out/r5p5/kb.json 2> gpurun_out/r5p5/kb.err || { tail gpurun_out/r5p5/kb.err; exit 42; }
python3 -c "import json; d=json.load(open('gpurun_out/r5p5/kb.json')); print({k: v['spatial'] for k, v in d.items()})"

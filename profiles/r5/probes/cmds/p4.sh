#!/bin/bash
# Round 5 probe 4: k_spatial1h (sample handles in LDS) -- GPU parity suite (frame paths) + smoke, then kbench of the
# handle pass (32x8 and 32x16 tiles) against the n_t-window pass.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p4
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    > gpurun_out/r5p4/tests.log 2>&1 || { tail -40 gpurun_out/r5p4/tests.log; exit 40; }
tail -3 gpurun_out/r5p4/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 41
timeout -k 10 400 python3 scripts/kbench.py --only default handles_off handles_t2 ntl_t2 --rounds 7 --frames 10 \
    > gpurun_out/r5p4/kb.json 2> gpurun_out/r5p4/kb.err || { tail gpurun_out/r5p4/kb.err; exit 42; }
cat gpurun_out/r5p4/kb.json

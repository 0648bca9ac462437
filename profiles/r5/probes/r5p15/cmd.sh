#!/bin/bash
# Round 5 probe 15 (p13 with the light table in the binning arrays): final shading over the last handle pass's sample handles (k_final_n1h_sorted, the pass skipping its
# reservoir planes) -- the parity tests of the handle path, then kbench default against spatial.handles = 2.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p15
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "handles or c4_c5 or full_size or miss_tiles or smoke" -m gpu > gpurun_out/r5p15/tests.log 2>&1 \
    || { tail -30 gpurun_out/r5p15/tests.log; exit 40; }
tail -3 gpurun_out/r5p15/tests.log
for rep in 1 2; do
    timeout -k 10 300 python3 scripts/kbench.py --only default hfinal_off --rounds 9 --frames 10 \
        > gpurun_out/r5p15/kbench_$rep.json 2> gpurun_out/r5p15/kbench_$rep.err || { tail -5 gpurun_out/r5p15/kbench_$rep.err; exit 41; }
    python3 - gpurun_out/r5p15/kbench_$rep.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for v, r in d.items():
    print(v, r, "sum", round(sum(r.values()), 1))
PY
done


#!/bin/bash
# Round 5 probe 6: k_spatial1h with the material table in LDS and the heuristic's window reads batched -- handle parity,
# kbench A/B against the committed handle kernel (variant h1), SQ counters of k_spatial1h_t2 and k_spatial1_ntl.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p6
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "handles or render_frame or full_size_c2" > gpurun_out/r5p6/tests.log 2>&1 || { tail -40 gpurun_out/r5p6/tests.log; exit 40; }
tail -2 gpurun_out/r5p6/tests.log
bash scripts/kbench_libs.sh r5p6/times "--only default handles_off --rounds 7 --frames 10" h1 || exit 41
bash scripts/pmc_kbench.sh r5p6/sq "--only default handles_off --rounds 1 --frames 3" \
 "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
 "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LEVEL_WAVES SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES" || exit 42
python3 scripts/pmc_summary.py gpurun_out/r5p6/sq spatial > gpurun_out/r5p6/sq_summary.txt
cat gpurun_out/r5p6/sq_summary.txt

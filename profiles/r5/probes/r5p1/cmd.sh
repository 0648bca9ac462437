#!/bin/bash
# Round 5 probe 1: is the spatial pass load phase + compute in series?  kbench of the shipped library against the
# L2-resident-load variants (scripts/budget_variants.py l2res*), then two SQ counter passes over the shipped frame
# (RIS's non-VALU time).
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
bash scripts/kbench_libs.sh r5p1/times "--only default --rounds 5 --frames 10" no_gather skeleton l2res l2res_no_phat l2res_no_gather || exit 40
bash scripts/pmc_kbench.sh r5p1/sq "--only default --rounds 1 --frames 3" \
 "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
 "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_BUSY_CYCLES" || exit 41
python3 scripts/pmc_summary.py gpurun_out/r5p1/sq > gpurun_out/r5p1/sq_summary.txt

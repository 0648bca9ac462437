#!/bin/bash
# Vector-memory-pipeline and VALU counters of the frame kernels (TA / TD / TCP busy and stall cycles, SQ issue and
# wait), one rocprofv3 --pmc pass per group over scripts/kbench.py.  Summaries: profiles/r2/pmc_mempipe/.
#   scripts/pmc_mempipe.sh <tag> ["<kbench args>"]
TAG=${1:-mempipe}
KARGS=${2:-"--only default --rounds 1 --frames 3"}
bash scripts/pmc_kbench.sh "$TAG" "$KARGS" \
 "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
 "TD_TD_BUSY_sum TD_TC_STALL_sum" \
 "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
 "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_ANY" \
 "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VMEM_RD"

#!/bin/bash
# Round 6 s2: handle pass probes -- the sweep (k_spatial1h_sw) and gathered handles (k_spatial1hg_t2, 8 waves per SIMD):
# parity, cfg_kbench C2, then SQ counters of k_spatial1h_t2 / _sw / _hg (one kbench process per counter group).
set -o pipefail
OUT=gpurun_out/r6s2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k "handles" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 21; }
tail -2 $OUT/tests.log
timeout -k 10 300 python3 scripts/cfg_kbench.py --config c2 --rounds 7 --frames 10 --variants t2:spatial.sweep=0 hg:spatial.sweep=100 sw2:spatial.sweep=2 > $OUT/c2.json 2> $OUT/c2.err || { tail -20 $OUT/c2.err; exit 22; }
cat $OUT/c2.json
bash scripts/pmc_kbench.sh r6s2 "--rounds 1 --frames 5 --only default sweep2 hg" \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM GRBM_GUI_ACTIVE" || exit 23
python3 scripts/pmc_summary.py gpurun_out/r6s2 spatial > $OUT/sq_summary.txt && cat $OUT/sq_summary.txt

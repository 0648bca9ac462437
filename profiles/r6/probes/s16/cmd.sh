#!/bin/bash
# Round 6 s16: compiler scheduling strategies for kernels.hip (max-ilp, max-memory-clause, wave priority) -- a parity
# subset per variant, then C2 A/B twice (interleaved runs by ab_libs_cfg's order).
set -o pipefail
OUT=gpurun_out/r6s16
mkdir -p $OUT
export TMPDIR=/tmp
for V in ilp prio memclause; do
  ROMIS_AMD_LIB=$PWD/romis_amd/_build/variants/$V/libromis_amd.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "render_frame or handles_frames" > $OUT/parity_$V.log 2>&1 || { tail -20 $OUT/parity_$V.log; exit 21; }
  tail -1 $OUT/parity_$V.log
done
bash scripts/ab_libs_cfg.sh r6s16 c2 "--rounds 5 --frames 10" ilp prio memclause || exit 22
bash scripts/ab_libs_cfg.sh r6s16b c2 "--rounds 5 --frames 10" ilp prio memclause || exit 23

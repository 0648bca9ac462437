#!/bin/bash
# Round 4, third GPU call: the full GPU suite (RIS keeps the accepted candidate's index, the exact positive-p-hat
# test in the unbiased Z loops, pruned spatial variants), RIS at 6 waves per SIMD and the grid-light no-load bound
# (variant libraries), and the bench with the GEMM clock pre-warm.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4c
mkdir -p $OUT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 \
    || { tail -40 $OUT/tests.log; exit 21; }
tail -3 $OUT/tests.log
for c in c2 c4 c5; do
  for lib in shipped ris_wpe6; do
    if [ $lib = shipped ]; then unset ROMIS_AMD_LIB; else export ROMIS_AMD_LIB="$REPO/romis_amd/_build/variants/$lib/libromis_amd.so"; fi
    timeout -k 10 300 python3 scripts/cfg_kbench.py --config $c --rounds 3 --frames $([ $c = c5 ] && echo 3 || echo 10) \
        --variants default: gridtable:ris.compact=2 > $OUT/kb_${c}_$lib.json 2> $OUT/kb_${c}_$lib.err || { tail -5 $OUT/kb_${c}_$lib.err; exit 22; }
    echo "$c $lib $(cat $OUT/kb_${c}_$lib.json)"
  done
done
unset ROMIS_AMD_LIB
for rep in 1 2; do
  for v in "base:" "gemm500:--prewarm-gemm-ms 500"; do
    name=${v%%:*}; extra=${v#*:}
    timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline $extra > "$OUT/${name}_$rep.json" 2> "$OUT/${name}_$rep.err" || { tail -5 "$OUT/${name}_$rep.err"; exit 11; }
    python3 -c "import json; d=json.load(open('$OUT/${name}_$rep.json')); print('$name', d['ms_per_step'], d['value'], d['roofline']['avg_launch_us'])"
  done
done

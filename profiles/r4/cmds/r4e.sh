#!/bin/bash
# Round 4, fifth GPU call: frames in flight (frames.inflight = 2) -- parity, then the driver's bench command with
# and without it, and a kernel trace of the pipelined bench (the spatial pass must run alone).
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4e
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_halo.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -k "in_flight or full_size_c2 or c3_sequence or record_only or stitch or unbiased or c4_c5 or extreme or render_frame_matches" > $OUT/tests.log 2>&1 \
    || { tail -30 $OUT/tests.log; exit 21; }
tail -1 $OUT/tests.log
for rep in 1 2; do
  for v in "serial:--inflight 1" "inflight2:--inflight 2"; do
    name=${v%%:*}; extra=${v#*:}
    timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline $extra > "$OUT/${name}_$rep.json" 2> "$OUT/${name}_$rep.err" || { tail -5 "$OUT/${name}_$rep.err"; exit 11; }
    python3 -c "import json; d=json.load(open('$OUT/${name}_$rep.json')); print('$name', d['ms_per_step'], d['value'], d['roofline']['avg_launch_us'], d['kernels']['primary_ris']['us_per_launch'])"
  done
done
for c in c3 c4; do
  timeout -k 10 240 python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/${c}_inflight2.json" 2> "$OUT/${c}.err" || { tail -5 "$OUT/${c}.err"; exit 12; }
  timeout -k 10 240 python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --inflight 1 > "$OUT/${c}_serial.json" 2> "$OUT/${c}s.err" || { tail -5 "$OUT/${c}s.err"; exit 12; }
  python3 -c "import json; a=json.load(open('$OUT/${c}_serial.json')); b=json.load(open('$OUT/${c}_inflight2.json')); print('$c', a['ms_per_step'], b['ms_per_step'])"
done
timeout -k 10 300 python3 scripts/cfg_kbench.py --config c5 --rounds 3 --frames 3 --variants default: > $OUT/kb_c5.json 2> $OUT/kb_c5.err || { tail -5 $OUT/kb_c5.err; exit 14; }
cat $OUT/kb_c5.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 bench.py --gpus 1 --steps 20 \
    --warmup 5 --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace.err || { tail -5 $OUT/trace.err; exit 13; }
python3 scripts/gap_analysis.py $OUT/trace/run_kernel_trace.csv --warmup 5 --steps 20 > $OUT/frames.json

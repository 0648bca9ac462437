#!/bin/bash
# Round 5 probe 37: a context's own predecessor frame needs no event wait / read event / pool wait (same stream) --
# the whole GPU suite, then C3's bench line and kernel trace (the in-frame gaps after the temporal kernel).
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
OUT=$REPO/gpurun_out/r5p37
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 \
    || { tail -30 "$OUT/tests.log"; exit 40; }
tail -2 "$OUT/tests.log"
timeout -k 10 240 python3 bench.py --config c3 --steps 200 --warmup 20 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" \
    || { tail -5 "$OUT/bench_c3.err"; exit 41; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c3" -o run -- \
    python3 bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c3_bench.json" 2> "$OUT/c3.err" || exit 42
python3 scripts/gap_analysis.py "$OUT/c3/run_kernel_trace.csv" --warmup 5 --steps 20 > "$OUT/c3_frames.json" || exit 43
python3 -c "import json;d=json.loads(open('$OUT/bench_c3.json').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['value']);t=json.load(open('$OUT/c3_frames.json'))['timed'];print(t['wall_us_per_frame_first_start_to_last_end'],t['kernel_sum_us'],t['in_frame_gaps_us'],t['between_frames_us'])"

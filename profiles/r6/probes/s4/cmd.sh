#!/bin/bash
# Round 6 s4: the gathered-handle default (k_spatial1hg_t2) through the parity tests that cover the handle passes, the miss
# tiles (ghost tiles now against the oracle) and the full-size balanced C4 / C5 splits; then C4f tile orders, 7 rounds.
set -o pipefail
OUT=gpurun_out/r6s4
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "handles or miss_tiles or temporal_sequence or c2 or c3" > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 21; }
tail -2 $OUT/parity.log
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_halo.py -x -v --timeout 600 --timeout-method thread -k "full_size" > $OUT/halo.log 2>&1 || { tail -30 $OUT/halo.log; exit 22; }
tail -3 $OUT/halo.log
VARS="r1:spatial.xcd_rows=255 c4x8:spatial.xcd_rows=4,spatial.xcd_cols=8 c2x8:spatial.xcd_rows=2,spatial.xcd_cols=8 c2x4:spatial.xcd_rows=2,spatial.xcd_cols=4 c4x4:spatial.xcd_rows=4,spatial.xcd_cols=4"
timeout -k 10 400 python3 scripts/cfg_kbench.py --config c4f --rounds 7 --frames 3 --variants $VARS > $OUT/c4f_times.json 2> $OUT/c4f_times.err || { tail -5 $OUT/c4f_times.err; exit 23; }
cat $OUT/c4f_times.json
for V in $VARS; do
  N=${V%%:*}
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/c4f_${N}_$C -o run -- python3 scripts/cfg_kbench.py --config c4f --rounds 1 --frames 3 --variants "$V" > $OUT/c4f_${N}_$C.json 2> $OUT/c4f_${N}_$C.err || exit 24
  done
done
python3 - <<'PY'
import csv, glob
for f in sorted(glob.glob("gpurun_out/r6s4/c4f_*_*_SIZE/run_counter_collection.csv")):
    rows=[r for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith("k_spatial")]
    c=rows[0]["Counter_Name"]; v=[float(r["Counter_Value"]) for r in rows if r["Counter_Name"]==c]
    mb=sum(v)/len(v)*1024/1e6*(2 if c=="FETCH_SIZE" else 1)
    print(f.split("/")[2], c, "MB/launch (FETCH doubled)", round(mb,1))
PY

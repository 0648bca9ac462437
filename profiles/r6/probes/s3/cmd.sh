#!/bin/bash
# Round 6 s3: (a) C2 driver-form bench, handle windows in LDS vs gathered handles (spatial.gather);
# (b) C4f spatial pass (k_spatial1g_t2) under XCD tile orders -- time and FETCH_SIZE;
# (c) SQ counters of final shading at C2 and C4f.
set -o pipefail
OUT=gpurun_out/r6s3
mkdir -p $OUT
export TMPDIR=/tmp
for V in 0 1; do
  timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --tune spatial.gather=$V > $OUT/bench_c2_gather$V.json 2> $OUT/bench_c2_gather$V.err || { tail -5 $OUT/bench_c2_gather$V.err; exit 21; }
  python3 -c "import json;d=json.loads(open('$OUT/bench_c2_gather$V.json').read().splitlines()[-1]);print('gather$V',d['ms_per_step'],d['roofline']['achieved'],d['roofline']['frac'])"
done
VARS="r1:spatial.xcd_rows=255 r2:spatial.xcd_rows=2 r4:spatial.xcd_rows=4 band:spatial.xcd_rows=0 c4x15:spatial.xcd_rows=4,spatial.xcd_cols=15 c8x15:spatial.xcd_rows=8,spatial.xcd_cols=15 c4x8:spatial.xcd_rows=4,spatial.xcd_cols=8"
timeout -k 10 400 python3 scripts/cfg_kbench.py --config c4f --rounds 5 --frames 3 --variants $VARS > $OUT/c4f_times.json 2> $OUT/c4f_times.err || { tail -5 $OUT/c4f_times.err; exit 22; }
cat $OUT/c4f_times.json
for V in $VARS; do
  N=${V%%:*}
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c4f_${N}_FETCH -o run -- python3 scripts/cfg_kbench.py --config c4f --rounds 1 --frames 3 --variants "$V" > $OUT/c4f_${N}_FETCH.json 2> $OUT/c4f_${N}_FETCH.err || exit 23
done
for C in c2 c4f; do
  i=0; mkdir -p $OUT/final_$C
  for G in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d $OUT/final_$C/pmc$i -o run -- python3 scripts/cfg_kbench.py --config $C --rounds 1 --frames 3 > $OUT/final_$C/pmc$i.json 2> $OUT/final_$C/pmc$i.err || exit 24
    i=$((i + 1))
  done
  python3 scripts/pmc_summary.py $OUT/final_$C k_final k_spatial k_primary > $OUT/final_$C/sq_summary.txt && cat $OUT/final_$C/sq_summary.txt
done
python3 - <<'PY'
import csv, glob
for f in sorted(glob.glob("gpurun_out/r6s3/c4f_*_FETCH/run_counter_collection.csv")):
    v=[float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith("k_spatial") and r["Counter_Name"]=="FETCH_SIZE"]
    print(f.split("/")[2], "FETCH_SIZE KiB/launch", round(sum(v)/len(v)), "x2 MB", round(2*sum(v)/len(v)*1024/1e6,1))
PY

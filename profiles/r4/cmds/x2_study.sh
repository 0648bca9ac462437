#!/bin/bash
# Round 4: the cross-lane WRS spatial kernel (k_spatial1_x2, spatial.lds = 4) against k_spatial1_ntl (spatial.lds = 3):
# parity, kernel times at C2 / C4 (cfg_kbench, interleaved, RGB must match), and SQ cycle counters of both.
#   scripts/r4/x2_study.sh <tag>
set -o pipefail
TAG=${1:-x2}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$REPO" || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "x2" > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 21; }
tail -2 "$OUT/tests.log"
for c in c2 c4; do
    timeout -k 10 300 python3 scripts/cfg_kbench.py --config $c --rounds 5 --frames 10 \
        --variants ntl:spatial.lds=3,spatial.th=1 x2:spatial.lds=4,spatial.th=1 > "$OUT/kb_$c.json" 2> "$OUT/kb_$c.err" \
        || { tail -5 "$OUT/kb_$c.err"; exit 22; }
    cat "$OUT/kb_$c.json"
done
i=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" \
         "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD"; do
    for v in "ntl:spatial.lds=3,spatial.th=1" "x2:spatial.lds=4,spatial.th=1"; do
        name=${v%%:*}
        timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d "$OUT/pmc${i}_$name" -o run -- \
            python3 scripts/cfg_kbench.py --config c2 --rounds 1 --frames 5 --variants "$v" \
            > "$OUT/pmc${i}_$name.json" 2> "$OUT/pmc${i}_$name.err" || { tail -5 "$OUT/pmc${i}_$name.err"; exit 23; }
    done
    i=$((i + 1))
done
echo "[x2] done" >&2

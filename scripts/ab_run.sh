set -o pipefail
O=gpurun_out/${1:-ab}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 21; }
tail -2 $O/tests.log
timeout -k 10 300 python3 scripts/cfg_kbench.py --config c2 --rounds 7 --frames 10 --variants compact:ris.compact=1 general:ris.compact=0 > $O/kb_c2.json || exit 22
cat $O/kb_c2.json
timeout -k 10 300 python3 scripts/cfg_kbench.py --config c2 --N 2 --rounds 5 --frames 10 --variants compact:ris.compact=1 general:ris.compact=0 > $O/kb_c2n2.json || exit 23
cat $O/kb_c2n2.json
for C in c4 c5; do
  R=5; [ $C = c5 ] && R=3
  timeout -k 10 300 python3 scripts/cfg_kbench.py --config $C --rounds $R --frames 5 --variants compact:ris.compact=1 general:ris.compact=0 > $O/kb_$C.json || exit 24
  cat $O/kb_$C.json
done

#!/bin/bash
# Run scripts/kbench.py against the shipped library and each named variant library (_build/variants/<name>).
#   scripts/kbench_libs.sh <tag> "<kbench args>" <variant> ...
set -o pipefail
TAG=$1; shift
KARGS=$1; shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
mkdir -p "gpurun_out/$TAG"
timeout -k 10 200 python3 scripts/kbench.py $KARGS > "gpurun_out/$TAG/shipped.json" 2> "gpurun_out/$TAG/shipped.err" || exit 30
for V in "$@"; do
    ROMIS_AMD_LIB="$REPO/romis_amd/_build/variants/$V/libromis_amd.so" timeout -k 10 200 python3 scripts/kbench.py $KARGS \
        > "gpurun_out/$TAG/$V.json" 2> "gpurun_out/$TAG/$V.err" || exit 31
done
python3 - "$REPO/gpurun_out/$TAG" <<'PY'
import json, glob, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.load(open(f))
    print(os.path.basename(f)[:-5].ljust(12), "  ".join(f"{k}:{v.get('spatial')}/{v.get('primary_ris')}/{v.get('final')}" for k, v in d.items()))
PY

#!/bin/bash
# Round 4, first GPU call: the gap study (scripts/r4/gap_study.sh), then the new / changed GPU tests.
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO" || exit 1
export TMPDIR=/tmp
bash scripts/r4/gap_study.sh gap || exit $?
mkdir -p gpurun_out/r4a
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_halo.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "record_only or halo_frames_match or c2_frame_band" > gpurun_out/r4a/tests.log 2>&1
rc=$?
tail -30 gpurun_out/r4a/tests.log
exit $rc

#!/bin/bash
# Round 6 s19: k_spatial1hgg (spatial.gather = 2) at 6 waves per SIMD without spills, 32 x 8 tiles (shipped build) and
# 32 x 16 tiles (build variant hgg_t2), against the gathered-handle pass k_spatial1hg_t2 (default), C2 and C4f.
set -o pipefail
O=gpurun_out/s19; mkdir -p $O; export TMPDIR=/tmp
for V in shipped hgg_t2; do
    LIB=romis_amd/_build/libromis_amd.so
    [ "$V" != shipped ] && LIB=romis_amd/_build/variants/$V/libromis_amd.so
    ROMIS_AMD_LIB=$PWD/$LIB timeout -k 10 300 python3 scripts/cfg_kbench.py --config c2 --rounds 9 --frames 10 \
        --variants default: gall:spatial.gather=2 > $O/c2_$V.json || exit 21
    echo "$V $(cat $O/c2_$V.json)"
done

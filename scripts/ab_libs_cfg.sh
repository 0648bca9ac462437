#!/bin/bash
# cfg_kbench of one config against the shipped library and build variants (scripts/define_variants.py):
#   scripts/ab_libs_cfg.sh <tag> <config> "<cfg_kbench args>" <variant> ...
set -o pipefail
TAG=$1; CFG=$2; KARGS=$3; shift 3
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
for V in shipped "$@"; do
    LIB=romis_amd/_build/libromis_amd.so
    [ "$V" != shipped ] && LIB=romis_amd/_build/variants/$V/libromis_amd.so
    ROMIS_AMD_LIB=$PWD/$LIB timeout -k 10 300 python3 scripts/cfg_kbench.py --config $CFG $KARGS > $O/${CFG}_$V.json || exit 40
    echo "$V $(cat $O/${CFG}_$V.json)"
done

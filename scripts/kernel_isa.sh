#!/bin/bash
# Disassemble one kernel of the built gfx950 code object: scripts/kernel_isa.sh <kernel> [object]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
K=$1
OBJ=${2:-$ROOT/romis_amd/_build/kernels.hip.o}
TMP=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section .hip_fatbin="$TMP/fb.bin" "$OBJ"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --type=o --input="$TMP/fb.bin" --output="$TMP/k.hsaco" \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --unbundle
/opt/rocm/lib/llvm/bin/llvm-objdump -d --no-show-raw-insn --disassemble-symbols="$K" "$TMP/k.hsaco" | tail -n +7
rm -rf "$TMP"

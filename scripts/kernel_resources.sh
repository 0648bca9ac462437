#!/bin/bash
# Per-kernel VGPR / SGPR / scratch / LDS of the built gfx950 code object (romis_amd/_build/kernels.hip.o).
#   scripts/kernel_resources.sh [kernel-name-regex]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OBJ=${OBJ:-$ROOT/romis_amd/_build/kernels.hip.o}
TMP=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section .hip_fatbin="$TMP/fb.bin" "$OBJ"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --type=o --input="$TMP/fb.bin" --output="$TMP/k.hsaco" \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --unbundle
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$TMP/k.hsaco" | python3 -c '
import sys, re
pat = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
txt = sys.stdin.read()
for blk in txt.split("  - .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if pat and not pat.search(name): continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
    print("%-40s vgpr %4s sgpr %4s scratch %5s lds %6s" % (name, g("vgpr_count"), g("sgpr_count"),
          g("private_segment_fixed_size"), g("group_segment_fixed_size")))
' "$@"
rm -rf "$TMP"

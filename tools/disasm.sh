#!/bin/bash
# Disassemble the gfx950 code object of one built object file (development aid).
# Usage: tools/disasm.sh <object.o> <out.s>
set -euo pipefail
B=/opt/rocm/lib/llvm/bin
t=$(mktemp -d)
$B/llvm-objcopy -O binary --only-section=.hip_fatbin "$1" "$t/fat"
$B/clang-offload-bundler --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input="$t/fat" --output="$t/co"
$B/llvm-objdump -d "$t/co" > "$2"
rm -rf "$t"

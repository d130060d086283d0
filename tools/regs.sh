#!/bin/bash
# Register / scratch usage of every kernel in one HIP source (development aid).
# Usage: tools/regs.sh <file.hip> [name-filter]
set -euo pipefail
src=$(realpath "$1"); filt=${2:-.}
d=$(mktemp -d)
(cd "$d" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -c "$src" -o x.o -save-temps 2>/dev/null)
awk '/^[ \t]+\.name:/{n=$2} /\.private_segment_fixed_size:/{p=$2} /\.sgpr_count:/{s=$2} /\.vgpr_count:/{v=$2} /\.vgpr_spill_count:/{print n, "vgpr", v, "sgpr", s, "scratch", p, "spill", $2}' "$d"/*gfx950*.s | grep -E "$filt" || true
rm -rf "$d"

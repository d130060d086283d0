# A/B of two library builds on one box: bash tools/_ab/ab_lib.sh <out> <rounds> <bench args...>
set -o pipefail
OUT=$1; R=$2; shift 2
mkdir -p "$(dirname "$OUT")"
LIB=reed-solomon-simd_amd/lib/librs_mi355x.so
for ((i = 0; i < R; ++i)); do
  for v in A B; do
    cp tools/_ab/lib$v.so $LIB
    line=$(timeout -k 10 300 python -u bench.py "$@" 2>/dev/null | tail -1) || { echo "$v failed"; exit 1; }
    echo "$v $(echo "$line" | python -c "
import json,sys
d=json.loads(sys.stdin.read())
print(d['value'], d.get('decode_GiBps') and (d['decode_GiBps'].get('1pct'), d['decode_GiBps'].get('100pct')))
")"
  done
done | tee "$OUT"
cp tools/_ab/libA.so $LIB

#!/bin/bash
# A/B of library variants on the large configs: for each variant name (main = the in-tree
# build, else lib/variants/librs_mi355x_<name>.so) the pass-path GPU tests, then the
# config 3/4/5 bench lines, under gpurun_out/<tag>/<variant>/.
#   bash tools/ab_variant.sh <tag> main lr4 ...
set -euo pipefail
source "$(dirname "$0")/ab_common.sh"
TAG=$1; shift
for v in "$@"; do
  O=gpurun_out/$TAG/$v; mkdir -p $O
  use_lib $v
  timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu \
    -k "streaming or config5 or config4 or baseline_decode_8192 or pass_path or loss_patterns" > $O/tests.log 2>&1
  timeout -k 10 200 python -u bench.py --no-cpu --no-host --no-copy --batch 1 --config 32768x32768x64k --steps 10 --warmup 2 > $O/c5.json 2>>$O/err.log
  timeout -k 10 200 python -u bench.py --no-cpu --no-host --no-copy --batch 1 --config 8192x8192x64k --steps 10 --warmup 2 > $O/c4.json 2>>$O/err.log
  timeout -k 10 200 python -u bench.py --no-cpu --no-host --no-copy --batch 1 --config 32768x32768x1k --steps 30 --warmup 3 > $O/c3.json 2>>$O/err.log
done

#!/bin/bash
# A/B helper: GPU tests of the large-config paths and the config 3/4/5 bench lines
# (tag in $1), e.g. bash tools/ab_stream.sh r02s
set -euo pipefail
O=gpurun_out/${1:-ab}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "streaming or config5 or config4 or baseline_decode_8192 or two_streams or pass_path" > $O/tests.log 2>&1
timeout -k 10 200 python -u bench.py --no-cpu --no-host --no-copy --config 32768x32768x64k --steps 10 --warmup 2 > $O/c5.json 2>>$O/err.log
timeout -k 10 200 python -u bench.py --no-cpu --no-host --no-copy --config 8192x8192x64k --steps 10 --warmup 2 > $O/c4.json 2>>$O/err.log
timeout -k 10 200 python -u bench.py --no-cpu --no-host --no-copy --config 32768x32768x1k --steps 30 --warmup 3 > $O/c3.json 2>>$O/err.log

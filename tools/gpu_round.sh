#!/bin/bash
# One GPU-box session: parity tests, bench line, rocprofv3 kernel-trace summary
# and the two HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs).
# Usage (from the repo root, on the box):  bash tools/gpu_round.sh <tag> [pytest-args...]
# Every GPU step has its own time limit; the script stops at the first failure.
set -euo pipefail
TAG=${1:-r01}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "$@" \
    > "$OUT/pytest_gpu.log" 2>&1
  tail -3 "$OUT/pytest_gpu.log"
fi

timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"

BENCH="bench.py --no-cpu --no-host --steps 200 --warmup 20"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/kt" -o run -- python3 $BENCH \
  > "$OUT/kt.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/pmc_fetch" -o run -- python3 $BENCH \
  > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/pmc_write" -o run -- python3 $BENCH \
  > "$OUT/pmc_write.log" 2>&1
if [ "${CONFIGS:-0}" = "1" ]; then  # the other single-GPU BASELINE configs
  timeout -k 10 300 python -u bench.py --no-cpu --config 32768x32768x1k --steps 50 --warmup 5 \
    > "$OUT/bench_config3.json" 2>> "$OUT/bench.err"
  timeout -k 10 300 python -u bench.py --no-cpu --config 8192x8192x64k --steps 10 --warmup 2 \
    > "$OUT/bench_config4.json" 2>> "$OUT/bench.err"
  timeout -k 10 300 python -u bench.py --config 32768x32768x64k --steps 10 --warmup 2 \
    > "$OUT/bench_config5_n1.json" 2>> "$OUT/bench.err"
fi
echo "gpu_round $TAG done"

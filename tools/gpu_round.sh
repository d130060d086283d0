#!/bin/bash
# One GPU-box session: parity tests, bench lines, rocprofv3 kernel-trace
# summaries and the PMC passes (FETCH_SIZE, WRITE_SIZE, SQ counters -- each in
# its own run) per bench config.
# Usage (from the repo root, on the box):  bash tools/gpu_round.sh <tag> [pytest-args...]
#   SKIP_TESTS=1   skip the GPU test suite
#   CONFIGS=1      also the other single-GPU BASELINE configs (3, 4, 5 at N = 1)
#   SHAPES=1       also the reference README's shape table (bench.py --shape-table)
# Every GPU step has its own time limit; the script stops at the first failure.
set -euo pipefail
TAG=${1:-r02}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
    > "$OUT/pytest_gpu.log" 2>&1
  tail -3 "$OUT/pytest_gpu.log"
fi

timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"

# profile one bench command: kernel trace + 3 PMC passes (separate runs)
profile() {  # profile <config-name> <bench args...>
  local cfg=$1
  shift
  local d="$OUT/pmc/$cfg"
  mkdir -p "$d" "$OUT/kt"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/kt/$cfg" -o run -- python3 bench.py "$@" \
    > "$OUT/kt_$cfg.log" 2>&1
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -f csv -d "$d/fetch" -o run -- python3 bench.py "$@" \
    > "$d/fetch.log" 2>&1
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -f csv -d "$d/write" -o run -- python3 bench.py "$@" \
    > "$d/write.log" 2>&1
  timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES \
    SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_WAVE_CYCLES -f csv -d "$d/sq" -o run -- python3 bench.py "$@" \
    > "$d/sq.log" 2>&1
  echo "profiled $cfg"
}

profile 1024x1024x1k --no-cpu --no-host --no-copy --no-sharded --no-configs --batch 1 --steps 200 --warmup 20
if [ "${CONFIGS:-0}" = "1" ]; then  # the other single-GPU BASELINE configs
  timeout -k 10 300 python -u bench.py --no-cpu --config 32768x32768x1k --steps 50 --warmup 5 \
    > "$OUT/bench_config3.json" 2>> "$OUT/bench.err"
  timeout -k 10 300 python -u bench.py --no-cpu --config 8192x8192x64k --steps 10 --warmup 2 \
    > "$OUT/bench_config4.json" 2>> "$OUT/bench.err"
  timeout -k 10 300 python -u bench.py --config 32768x32768x64k --steps 10 --warmup 2 --cpu-seconds 5 \
    > "$OUT/bench_config5_n1.json" 2>> "$OUT/bench.err"
  profile 32768x32768x1k --no-cpu --no-host --no-copy --batch 1 --config 32768x32768x1k --steps 20 --warmup 3
  profile 8192x8192x64k --no-cpu --no-host --no-copy --batch 1 --config 8192x8192x64k --steps 5 --warmup 2
  profile 32768x32768x64k --no-cpu --config 32768x32768x64k --steps 5 --warmup 2 --profile-steps 30
fi
if [ "${SHAPES:-0}" = "1" ]; then  # the reference README's shape table
  timeout -k 10 300 python -u bench.py --shape-table --steps 50 > "$OUT/shape_table.json" 2>> "$OUT/bench.err"
fi
echo "gpu_round $TAG done"

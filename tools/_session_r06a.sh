# r06a: the half-split race demonstration, the LDS-multiply probe, the GPU suite, the bench line
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06a
timeout -k 10 120 tools/probe_bin/lds_mul_probe 200 > gpurun_out/r06a/lds_mul_probe.txt 2>&1 || exit $?
cat gpurun_out/r06a/lds_mul_probe.txt
bash tools/half_race_demo.sh gpurun_out/r06a/half_race || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06a/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r06a/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
/usr/bin/time -v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06a/bench.json 2> gpurun_out/r06a/bench.err
rc=$?; tail -c 2500 gpurun_out/r06a/bench.json; grep -E "Elapsed|Maximum resident" gpurun_out/r06a/bench.err; exit $rc

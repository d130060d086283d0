set -uo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "c_oneshot and 3-5-64" -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | grep -E "assert|Error|^E " | head -20

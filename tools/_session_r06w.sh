# r06w: the closing session on the final build (round 6, after the top-pass butterfly pruning) -- GPU suite, bench lines (configs 2-5),
# kernel traces, PMC traffic, the shape table
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
CONFIGS=1 SHAPES=1 bash tools/gpu_round.sh r06w

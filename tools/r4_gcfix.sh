set -o pipefail
cd "$GRAFT_REPO_ROOT"
WORKERS=64 bash tools/gpu_tasks.sh r4_gc bench && NAME=r4_cfg4_pre bash tools/r4_cfg4.sh

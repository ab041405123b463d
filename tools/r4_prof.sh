# round-4 GPU job: smoke, then marker-bounded kernel profiles of the final tree at 64 and 8 workers
set -o pipefail
cd "$GRAFT_REPO_ROOT"
WORKERS=64 bash tools/gpu_tasks.sh r4_prof64 smoke prof && WORKERS=8 bash tools/gpu_tasks.sh r4_prof8 prof

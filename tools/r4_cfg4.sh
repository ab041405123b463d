# round-4 GPU job: config 4 (100M x 1024 HBM semantic store in the agent loop, engine encoder);
# EXTRA adds batcher knobs (e.g. "--memory-min-batch 24 --memory-wait-ms 20"), NAME the out dir
set -o pipefail
cd "$GRAFT_REPO_ROOT"
BENCH_ARGS="--memory-rows 100000000 --embedder engine $EXTRA" bash tools/gpu_tasks.sh ${NAME:-r4_cfg4} bench

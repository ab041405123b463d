# Per-step semantic memory beside the engine: 10M-row index, 64 workers; then a kernel trace
# of the same run for the cosine top-k kernel's share of GPU time.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/mem
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --memory-rows 10000000 > gpurun_out/mem/mem10m.log 2>&1 && \
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/mem/prof -o m -- python3 bench.py --steps 2 --warmup 1 --memory-rows 10000000 > gpurun_out/mem/prof.log 2>&1
echo EXIT $?

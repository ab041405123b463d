# Step token budget sensitivity at 64 workers (1 GPU): 2048 (default) vs 1536 vs 1024.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/mbt2
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/mbt2/b2048.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --max-batched-tokens 1536 > gpurun_out/mbt2/b1536.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --max-batched-tokens 1024 > gpurun_out/mbt2/b1024.log 2>&1
echo EXIT $?

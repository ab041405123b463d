# GPU round check: every GPU test, then the bench at 8/16/32 workers (per-rank loads of N=8/4/2) and 64 (N=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u tools/wide_gemm_bench.py > gpurun_out/wide_bench.jsonl 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 8 > gpurun_out/bench_w8.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 16 > gpurun_out/bench_w16.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 32 > gpurun_out/bench_w32.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1
echo EXIT $?

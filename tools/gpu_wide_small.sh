set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "wide_gemm" --timeout 120 --timeout-method thread > gpurun_out/pytest_wide.log 2>&1 && \
timeout -k 10 400 python -u tools/wide_gemm_bench.py 24,32,48 > gpurun_out/wide_bench_small.jsonl 2>&1
echo EXIT $?

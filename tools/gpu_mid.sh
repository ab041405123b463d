# Mid-size GEMM: numerics tests, then the cache-cold sweep against hipBLASLt.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/mid
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "mid" --timeout 120 --timeout-method thread > gpurun_out/mid/pytest.log 2>&1 && \
timeout -k 10 400 python -u tools/mid_gemm_bench.py > gpurun_out/mid/sweep.jsonl 2>&1
echo EXIT $?

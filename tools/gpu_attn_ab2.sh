# Attention softmax rework: full GPU kernel+engine tests, then the 1-GPU bench at 64 workers.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/attab2
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -v --timeout 180 --timeout-method thread > gpurun_out/attab2/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/attab2/w64.log 2>&1
echo EXIT $?

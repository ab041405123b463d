# Wide path (17-48 tokens) with the fused decode QKV+RoPE kernel: engine numerics, bench at 8/16 workers.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wq
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_tp_gpu.py -x -q --timeout 180 --timeout-method thread > gpurun_out/wq/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 8 > gpurun_out/wq/w8.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 16 > gpurun_out/wq/w16.log 2>&1
echo EXIT $?

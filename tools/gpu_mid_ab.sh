# Mid-size path: kernel + engine GPU tests, then bench A/B (mid path on vs off) at 64 and 16 workers.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/midab
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -v -k "mid or engine or greedy or llama3 or prefix or grammar or invariance" --timeout 180 --timeout-method thread > gpurun_out/midab/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/midab/w64_mid.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --mid-max-t 0 > gpurun_out/midab/w64_lib.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 16 > gpurun_out/midab/w16_mid.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 16 --mid-max-t 0 > gpurun_out/midab/w16_lib.log 2>&1
echo EXIT $?

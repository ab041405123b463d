# Round-2 re-entry check on the restored tree: GPU tests, smoke(), bench at 8 and 64 workers.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2c
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r2c/pytest_gpu.log 2>&1 && \
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2c/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 8 > gpurun_out/r2c/bench_w8.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r2c/bench_w64.log 2>&1
echo EXIT $?

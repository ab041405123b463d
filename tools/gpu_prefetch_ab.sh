# Decode-step weight prefetch by the attention grid's idle workgroups: kernel + engine GPU tests,
# then bench A/B at 8 and 16 workers.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pfab
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "attention or engine or greedy or llama3" --timeout 180 --timeout-method thread > gpurun_out/pfab/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 8 > gpurun_out/pfab/w8_pf.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 8 --no-prefetch > gpurun_out/pfab/w8_nopf.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 16 > gpurun_out/pfab/w16_pf.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 16 --no-prefetch > gpurun_out/pfab/w16_nopf.log 2>&1
echo EXIT $?

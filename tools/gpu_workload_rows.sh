# Workload sensitivity rows for BENCHMARKS.md: default, --reply-tokens 128, --memory-rows 10M
# (per-step lookups co-resident with the engine), plus the memory test tier.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wl
timeout -k 10 300 python -u -m pytest tests/test_memory_loop.py tests/test_kernels_gpu.py -x -q -k "memory or cosine or sharded" --timeout 120 --timeout-method thread > gpurun_out/wl/pytest.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --reply-tokens 128 > gpurun_out/wl/reply128.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --memory-rows 10000000 > gpurun_out/wl/mem10m.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --workers 8 --memory-rows 10000000 > gpurun_out/wl/mem10m_w8.log 2>&1
echo EXIT $?

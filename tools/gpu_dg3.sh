# Decode GEMM: 16 chunks per round for 8-wave workgroups (M <= 16): numerics, microbench, bench at 8/16 workers.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dg3
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "decode" --timeout 180 --timeout-method thread > gpurun_out/dg3/pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/decode_gemm_bench.py 8,16 > gpurun_out/dg3/micro.jsonl 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 8 > gpurun_out/dg3/w8.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 16 > gpurun_out/dg3/w16.log 2>&1
echo EXIT $?

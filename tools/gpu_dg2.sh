# Decode GEMM with every round's loads issued up front: numerics, microbench (M=8,16), bench at 8/16 workers.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dg2
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "decode or engine or greedy or llama3 or qkv" --timeout 180 --timeout-method thread > gpurun_out/dg2/pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/decode_gemm_bench.py 8,16 > gpurun_out/dg2/micro.jsonl 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 8 > gpurun_out/dg2/w8.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 16 > gpurun_out/dg2/w16.log 2>&1
echo EXIT $?

set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "decode" --timeout 120 --timeout-method thread > gpurun_out/pytest_dg.log 2>&1 && \
timeout -k 10 400 python -u tools/decode_gemm_bench.py 8,16 > gpurun_out/dg3.jsonl 2>&1
echo EXIT $?

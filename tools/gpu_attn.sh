set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -v -k "attention or greedy or prefix or grammar or invariance" --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1 && \
timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/attn_main.jsonl 2>&1 && \
timeout -k 10 200 python -u tools/attn_bench.py --small > gpurun_out/attn_small.jsonl 2>&1
echo EXIT $?

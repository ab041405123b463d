# Attention change check: attention/engine GPU tests, small-batch microbench, 8- and 64-worker bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -v -k "attention or greedy or prefix or grammar or invariance" --timeout 120 --timeout-method thread > gpurun_out/ab/pytest_attn.log 2>&1 && \
timeout -k 10 200 python -u tools/attn_bench.py --small > gpurun_out/ab/attn_small.jsonl 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 8 > gpurun_out/ab/bench_w8.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/ab/bench_w64.log 2>&1
echo EXIT $?

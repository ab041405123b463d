# Wide (LDS-staged, 4-wave) prefill attention: numerics, then the microbenchmark (32 vs 128 columns per item).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/attn2
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "attention" --timeout 120 --timeout-method thread > gpurun_out/attn2/pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/attn_bench.py --iters 30 > gpurun_out/attn2/bench.jsonl 2>&1
echo EXIT $?

# 32-row mid tiles (fm = 1): mid GEMM tests, then the fused-form config sweep at 17-64 rows.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fm1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -k "mid" --timeout 180 --timeout-method thread > gpurun_out/fm1/pytest.log 2>&1 || exit $?
timeout -k 10 900 python -u tools/mid_gemm_bench.py 17,24,32,48,64 --fused-sweep > gpurun_out/fm1/sweep.jsonl 2> gpurun_out/fm1/sweep.err
echo EXIT $?

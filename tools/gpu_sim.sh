set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "cosine or semantic" --timeout 120 --timeout-method thread > gpurun_out/pytest_sim.log 2>&1 && \
timeout -k 10 500 python -u benchmarks/semantic_store.py > gpurun_out/config4.log 2>&1
echo EXIT $?

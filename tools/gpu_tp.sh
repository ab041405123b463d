# TP=2 engine on GPU 0 with the custom all-reduce (ranks share the GPU).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tp_gpu.py > gpurun_out/tp_gpu.log 2>&1
rc=$?
tail -60 gpurun_out/tp_gpu.log
exit $rc

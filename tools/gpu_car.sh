# Custom P2P all-reduce: kernel tests (single-process multi-rank + 2-process IPC on GPU 0).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_custom_ar_gpu.py > gpurun_out/car_tests.log 2>&1
rc=$?
tail -30 gpurun_out/car_tests.log
exit $rc

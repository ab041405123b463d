# GPU tier with the mid path from 17 tokens (wide path off by default), then the default
# bench at 16 and 8 workers.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/widemax2
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > gpurun_out/widemax2/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workers 16 --steps 4 --warmup 1 > gpurun_out/widemax2/w16.json 2> gpurun_out/widemax2/w16.err || exit $?
timeout -k 10 300 python -u bench.py --workers 8 --steps 6 --warmup 1 > gpurun_out/widemax2/w8.json 2> gpurun_out/widemax2/w8.err || exit $?
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/widemax2/w64.json 2> gpurun_out/widemax2/w64.err || exit $?
echo EXIT 0

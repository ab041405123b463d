# End-of-session check: every GPU test, smoke(), default bench, and a kernel profile of the default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1 && \
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/final/bench.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof -o w64 -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/final/prof.log 2>&1
echo EXIT $?

# Decode split-K slabs padded to whole 256-B spans: GPU tier, split-K repeat check,
# 8-worker (decode-bound) and default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/slabpad
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > gpurun_out/slabpad/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/splitk_check.py --reps 300 > gpurun_out/slabpad/splitk.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 8 > gpurun_out/slabpad/w8.json 2> gpurun_out/slabpad/w8.err || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/slabpad/bench_default.json 2> gpurun_out/slabpad/bench_default.err || exit $?
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/slabpad/smoke.log 2>&1 || exit $?
echo EXIT 0

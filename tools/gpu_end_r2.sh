# End-of-session check on the final tree: GPU tier, smoke, default bench, 64-worker kernel
# profile (summary), driver-command bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/end2
export TMPDIR=/tmp
P=/tmp/pilottai_prof
rm -rf $P && mkdir -p $P
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > gpurun_out/end2/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/end2/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/end2/bench_default.json 2> gpurun_out/end2/bench_default.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/w64 -o w64 -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/end2/prof_w64.log 2>&1 || exit $?
python3 tools/prof_summary.py $P/w64/*/*.db $P/w64/*.db --after-frac 0.5 --top 40 > gpurun_out/end2/w64_kernels.md 2>&1 || exit $?
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/end2/driver_cmd.json 2> gpurun_out/end2/driver_cmd.err || exit $?
echo EXIT 0

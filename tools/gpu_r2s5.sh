# Session check on the restored tree: GPU test tier, smoke, the default bench, and a
# 64-worker kernel profile (summary only).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s5
export TMPDIR=/tmp
P=/tmp/pilottai_prof
rm -rf $P && mkdir -p $P
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/s5/pytest_gpu.log 2>&1 && \
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s5/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/s5/bench.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/w64 -o w64 -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/s5/prof_run.log 2>&1 && \
python3 tools/prof_summary.py $P/w64/*/*.db $P/w64/*.db --after-frac 0.5 --top 40 > gpurun_out/s5/w64_kernels.md 2>&1
echo EXIT $?

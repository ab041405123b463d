# Per-GPU load of the N=2/4/8 agent-DP runs simulated on one GPU (64/N workers), plus a
# kernel profile of the 8-worker (N=8 per-rank) case.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sim
for w in 8 16 32; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers $w > gpurun_out/sim/bench_w$w.log 2>&1 || exit $?
done
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/sim/prof_w8 -o w8 -- python3 bench.py --steps 3 --warmup 1 --workers 8 > gpurun_out/sim/prof_w8.log 2>&1
echo EXIT $?

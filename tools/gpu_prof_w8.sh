# Kernel profile of the 8-worker agent step (the per-rank load of the N=8 agent-DP run).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_w8
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_w8 -o w8 -- python3 bench.py --steps 3 --warmup 1 --workers 8 > gpurun_out/prof_w8/run.log 2>&1
echo EXIT $?

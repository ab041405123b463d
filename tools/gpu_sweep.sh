# N=1 bench (64 workers) over the per-step token budget.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep64
for t in 1024 1536 2048; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --max-batched-tokens $t > gpurun_out/sweep64/mbt$t.log 2>&1 || exit $?
done
echo EXIT 0

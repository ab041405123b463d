# N=1 bench (64 workers) at larger per-step token budgets.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/mbt
for t in 3072 4096; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --max-batched-tokens $t > gpurun_out/mbt/t$t.log 2>&1 || exit $?
  tail -1 gpurun_out/mbt/t$t.log | cut -c1-300
done
echo EXIT 0

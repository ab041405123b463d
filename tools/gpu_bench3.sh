# bench.py at 8, 16 and 64 workers (per-rank loads of N=8, N=4 and N=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/b3
for w in 8 16 64; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers $w > gpurun_out/b3/w${w}.log 2>&1 || exit $?
  tail -1 gpurun_out/b3/w${w}.log
done
echo EXIT 0

# 8-worker bench (per-rank load of the N=8 run) over the fused-decode step threshold.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
for t in 16 32 64; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 8 --fused-max-t $t > gpurun_out/sweep/w8_t$t.log 2>&1 || exit $?
done
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 16 > gpurun_out/sweep/w16.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 32 > gpurun_out/sweep/w32.log 2>&1
echo EXIT $?

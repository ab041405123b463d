# A/B: packed small-batch path up to 64 tokens vs the default (32) at 16 and 32 workers.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab64
for w in 16 32; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers $w --wide-max-t 64 > gpurun_out/ab64/w${w}_t64.log 2>&1 || exit $?
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers $w > gpurun_out/ab64/w${w}_t32.log 2>&1 || exit $?
done
echo EXIT 0

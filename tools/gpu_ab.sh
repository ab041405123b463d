# A/B of the packed small-batch path (wide) against the library path at 16/32 workers.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for w in 16 32; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers $w > gpurun_out/ab/w${w}_wide.log 2>&1 || exit $?
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers $w --wide-max-t 16 > gpurun_out/ab/w${w}_lib.log 2>&1 || exit $?
done
echo EXIT 0

# A/B: down projection on 2 column tiles x 16 waves x 2 K-slices for 9-16-row decode steps.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ds
for w in 8 16; do
  PILOTTAI_DOWN_CFG=2,16,2 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers $w > gpurun_out/ds/w${w}_split.log 2>&1 || exit $?
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers $w > gpurun_out/ds/w${w}_base.log 2>&1 || exit $?
done
echo EXIT 0

# End-of-session numbers on the final tree: the driver's own command (20 steps after 5
# warmup), and the per-rank loads of N = 2, 4, 8 (32, 16, 8 workers on one GPU).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final2
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final2/driver_cmd.json 2> gpurun_out/final2/driver_cmd.err || exit $?
for W in 32 16 8; do
  timeout -k 10 300 python -u bench.py --workers $W --steps 6 --warmup 1 > gpurun_out/final2/w${W}.json 2> gpurun_out/final2/w${W}.err || exit $?
done
echo EXIT 0

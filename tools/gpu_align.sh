# Step-size alignment (--token-align) at 64 workers: 256 (default) vs 128 vs 0, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/align
for r in 1 2; do
  for a in 256 128 0; do
    timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --token-align $a > gpurun_out/align/w64_a${a}_r${r}.json 2> gpurun_out/align/w64_a${a}_r${r}.err || exit $?
  done
done
echo EXIT 0

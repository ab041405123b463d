# Step token budget at the per-rank loads of N = 4 and 8 (16 and 8 workers per GPU):
# 1024 / 1536 / 2048, then 2048 / 3072 / 4096, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/mbt3
for r in 1 2; do
  for b in 2048 3072 4096; do
    timeout -k 10 300 python -u bench.py --workers 8 --steps 6 --warmup 1 --max-batched-tokens $b > gpurun_out/mbt3/w8_b${b}_r${r}.json 2> gpurun_out/mbt3/w8_b${b}_r${r}.err || exit $?
    timeout -k 10 300 python -u bench.py --workers 16 --steps 4 --warmup 1 --max-batched-tokens $b > gpurun_out/mbt3/w16_b${b}_r${r}.json 2> gpurun_out/mbt3/w16_b${b}_r${r}.err || exit $?
  done
done
echo EXIT 0

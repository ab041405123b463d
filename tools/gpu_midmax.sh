# Mid/library boundary: --mid-max-t 256 (default) vs 320 vs 384 at 64 workers, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/midmax
for r in 1 2; do
  for t in 256 320 384; do
    timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --mid-max-t $t > gpurun_out/midmax/w64_t${t}_r${r}.json 2> gpurun_out/midmax/w64_t${t}_r${r}.err || exit $?
  done
done
echo EXIT 0

# Attention width policy: 4-wave LDS-staged prefill items from 2048 (default) / 1024 / 512
# prefill tokens per step, 64 workers, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/attwide
for r in 1 2; do
  for t in 2048 1024 512; do
    timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --att-wide-min-tokens $t > gpurun_out/attwide/w64_t${t}_r${r}.json 2> gpurun_out/attwide/w64_t${t}_r${r}.err || exit $?
  done
done
echo EXIT 0

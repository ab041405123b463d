# Decode/mid boundary: --fused-max-t 16 (default) vs 8 (9-16-token steps on the mid path;
# re-run after the 32-row mid tiles landed),
# 8 and 16 workers, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fusedmax2
for r in 1 2; do
  for t in 16 8; do
    timeout -k 10 300 python -u bench.py --workers 8 --steps 6 --warmup 1 --fused-max-t $t > gpurun_out/fusedmax2/w8_t${t}_r${r}.json 2> gpurun_out/fusedmax2/w8_t${t}_r${r}.err || exit $?
    timeout -k 10 300 python -u bench.py --workers 16 --steps 4 --warmup 1 --fused-max-t $t > gpurun_out/fusedmax2/w16_t${t}_r${r}.json 2> gpurun_out/fusedmax2/w16_t${t}_r${r}.err || exit $?
  done
done
echo EXIT 0

# Wide/mid boundary: --wide-max-t 48 (current) vs 32 vs 16 (17-48-token steps on the mid
# path), 16 and 8 workers, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/widemax
for r in 1 2; do
  for t in 48 32 16; do
    timeout -k 10 300 python -u bench.py --workers 16 --steps 4 --warmup 1 --wide-max-t $t > gpurun_out/widemax/w16_t${t}_r${r}.json 2> gpurun_out/widemax/w16_t${t}_r${r}.err || exit $?
    timeout -k 10 300 python -u bench.py --workers 8 --steps 6 --warmup 1 --wide-max-t $t > gpurun_out/widemax/w8_t${t}_r${r}.json 2> gpurun_out/widemax/w8_t${t}_r${r}.err || exit $?
  done
done
echo EXIT 0

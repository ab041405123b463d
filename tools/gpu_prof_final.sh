# Kernel profiles at the per-rank loads of N = 8 and 4 (8 and 16 workers) on the final tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/proff
export TMPDIR=/tmp
P=/tmp/pilottai_prof
rm -rf $P && mkdir -p $P
for W in 8 16; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/w$W -o w$W -- python3 bench.py --steps 6 --warmup 1 --workers $W > gpurun_out/proff/prof_w${W}.log 2>&1 || exit $?
  python3 tools/prof_summary.py $P/w$W/*/*.db $P/w$W/*.db --after-frac 0.3 --top 30 > gpurun_out/proff/w${W}_kernels.md 2>&1 || exit $?
done
echo EXIT 0

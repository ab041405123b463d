# Kernel profiles of bench.py at 8 workers (per-rank load of N=8) and 64 workers (N=1); summaries only
# (the rocpd databases exceed gpurun's copy-back cap).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
P=/tmp/pilottai_prof
rm -rf $P && mkdir -p $P
for W in 8 64; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/w$W -o w$W -- python3 bench.py --steps 3 --warmup 1 --workers $W > gpurun_out/prof/w${W}_run.log 2>&1 || exit $?
  python3 tools/prof_summary.py $P/w$W/*/*.db $P/w$W/*.db --after-frac 0.5 --top 40 > gpurun_out/prof/w${W}_kernels.md 2>&1 || exit $?
done
echo EXIT 0

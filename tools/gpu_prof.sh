# Kernel profile of bench.py at W workers (default 32); summary only (rocpd DBs exceed the copy-back cap).
set -o pipefail
cd $GRAFT_REPO_ROOT
W=${W:-32}
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
P=/tmp/pilottai_prof
rm -rf $P && mkdir -p $P
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/w$W -o w$W -- python3 bench.py --steps 3 --warmup 1 --workers $W $EXTRA > gpurun_out/prof/w${W}_run.log 2>&1 && \
python3 tools/prof_summary.py $P/w$W/*/*.db $P/w$W/*.db --after-frac 0.5 --top 40 > gpurun_out/prof/w${W}_kernels.md 2>&1
echo EXIT $?

# Kernel profiles of bench.py: 8 workers (the per-rank load of the N=8 agent-DP run) and 64 workers (N=1).
# Summaries only are kept (the rocpd databases exceed gpurun's 64 MiB copy-back).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
P=/tmp/pilottai_prof
rm -rf $P && mkdir -p $P
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/w8 -o w8 -- python3 bench.py --steps 3 --warmup 1 --workers 8 > gpurun_out/prof/w8_run.log 2>&1 && \
python3 tools/prof_summary.py $P/w8/*/*.db $P/w8/*.db --after-frac 0.5 --top 40 > gpurun_out/prof/w8_kernels.md 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/w64 -o w64 -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof/w64_run.log 2>&1 && \
python3 tools/prof_summary.py $P/w64/*/*.db $P/w64/*.db --after-frac 0.5 --top 40 > gpurun_out/prof/w64_kernels.md 2>&1
echo EXIT $?

# Kernel-trace the 8-worker bench (per-GPU load of the 8-GPU run) and split the idle time
# into step gaps (host) and in-graph gaps (kernel boundaries): tools/gap_analysis.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/gaps
P=/tmp/pilottai_gaps
rm -rf $P && mkdir -p $P
timeout -k 10 400 rocprofv3 --kernel-trace -d $P/w8 -o w8 -- python3 bench.py --steps 3 --warmup 1 --workers 8 > gpurun_out/gaps/w8_run.log 2>&1 && \
python3 tools/gap_analysis.py "$P/w8/**/*.db" --after-frac 0.5 > gpurun_out/gaps/w8_gaps.jsonl 2>&1 && \
python3 tools/prof_summary.py "$P/w8/**/*.db" --after-frac 0.5 --top 30 > gpurun_out/gaps/w8_kernels.md 2>&1
echo EXIT $?

# round-5 GPU job: marker-bounded kernel profile of the headline bench (64 workers)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_prof64${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 500 rocprofv3 --kernel-trace -d $O/prof -- python3 bench.py --steps 2 --warmup 1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 tools/prof_summary.py $(find $O/prof -name "*.db" | head -1) --between-markers --top 45 > $O/w64_kernels.md 2>&1 || { tail -20 $O/w64_kernels.md; exit 1; }
head -60 $O/w64_kernels.md

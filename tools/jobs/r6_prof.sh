# round-6 GPU job: marker-bounded kernel profiles of the 8-worker run and of config 4 (q16)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_prof${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace -d $O/w8 -- python3 bench.py --workers 8 --steps 3 --warmup 1 > $O/w8.log 2>&1 || { rc=$?; tail -20 $O/w8.log; exit $rc; }
python3 tools/prof_summary.py $(find $O/w8 -name "*.db" | head -1) --between-markers --top 40 > $O/w8_kernels.md 2>&1 || { rc=$?; tail -20 $O/w8_kernels.md; exit $rc; }
head -12 $O/w8_kernels.md
rm -rf $O/w8  # the trace database: the summary above is what is kept
timeout -s KILL 500 rocprofv3 --kernel-trace -d $O/cfg4 -- python3 bench.py --memory-rows 100000000 --embedder engine --steps 2 --warmup 1 > $O/cfg4.log 2>&1 || { rc=$?; tail -20 $O/cfg4.log; exit $rc; }
python3 tools/prof_summary.py $(find $O/cfg4 -name "*.db" | head -1) --between-markers --top 40 > $O/cfg4_kernels.md 2>&1 || { rc=$?; tail -20 $O/cfg4_kernels.md; exit $rc; }
head -20 $O/cfg4_kernels.md
rm -rf $O/cfg4

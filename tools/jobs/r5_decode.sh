# round-5 GPU job: decode-dominated regimes -- 8 workers (throughput, step buckets, a
# marker-bounded kernel profile) and 128-token replies
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_decode${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --workers 8 --steps 3 --warmup 1 > $O/w8.log 2>&1 || { tail -20 $O/w8.log; exit 1; }
grep '"metric"' $O/w8.log | cut -c1-2500
timeout -k 10 300 python -u bench.py --reply-tokens 128 --steps 2 --warmup 1 > $O/r128.log 2>&1 || { tail -20 $O/r128.log; exit 1; }
grep '"metric"' $O/r128.log | cut -c1-1500
timeout -s KILL 400 rocprofv3 --kernel-trace -d $O/prof_w8 -- python3 bench.py --workers 8 --steps 2 --warmup 1 > $O/prof_w8.log 2>&1 || { tail -20 $O/prof_w8.log; exit 1; }
python3 tools/prof_summary.py $(find $O/prof_w8 -name "*.db" | head -1) --between-markers --top 30 > $O/w8_kernels.md 2>&1 || { tail -20 $O/w8_kernels.md; exit 1; }
head -45 $O/w8_kernels.md

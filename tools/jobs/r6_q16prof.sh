# round-6 GPU job: where the q16 pass's time goes (kernel trace of the 100M-row store bench)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_q16prof${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 -u benchmarks/semantic_store.py --rows 100000000 --storage q16 --steps 5 > $O/store.log 2>&1 || { tail -20 $O/store.log; exit 1; }
grep '"metric"' $O/store.log | cut -c1-400
f=$(ls $O/prof/*/run_kernel_stats.csv $O/prof/run_kernel_stats.csv 2>/dev/null | head -1)
head -12 "$f" | cut -c1-200

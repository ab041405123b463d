# round-6 GPU job: q16 GPU tests, then the 100M-row pass under a kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_q16b${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_q16_gpu.py -x -v --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { rc=$?; tail -40 $O/tests.log; exit $rc; }
grep -E "passed|failed" $O/tests.log | tail -2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 -u benchmarks/semantic_store.py --rows 100000000 --storage q16 --steps 5 > $O/store.log 2>&1 || { rc=$?; tail -20 $O/store.log; exit $rc; }
grep '"metric"' $O/store.log | cut -c1-330
grep -h "q16::stage" $O/prof/run_kernel_stats.csv | cut -c1-40,200-400

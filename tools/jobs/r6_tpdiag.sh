# round-6 GPU job: which share-GPU TP rehearsals run (no -x: every case reported)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_tpdiag${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_tp_gpu.py -v -s --timeout 150 --timeout-method thread \
  > $O/tests.log 2>&1
grep -E "PASSED|FAILED|greedy sequences|passed|failed|timed out \(" $O/tests.log | tail -20

# round-4 GPU job: the full GPU test tier (one pytest process)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_tests${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log

# round-6 GPU job: the full GPU tier (one pytest process) and smoke on the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_tier${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/tests.log | head -20; tail -1 $O/tests.log; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { rc=$?; tail -20 $O/smoke.log; exit $rc; }
tail -1 $O/smoke.log

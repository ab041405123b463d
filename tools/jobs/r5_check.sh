# round-5 GPU job: prefill GEMM + engine GPU tests on the current tree, then the headline bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_check${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread ${TESTS:-tests/test_prefill_gemm_gpu.py tests/test_engine_gpu.py} > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
if [ -z "${NOBENCH:-}" ]; then
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '"metric"' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({k: d[k] for k in ('value','p50_task_latency_ms','step_buckets')}))"
fi
if [ -n "${CFG4:-}" ]; then
timeout -k 10 420 python -u bench.py --memory-rows 100000000 --embedder engine --steps 3 --warmup 1 > $O/cfg4.log 2>&1 || { tail -30 $O/cfg4.log; exit 1; }
grep '"metric"' $O/cfg4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({k: d[k] for k in ('value','p50_task_latency_ms','memory')}))"
fi

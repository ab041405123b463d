# round-6 GPU job: attention with the split path compiled out by default -- kernel tests, engine
# tests, step cases, the driver's bench command
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_attfix${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/tests.log | head; tail -1 $O/tests.log; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/attn_bench.py --cases prefill2048,step2048,mix,prefill4x512 --qcols 128 --split-keys 0 \
  > $O/attn_bench.jsonl 2> $O/attn_bench.err || { rc=$?; tail -5 $O/attn_bench.err; exit $rc; }
cat $O/attn_bench.jsonl | cut -c1-160
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20.log 2>&1 || { rc=$?; tail -20 $O/b20.log; exit $rc; }
grep '"metric"' $O/b20.log > $O/b20.json && python3 -c "import json; d=json.load(open('$O/b20.json')); print('steps20', d['value'], d['p50_task_latency_ms'], d['step_buckets'].get('2048'), d['step_buckets'].get('512'))"

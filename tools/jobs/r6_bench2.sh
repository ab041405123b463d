# round-6 GPU job: the driver's bench command + the 8-worker and reply-128 rows on the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_bench2${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20.log 2>&1 || { rc=$?; tail -20 $O/b20.log; exit $rc; }
grep '"metric"' $O/b20.log > $O/b20.json && python3 -c "import json; d=json.load(open('$O/b20.json')); print('steps20', d['value'], d['p50_task_latency_ms'], d['step_buckets'].get('2048'))"
timeout -k 10 300 python -u bench.py --workers 8 --steps 5 --warmup 1 > $O/w8.log 2>&1 || { rc=$?; tail -20 $O/w8.log; exit $rc; }
grep '"metric"' $O/w8.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('w8', d['value'], d['p50_task_latency_ms'])"
timeout -k 10 400 python -u bench.py --reply-tokens 128 --steps 3 --warmup 1 > $O/r128.log 2>&1 || { rc=$?; tail -20 $O/r128.log; exit $rc; }
grep '"metric"' $O/r128.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('r128', d['value'], d['p50_task_latency_ms'])"

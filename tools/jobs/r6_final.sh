# round-6 GPU job: the full GPU tier (one pytest process), smoke, the driver's bench command, the
# 8-worker and reply-128 rows, and a marker-bounded kernel profile of the headline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_final${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
# a failing test (status 1) is recorded and the benches still run; a time limit or abort ends here
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/tests.log | head -20
tail -2 $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { rc=$?; tail -20 $O/smoke.log; exit $rc; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20.log 2>&1 || { rc=$?; tail -20 $O/b20.log; exit $rc; }
grep '"metric"' $O/b20.log > $O/b20.json && python3 -c "import json; d=json.load(open('$O/b20.json')); print('steps20', d['value'], d['p50_task_latency_ms'], d['seconds'], d['step_buckets'].get('2048'))"
timeout -k 10 300 python -u bench.py --workers 8 --steps 5 --warmup 1 > $O/w8.log 2>&1 || { rc=$?; tail -20 $O/w8.log; exit $rc; }
grep '"metric"' $O/w8.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('w8', d['value'], d['p50_task_latency_ms'])"
timeout -k 10 400 python -u bench.py --reply-tokens 128 --steps 3 --warmup 1 > $O/r128.log 2>&1 || { rc=$?; tail -20 $O/r128.log; exit $rc; }
grep '"metric"' $O/r128.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('r128', d['value'], d['p50_task_latency_ms'])"
timeout -s KILL 500 rocprofv3 --kernel-trace -d $O/prof -- python3 bench.py --steps 2 --warmup 1 > $O/prof.log 2>&1 || { rc=$?; tail -20 $O/prof.log; exit $rc; }
python3 tools/prof_summary.py $(find $O/prof -name "*.db" | head -1) --between-markers --top 45 > $O/w64_kernels.md 2>&1 || { rc=$?; tail -20 $O/w64_kernels.md; exit $rc; }
head -30 $O/w64_kernels.md

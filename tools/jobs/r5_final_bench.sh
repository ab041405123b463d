# round-5 GPU job: driver-length headline bench + the decode-regime rows on the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_final${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20.log 2>&1 || { tail -20 $O/b20.log; exit 1; }
grep '"metric"' $O/b20.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('steps20', d['value'], d['p50_task_latency_ms'], d['seconds'])"
timeout -k 10 300 python -u bench.py --workers 8 --steps 5 --warmup 1 > $O/w8.log 2>&1 || { tail -20 $O/w8.log; exit 1; }
grep '"metric"' $O/w8.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('w8', d['value'], d['p50_task_latency_ms'])"
timeout -k 10 400 python -u bench.py --reply-tokens 128 --steps 3 --warmup 1 > $O/r128.log 2>&1 || { tail -20 $O/r128.log; exit 1; }
grep '"metric"' $O/r128.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('r128', d['value'], d['p50_task_latency_ms'])"

# round-5 GPU job: step-size cap A/B on the headline bench (alternating, same box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_cap${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
for cap in ${CAPS:-2048 4096}; do
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --max-batched-tokens $cap > $O/b$cap.$rep.log 2>&1 || { tail -20 $O/b$cap.$rep.log; exit 1; }
echo "cap $cap rep $rep $(grep '"metric"' $O/b$cap.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['p50_task_latency_ms'])")"
done
done

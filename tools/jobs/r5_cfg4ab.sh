# round-5 GPU job: config 4 with the first step's lookup started beside the opening calls
# (this tree) vs after them (the previous agent.py, copied in for the run), alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_cfg4ab${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
cp pilottai_amd/core/agent.py /tmp/agent_new.py
cp bench.py /tmp/bench_new.py
for rep in 1 2; do
for v in new old; do
if [ $v = old ]; then cp tools/jobs/alt/agent_before_first_lookup.py pilottai_amd/core/agent.py; cp tools/jobs/alt/bench_prev.py bench.py; else cp /tmp/agent_new.py pilottai_amd/core/agent.py; cp /tmp/bench_new.py bench.py; fi
timeout -k 10 500 python -u bench.py --memory-rows 100000000 --embedder engine --steps 3 --warmup 1 > $O/$v.$rep.log 2>&1 || { tail -20 $O/$v.$rep.log; exit 1; }
echo "$v rep=$rep $(grep '"metric"' $O/$v.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['memory']; print(d['value'], d['p50_task_latency_ms'], m['lookup_p50_ms'], m['lookup_p99_ms'], m['passes'])")"
done
done
cp /tmp/agent_new.py pilottai_amd/core/agent.py
cp /tmp/bench_new.py bench.py

# round-5 GPU job: config 4 with writes and queries embedded in one engine call (this tree)
# vs in two calls in sequence (the previous batcher.py, copied in for the run), alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_sharedemb${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
cp pilottai_amd/memory/batcher.py /tmp/batcher_new.py
for rep in 1 2; do
for v in new old; do
if [ $v = old ]; then cp tools/jobs/alt/batcher_prev.py pilottai_amd/memory/batcher.py; else cp /tmp/batcher_new.py pilottai_amd/memory/batcher.py; fi
timeout -k 10 500 python -u bench.py --memory-rows 100000000 --embedder engine --steps 3 --warmup 1 > $O/$v.$rep.log 2>&1 || { tail -20 $O/$v.$rep.log; exit 1; }
echo "$v rep=$rep $(grep '"metric"' $O/$v.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['memory']; print(d['value'], d['p50_task_latency_ms'], m['lookup_p50_ms'], m['lookup_p99_ms'], m['passes'], m.get('shared_embeds'))")"
done
done
cp /tmp/batcher_new.py pilottai_amd/memory/batcher.py

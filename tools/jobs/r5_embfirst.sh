# round-5 GPU job: config 4 with embedding requests admitted first (default) vs FCFS
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_embfirst${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for v in 1 0; do
PILOTTAI_EMBED_FIRST=$v timeout -k 10 500 python -u bench.py --memory-rows 100000000 --embedder engine --steps 3 --warmup 1 > $O/e$v.$rep.log 2>&1 || { tail -20 $O/e$v.$rep.log; exit 1; }
echo "embed_first=$v rep=$rep $(grep '"metric"' $O/e$v.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['memory']; print(d['value'], d['p50_task_latency_ms'], m['lookup_p50_ms'], m['lookup_p99_ms'], m['passes'])")"
done
done

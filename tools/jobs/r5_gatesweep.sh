# round-5 GPU job: config 4 gate knobs on the final memory path (wait cap ms, trigger tokens),
# alternating, 2 reps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_gatesweep${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for cfg in "30 1024" "60 1024" "15 1024" "30 512" "60 512" "0 1024"; do
set -- $cfg
timeout -k 10 400 python -u bench.py --memory-rows 100000000 --embedder engine --steps 3 --warmup 1 --memory-gate-ms $1 --memory-gate-tokens $2 > $O/g$1_$2.$rep.log 2>&1 || { tail -20 $O/g$1_$2.$rep.log; exit 1; }
echo "gate_ms=$1 tokens=$2 rep=$rep $(grep '"metric"' $O/g$1_$2.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['memory']; print(d['value'], d['p50_task_latency_ms'], m['lookup_p50_ms'], m['lookup_p99_ms'], m['passes'], m['beside_heavy_frac'], m.get('lookup_anatomy_ms'))")"
done
done

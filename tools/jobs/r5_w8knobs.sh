# round-5 GPU job: decode-path boundary at 8 workers (alternating, same box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_w8knobs${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
declare -A V
V[base]=''
V[fused32]='--fused-max-t 32'
for rep in 1 2 3; do
for k in base fused32; do
timeout -k 10 300 python -u bench.py --workers 8 --steps 4 --warmup 1 ${V[$k]} > $O/$k.$rep.log 2>&1 || { tail -20 $O/$k.$rep.log; exit 1; }
echo "$k rep=$rep $(grep '"metric"' $O/$k.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['step_buckets']; print(d['value'], d['p50_task_latency_ms'], {k: b[k] for k in ('16','32','48') if k in b})")"
done
done

# round-5 GPU job: engine knobs re-checked on the new kernel routing (alternating, same box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_knobs${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
declare -A V
V[base]=''
V[mid384]='--mid-max-t 384'
V[align128]='--token-align 128'
for rep in 1 2 3; do
for k in base mid384 align128; do
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 ${V[$k]} > $O/$k.$rep.log 2>&1 || { tail -20 $O/$k.$rep.log; exit 1; }
echo "$k rep=$rep $(grep '"metric"' $O/$k.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['p50_task_latency_ms'])")"
done
done

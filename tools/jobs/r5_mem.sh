# round-5 GPU job: the node-wide memory store over 2 ranks sharing GPU 0, then config 4 with
# the index scans co-scheduled with compute-bound steps vs not
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_mem${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
PILOTTAI_DIST_BACKEND=gloo timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29551 bench.py --gpus 2 --share-gpu --memory-rows 20000000 --steps 2 \
  --warmup 1 > $O/share2_mem.log 2>&1 || { tail -30 $O/share2_mem.log; exit 1; }
grep '"metric"' $O/share2_mem.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({k: d[k] for k in ('value','n_gpus','rehearsal','world_size','memory')}))"
for g in 1024 0; do
timeout -k 10 420 python -u bench.py --memory-rows 100000000 --embedder engine --steps 3 --warmup 1 \
  --memory-gate-tokens $g > $O/cfg4_gate$g.log 2>&1 || { tail -30 $O/cfg4_gate$g.log; exit 1; }
grep '"metric"' $O/cfg4_gate$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({k: d[k] for k in ('value','p50_task_latency_ms','memory')}))"
done

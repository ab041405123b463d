# round-6 GPU job: config 4 on the shipped q16 default, and the N>1 bench path (2 ranks, one GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_cfg${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --memory-rows 100000000 --embedder engine --steps 3 --warmup 1 > $O/cfg4.log 2>&1 || { rc=$?; tail -20 $O/cfg4.log; exit $rc; }
grep '"metric"' $O/cfg4.log > $O/cfg4.json && python3 -c "
import json; d=json.load(open('$O/cfg4.json')); m=d['memory']
print('cfg4', d['value'], d['p50_task_latency_ms'], {k: m.get(k) for k in ('storage','lookup_ms_per_pass','lookup_p50_ms','lookup_p99_ms','passes','q16_fallbacks','stores','store_failures')})"
PILOTTAI_DIST_BACKEND=gloo timeout -k 10 420 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29573 bench.py --gpus 2 --share-gpu --steps 2 --warmup 1 > $O/dp2.log 2>&1 || { rc=$?; grep -v Gloo $O/dp2.log | tail -30; exit $rc; }
grep '"metric"' $O/dp2.log > $O/dp2.json && python3 -c "
import json; d=json.load(open('$O/dp2.json')); print('dp2', d['value'], d['n_gpus'], d['config']['parallelism'], d['world_size'], d['rehearsal'], d['llm_calls_per_rank'])"

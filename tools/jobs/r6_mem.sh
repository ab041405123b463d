# round-6 GPU job: node-wide memory through the production write path (2 ranks on one GPU),
# then config 4 (100M-row store, engine embedder) on the q16 two-stage scan and on bf16
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_mem${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
PILOTTAI_DIST_BACKEND=gloo timeout -k 10 420 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 2 --share-gpu --memory-rows 20000000 \
  --steps 2 --warmup 1 > $O/node_mem.log 2>&1 || { rc=$?; grep -v Gloo $O/node_mem.log | tail -30; exit $rc; }
grep '"metric"' $O/node_mem.log > $O/node_mem.json && python3 -c "
import json; d=json.load(open('$O/node_mem.json')); m=d['memory']
print('node-mem', d['value'], {k: m.get(k) for k in ('store','stores','store_failures','lookup_failures','node_hits','node_remote_hits','rows_total','lookups')})"
for st in q16 bf16; do
  timeout -k 10 500 python -u bench.py --memory-rows 100000000 --embedder engine --memory-storage $st --steps 3 --warmup 1 \
    > $O/cfg4_$st.log 2>&1 || { rc=$?; tail -20 $O/cfg4_$st.log; exit $rc; }
  grep '"metric"' $O/cfg4_$st.log > $O/cfg4_$st.json && python3 -c "
import json; d=json.load(open('$O/cfg4_$st.json')); m=d['memory']
print('cfg4 $st', d['value'], d['p50_task_latency_ms'], {k: m.get(k) for k in ('storage','lookup_ms_per_pass','lookup_p50_ms','lookup_p99_ms','passes','q16_fallbacks','stores','store_failures')})"
done

# round-5 GPU job: config 5's TP=2 shared-GPU rehearsal WITH hipGraphs, the TP step graph's
# launches per 70B layer, the 2-rank node-wide memory store rehearsal, config 4 gate A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_cfg${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
PILOTTAI_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29541 tools/graph_nodes.py --model llama-3-70b --share-gpu \
  --out $O/graph_nodes_tp2.jsonl > $O/graph_nodes_tp2.log 2>&1 || { tail -30 $O/graph_nodes_tp2.log; exit 1; }
cut -c1-300 $O/graph_nodes_tp2.jsonl
PILOTTAI_DIST_BACKEND=gloo timeout -k 10 700 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 benchmarks/workflow.py --share-gpu --clients 2 \
  --workflows 4 --warmup 1 --doc-words 120 --kv-gb 8 > $O/tp2.log 2>&1 || { tail -30 $O/tp2.log; exit 1; }
grep '"metric"' $O/tp2.log | cut -c1-600

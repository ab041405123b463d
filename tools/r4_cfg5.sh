# round-4 GPU job: config 5 on the round-4 tree -- Llama-3-70B TP=1 on one GPU, then the TP=2
# shared-GPU rehearsal (fused all-reduce + residual + row-statistics epilogue, radix-histogram
# top-k/top-p thresholds) with a crashed replica
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_cfg5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u benchmarks/workflow.py > $O/tp1.log 2>&1 || { tail -20 $O/tp1.log; exit 1; }
grep '"metric"' $O/tp1.log | cut -c1-400
PILOTTAI_DIST_BACKEND=gloo timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 benchmarks/workflow.py --share-gpu --no-graphs --clients 2 \
  --workflows 4 --warmup 1 --doc-words 120 --kv-gb 8 > $O/tp2.log 2>&1 || { tail -30 $O/tp2.log; exit 1; }
grep '"metric"' $O/tp2.log | cut -c1-400

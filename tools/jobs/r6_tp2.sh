# round-6 GPU job: the TP engine at 2/4 ranks on one GPU (eager and graphs), then config 5 at TP=4
# as a share-GPU rehearsal (4 ranks x 35 GB packed weights on one card) and bench --tp 2 (2 ranks)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_tp2${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
PILOTTAI_CAR_WG=8 GPU_MAX_HW_QUEUES=1 PILOTTAI_DIST_BACKEND=gloo timeout -k 10 420 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29551 benchmarks/workflow.py --share-gpu --clients 2 \
  --workflows 4 --warmup 1 --doc-words 120 --kv-gb 8 > $O/tp4.log 2>&1 || { grep -v Gloo $O/tp4.log | tail -40; exit 1; }
grep '"metric"' $O/tp4.log > $O/wf_tp4.json && cut -c1-900 $O/wf_tp4.json
PILOTTAI_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --tp 2 --share-gpu --steps 2 --warmup 1 \
  > $O/bench_tp2.log 2>&1 || { grep -v Gloo $O/bench_tp2.log | tail -30; exit 1; }
grep '"metric"' $O/bench_tp2.log | cut -c1-700

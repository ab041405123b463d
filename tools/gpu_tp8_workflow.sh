# 1-GPU rehearsal of BASELINE config 5 at TP=8: 8 ranks share GPU 0 (Llama-3-70B, 1/8 of the
# weights each, real IPC handles, custom P2P all-reduce for every row-parallel message, gloo
# control plane). Timing reflects 8 processes time-slicing one GPU, not xGMI.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PILOTTAI_DIST_BACKEND=gloo
timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29571 benchmarks/workflow.py --share-gpu --kv-gb 6 --clients 4 --workflows 8 --warmup 2 \
  --doc-words 120 > gpurun_out/tp8_workflow.log 2>&1
rc=$?
grep -v Gloo gpurun_out/tp8_workflow.log | tail -20
echo EXIT $rc
exit $rc

# 1-GPU rehearsal of BASELINE config 5 with tensor parallelism: 2 ranks share GPU 0 (Llama-3-70B,
# half of the weights each, real IPC handles, custom P2P all-reduce, gloo control plane).
# The TP=8 variant (tools/gpu_tp8_workflow.sh) does not finish on one GPU: 8 processes
# time-slicing one card with spinning all-reduces cost ~6 s per engine step.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PILOTTAI_DIST_BACKEND=gloo
timeout -k 10 700 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29572 benchmarks/workflow.py --share-gpu --kv-gb 16 --clients 2 --workflows 4 --warmup 1 \
  --doc-words 120 > gpurun_out/tp2_workflow.log 2>&1
rc=$?
grep -v Gloo gpurun_out/tp2_workflow.log | tail -8
echo EXIT $rc
exit $rc

# Node control plane with real engines: 2 ranks share GPU 0 (gloo collectives), ONE manager on
# rank 0 over both ranks' agents; plus the RCCL-branch GPU test.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/node2
export PILOTTAI_DIST_BACKEND=gloo
timeout -k 10 200 python -u -m pytest tests/test_rccl_gpu.py -x -v --timeout 180 --timeout-method thread > gpurun_out/node2/rccl.log 2>&1 && \
timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29561 bench.py --gpus 2 --share-gpu --steps 2 --warmup 1 --workers 32 --kv-gb 24 > gpurun_out/node2/bench.log 2>&1
echo EXIT $?

# 1-GPU rehearsal of the multi-rank bench: 2 ranks (16 workers each... 32 total) share GPU 0 over gloo.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PILOTTAI_DIST_BACKEND=gloo
timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29561 bench.py --gpus 2 --share-gpu --steps 2 --warmup 1 --workers 32 --kv-gb 24 > gpurun_out/rehearse2.log 2>&1
echo EXIT $?

# 1-GPU rehearsal of the 4-rank bench: 4 ranks (8 workers each, 32 total) share GPU 0 over gloo.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PILOTTAI_DIST_BACKEND=gloo
timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29563 bench.py --gpus 4 --share-gpu --steps 2 --warmup 1 --workers 32 --kv-gb 12 > gpurun_out/rehearse4.log 2>&1
rc=$?
grep '^{' gpurun_out/rehearse4.log | cut -c1-600
echo EXIT $rc
exit $rc

# round-4 GPU job: 2-rank bench rehearsal on one GPU (both ranks run a real engine; gloo)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_share2
mkdir -p $O
export TMPDIR=/tmp
PILOTTAI_DIST_BACKEND=gloo timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --steps 3 --warmup 1 --share-gpu > $O/share2.log 2>&1 || { tail -30 $O/share2.log; exit 1; }
grep '"metric"' $O/share2.log | cut -c1-400

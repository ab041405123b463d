# round-5 GPU job: the 2-rank data-parallel bench path on one shared GPU (rehearsal of the
# driver's multi-GPU run on the final tree)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_dp2${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --share-gpu --steps 3 --warmup 1 > $O/dp2.log 2>&1 || { tail -30 $O/dp2.log; exit 1; }
grep '"metric"' $O/dp2.log | cut -c1-900

# Large default KV pool + segmented-LRU prefix eviction: the driver's command (20 steps) and the 3-step run.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/slru
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/slru/drv.log 2>&1 && \
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --workers 8 > gpurun_out/slru/w8.log 2>&1
echo EXIT $?

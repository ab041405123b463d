# 1-GPU rehearsal of the TP all-reduce benchmark: 2 and 4 ranks share GPU 0 over IPC.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PILOTTAI_DIST_BACKEND=gloo
timeout -k 10 200 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 benchmarks/allreduce.py --share-gpu > gpurun_out/car_bench_w2.jsonl 2> gpurun_out/car_bench_w2.err && \
timeout -k 10 200 python -m torch.distributed.run --nnodes 1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29612 benchmarks/allreduce.py --share-gpu > gpurun_out/car_bench_w4.jsonl 2> gpurun_out/car_bench_w4.err
rc=$?
cat gpurun_out/car_bench_w2.jsonl gpurun_out/car_bench_w4.jsonl
exit $rc

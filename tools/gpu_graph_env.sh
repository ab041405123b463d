# Graph launch host cost under HIP runtime settings (packet capture, device kernargs).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/genv
timeout -k 10 200 python -u tools/graph_launch_bench.py --buckets 8,16 > gpurun_out/genv/default.jsonl 2>&1 && \
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 200 python -u tools/graph_launch_bench.py --buckets 8,16 > gpurun_out/genv/pktcap1.jsonl 2>&1 && \
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 python -u tools/graph_launch_bench.py --buckets 8,16 > gpurun_out/genv/pktcap0.jsonl 2>&1 && \
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python -u tools/graph_launch_bench.py --buckets 8,16 > gpurun_out/genv/devkarg.jsonl 2>&1
echo EXIT $?

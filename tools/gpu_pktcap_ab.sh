# Engine at 8 workers with graph packet capture on (package default) and with device kernargs too.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pkt
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 8 > gpurun_out/pkt/w8.log 2>&1 && \
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 8 > gpurun_out/pkt/w8_dk.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/pkt/w64.log 2>&1
echo EXIT $?

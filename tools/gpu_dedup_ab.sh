# In-flight prefix dedup A/B at 64 and 8 workers (1 GPU).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dedup
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/dedup/w64_on.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-prefix-dedup > gpurun_out/dedup/w64_off.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 8 > gpurun_out/dedup/w8_on.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 8 --no-prefix-dedup > gpurun_out/dedup/w8_off.log 2>&1
echo EXIT $?

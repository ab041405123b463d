# Engine host/device phase split at 8 and 64 workers (1 GPU), then a kernel-trace of the 8-worker run.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hostph
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 8 > gpurun_out/hostph/w8.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/hostph/w64.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/hostph/prof8 -o w8 -- python -u bench.py --steps 2 --warmup 1 --workers 8 > gpurun_out/hostph/prof8.log 2>&1
echo EXIT $?

# Prefill attention item width policy in the engine: wide items from 1024 / 1536 / 2048 prefill
# tokens (>= 2 sequences) vs never, 64 workers.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wideab
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --att-wide-min-tokens 1000000 > gpurun_out/wideab/never.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --att-wide-min-tokens 2048 > gpurun_out/wideab/t2048.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --att-wide-min-tokens 1024 > gpurun_out/wideab/t1024.log 2>&1
echo EXIT $?

# N=1 bench (64 workers) over step-size knobs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep64
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/sweep64/base.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --max-batched-tokens 3072 > gpurun_out/sweep64/mbt3072.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --max-batched-tokens 4096 > gpurun_out/sweep64/mbt4096.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --token-align 512 --align-slack 192 > gpurun_out/sweep64/align512.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --token-align 0 > gpurun_out/sweep64/noalign.log 2>&1
echo EXIT $?

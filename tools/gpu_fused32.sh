# Packed decode path up to 32 / 48 tokens (after the load-batching fix) vs the default 16, 8 and 16 workers.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/f32
timeout -k 10 300 python -u tools/decode_gemm_bench.py 32,48 > gpurun_out/f32/micro.jsonl 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 16 --fused-max-t 32 > gpurun_out/f32/w16_f32.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 16 > gpurun_out/f32/w16_f16.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 8 --fused-max-t 32 > gpurun_out/f32/w8_f32.log 2>&1
echo EXIT $?

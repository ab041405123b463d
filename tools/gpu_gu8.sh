# gate_up + SwiGLU at 8 / 16 rows: mid kernel (32-row tiles, fused sweep) vs the decode kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gu8
timeout -k 10 400 python -u tools/mid_gemm_bench.py 8,16 --fused-sweep > gpurun_out/gu8/mid.jsonl 2> gpurun_out/gu8/mid.err || exit $?
timeout -k 10 300 python -u tools/decode_variant_ab.py --variants 1 --ms 8,16 > gpurun_out/gu8/decode.jsonl 2> gpurun_out/gu8/decode.err || exit $?
echo EXIT 0

set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4_handoff
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/handoff_cost.py --rounds 9 --out gpurun_out/r4_handoff/cost.jsonl > gpurun_out/r4_handoff/cost.log 2>&1 || exit $?
timeout -k 10 700 python -u tools/splitk_check.py --reps 10000 --modes 1 --only attention --out gpurun_out/r4_handoff/splitk_attn.jsonl > gpurun_out/r4_handoff/splitk_attn.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/splitk_check.py --reps 10000 --modes 1 --only "decode_qkv_rope M9 S3" --out gpurun_out/r4_handoff/splitk_gemm.jsonl > gpurun_out/r4_handoff/splitk_gemm.log 2>&1 || exit $?
echo done

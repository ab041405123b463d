# round-5 GPU job: the four-wave 256 x 256 kernel (gemm_w4.h, prefill variant 10) -- fp32
# numerics first, then timings against the ping-pong kernel and hipBLASLt
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_w4${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_prefill_gemm_gpu.py \
  -k "256-10 or identity" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u tools/prefill_gemm_bench.py --shapes ${SHAPES:-sq,gate_up,down} --M ${MS:-2048,4096} --rounds 3 \
  --variants lib,pp256w,pp256w_fused,w4,w4_fused --out $O/bench.jsonl > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
cut -c1-400 $O/bench.jsonl

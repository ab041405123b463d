# round-5 GPU job: 256 x 192 ping-pong tiles -- fp32 numerics, then qkv timings against the
# 256-wide / 128-wide tiles and hipBLASLt; config 4 gate A/B after the cap fix
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_gemm192${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_prefill_gemm_gpu.py \
  -k "192 or identity" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python -u tools/prefill_gemm_bench.py --shapes qkv --M 1024,1280,1536,1792,2048,2304,4096 \
  --rounds 5 --variants lib,pp192w,pp256w,pp128w,pp192w_fused,pp256w_fused,pp128w_fused,ropekv192,ropekv256,ropekv128 \
  --out $O/qkv.jsonl > $O/qkv.log 2>&1 || { tail -30 $O/qkv.log; exit 1; }
cut -c1-900 $O/qkv.jsonl
if [ -n "${GATE:-}" ]; then
for g in 1024 0; do
timeout -k 10 420 python -u bench.py --memory-rows 100000000 --embedder engine --steps 3 --warmup 1 \
  --memory-gate-tokens $g > $O/cfg4_gate$g.log 2>&1 || { tail -30 $O/cfg4_gate$g.log; exit 1; }
grep '"metric"' $O/cfg4_gate$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({k: d[k] for k in ('value','p50_task_latency_ms','memory')}))"
done
fi

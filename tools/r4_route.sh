# round-4 GPU job: engine numerics with the stream routing tables, in-engine A/B of the tables
# against the round-3 choice (prefill-size and 64-row decode steps), stream hand-off stress
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_route${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_stream_gemm_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo '[{"STREAM_CFG": {}, "LM_HEAD_STREAM": []}, {}]' > $O/ov.json
timeout -k 10 600 python -u tools/midrange_ab.py --T 32,48,64,96,128,192,256 --reps 8 --overrides $O/ov.json --out $O/ab_prefill.jsonl > $O/ab_prefill.log 2>&1 || { tail -20 $O/ab_prefill.log; exit 1; }
cat $O/ab_prefill.jsonl
timeout -k 10 600 python -u tools/midrange_ab.py --T 64 --reps 4 --decode 64,550,24 --overrides $O/ov.json --out $O/ab_decode64.jsonl > $O/ab_decode.log 2>&1 || { tail -20 $O/ab_decode.log; exit 1; }
cat $O/ab_decode64.jsonl
timeout -k 10 600 python -u tools/splitk_check.py --reps ${REPS:-5000} --only stream --out $O/stream_handoff.jsonl > $O/handoff.log 2>&1 || { tail -20 $O/handoff.log; exit 1; }
cat $O/stream_handoff.jsonl

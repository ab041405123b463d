# round-4 GPU job: fused attention + O launch with split tile ownership and the sc1 hand-off:
# kernel tests, stamps per mode, in-engine A/B per mode
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_attno2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_attn_o_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for m in 0 4 1; do
  PILOTTAI_ATTN_O_MODE=$m timeout -k 10 120 python -u tools/attn_o_stamps.py --out $O/stamps_mode$m.jsonl > $O/stamps_mode$m.log 2>&1 || { tail -20 $O/stamps_mode$m.log; exit 1; }
  echo "stamps mode $m: $(cat $O/stamps_mode$m.jsonl)"
done
PILOTTAI_ATTN_O_FUSED=1 timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/engine_tests.log 2>&1 || { tail -40 $O/engine_tests.log; exit 1; }
tail -2 $O/engine_tests.log
echo '[{"ATTN_O_FUSED": false}, {"ATTN_O_FUSED": true}]' > $O/ov.json
for m in 0 4; do
  PILOTTAI_ATTN_O_MODE=$m timeout -k 10 400 python -u tools/midrange_ab.py --T 8 --reps 4 --decode 8,600,48 --overrides $O/ov.json --out $O/ab8_mode$m.jsonl > $O/ab8_mode$m.log 2>&1 || { tail -20 $O/ab8_mode$m.log; exit 1; }
  echo "ab8 mode $m: $(cat $O/ab8_mode$m.jsonl)"
done
PILOTTAI_ATTN_O_MODE=0 timeout -k 10 400 python -u tools/midrange_ab.py --T 16 --reps 4 --decode 16,800,48 --overrides $O/ov.json --out $O/ab16.jsonl > $O/ab16.log 2>&1 || { tail -20 $O/ab16.log; exit 1; }
echo "ab16: $(cat $O/ab16.jsonl)"

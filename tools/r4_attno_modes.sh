set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_attno_modes
mkdir -p $O
export TMPDIR=/tmp
echo '[{"ATTN_O_FUSED": false}, {"ATTN_O_FUSED": true}]' > $O/ov.json
for m in 1 0 3 2; do
  PILOTTAI_ATTN_O_MODE=$m timeout -k 10 400 python -u tools/midrange_ab.py --T 8 --reps 4 --decode 8,600,48 --overrides $O/ov.json --out $O/ab8_mode$m.jsonl > $O/ab8_mode$m.log 2>&1 || { tail -20 $O/ab8_mode$m.log; exit 1; }
  echo "mode $m: $(cat $O/ab8_mode$m.jsonl)"
done

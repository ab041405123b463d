# round-4 GPU job: decode partition rule x attention waves on the mid path (32 / 64 / 128-row decode steps)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_attmid2
mkdir -p $O
export TMPDIR=/tmp
echo '[{}, {"split_decode": false}, {"decode_part_target": 512}, {"decode_part_target": 512, "ATT_MID_WAVES": 8}, {"ATT_MID_WAVES": 8, "split_decode": false}, {"decode_part_target": 256, "ATT_MID_WAVES": 8}]' > $O/ov.json
for RC in 64,600 32,600 128,600 64,1200 16,1200; do
  R=${RC%,*}; C=${RC#*,}; T=$R; [ $R -lt 32 ] && T=32
  timeout -k 10 500 python -u tools/midrange_ab.py --T $T --reps 3 --decode $R,$C,40 --overrides $O/ov.json --out $O/ab.jsonl > $O/ab_${R}_$C.log 2>&1 || { tail -20 $O/ab_${R}_$C.log; exit 1; }
  echo "R=$R ctx=$C $(tail -1 $O/ab.jsonl)"
done

# round-4 GPU job: decode-sized steps, whole-context 8-wave items vs flash-decoding partitions
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_ssp
mkdir -p $O
export TMPDIR=/tmp
echo '[{}, {"small_step_part": 512}, {"small_step_part": 256}]' > $O/ov.json
for RC in 8,600 8,1200 16,800; do
  R=${RC%,*}; C=${RC#*,}
  timeout -k 10 400 python -u tools/midrange_ab.py --T $R --reps 4 --decode $R,$C,48 --overrides $O/ov.json --out $O/ab.jsonl > $O/ab_${R}_$C.log 2>&1 || { tail -20 $O/ab_${R}_$C.log; exit 1; }
  echo "R=$R ctx=$C $(tail -1 $O/ab.jsonl)"
done

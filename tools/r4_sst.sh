# round-4 GPU job: small_step_target (balanced partitions for decode-sized 8-wave steps) -- step A/B and 8-worker bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_sst
mkdir -p $O
export TMPDIR=/tmp
echo '[{}, {"small_step_target": 192}, {"small_step_target": 256}]' > $O/ov.json
for RC in 8,600 8,1200 16,800 4,900; do
  R=${RC%,*}; C=${RC#*,}; T=$R; [ $R -lt 8 ] && T=8
  timeout -k 10 400 python -u tools/midrange_ab.py --T $T --reps 4 --decode $R,$C,48 --overrides $O/ov.json --out $O/ab.jsonl > $O/ab_${R}_$C.log 2>&1 || { tail -20 $O/ab_${R}_$C.log; exit 1; }
  echo "R=$R ctx=$C $(tail -1 $O/ab.jsonl)"
done
for rep in 1 2; do
  for t in 192 0; do
    PILOTTAI_SMALL_STEP_TARGET=$t timeout -k 10 420 python -u bench.py --workers 8 --steps 3 --warmup 1 > $O/w8_${t}_$rep.log 2>&1 || { tail -20 $O/w8_${t}_$rep.log; exit 1; }
    echo "w8 target=$t rep=$rep $(grep '"metric"' $O/w8_${t}_$rep.log | tail -1 | cut -c120-175)"
  done
done

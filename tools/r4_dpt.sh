# round-4 GPU job: headline + reply-128 benches with the decode partition rule on (512) / off (0), alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_dpt
mkdir -p $O
export TMPDIR=/tmp
i=0
for t in 512 0 512 0; do
  i=$((i+1))
  PILOTTAI_DECODE_PART_TARGET=$t timeout -k 10 420 python -u bench.py --gpus 1 --steps 3 --warmup 1 > $O/bench_${t}_$i.log 2>&1 || { tail -20 $O/bench_${t}_$i.log; exit 1; }
  echo "target=$t run=$i $(tail -1 $O/bench_${t}_$i.log | cut -c1-200)"
done
for t in 512 0; do
  PILOTTAI_DECODE_PART_TARGET=$t timeout -k 10 600 python -u bench.py --gpus 1 --steps 3 --warmup 1 --reply-tokens 128 > $O/reply_$t.log 2>&1 || { tail -20 $O/reply_$t.log; exit 1; }
  echo "reply128 target=$t $(tail -1 $O/reply_$t.log | cut -c1-200)"
done

# round-5 GPU job: wide (128-column) prefill attention threshold on the (KV, slots) grid:
# --att-wide-min-tokens 1024 (default) vs 512 vs 2048, headline bench alternating, 2 reps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_widemin${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for w in 1024 512 2048; do
timeout -k 10 400 python -u bench.py --att-wide-min-tokens $w > $O/w$w.$rep.log 2>&1 || { tail -20 $O/w$w.$rep.log; exit 1; }
echo "wide_min=$w rep=$rep $(grep '"metric"' $O/w$w.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['step_buckets']; print(d['value'], b.get('512'), b.get('768'), b.get('1024'), b.get('2048'))")"
done
done

# round-5 GPU job: decode partition target of mid / large steps on the (KV, slots) grid:
# PILOTTAI_DECODE_PART_TARGET 384 (default) vs 256 vs 512, headline alternating, 2 reps,
# then --reply-tokens 128 at 384 vs 512
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_dpt${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for t in 384 256 512; do
PILOTTAI_DECODE_PART_TARGET=$t timeout -k 10 400 python -u bench.py > $O/d$t.$rep.log 2>&1 || { tail -20 $O/d$t.$rep.log; exit 1; }
echo "target=$t rep=$rep $(grep '"metric"' $O/d$t.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['step_buckets']; print(d['value'], b.get('64'), b.get('128'), b.get('256'))")"
done
done
for t in 384 512; do
PILOTTAI_DECODE_PART_TARGET=$t timeout -k 10 500 python -u bench.py --reply-tokens 128 > $O/r$t.log 2>&1 || { tail -20 $O/r$t.log; exit 1; }
echo "r128 target=$t $(grep '"metric"' $O/r$t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['step_buckets']; print(d['value'], b.get('64'), b.get('128'))")"
done

# round-5 GPU job: decode-sized steps on the (KV, slots) attention grid -- the partition
# target of 8-wave steps (small_step_target 192, the default) vs no split (0), R-row steps
# from tools/rows_anatomy.py alternating, then the 8-worker bench both ways
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_smallpart${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for t in 192 0; do
for R in 8 16 32; do
PILOTTAI_SMALL_STEP_TARGET=$t timeout -k 10 200 python -u tools/rows_anatomy.py --rows $R --ctx ${CTX:-600} --steps 32 --out $O/rows.jsonl > $O/r$R.$t.$rep.log 2>&1 || { tail -20 $O/r$R.$t.$rep.log; exit 1; }
echo "target=$t R=$R rep=$rep $(tail -1 $O/rows.jsonl)"
done
done
done
for rep in 1 2; do
for t in 192 0; do
PILOTTAI_SMALL_STEP_TARGET=$t timeout -k 10 300 python -u bench.py --workers 8 > $O/w8.$t.$rep.log 2>&1 || { tail -20 $O/w8.$t.$rep.log; exit 1; }
echo "w8 target=$t rep=$rep $(grep '"metric"' $O/w8.$t.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['step_buckets']; print(d['value'], {k:v for k,v in b.items() if int(k)<=32})")"
done
done

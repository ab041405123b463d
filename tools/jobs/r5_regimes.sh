# round-5 GPU job: the decode-dominated regimes on the current tree (8 workers, 128-token
# replies) and the decode attention microbenchmark
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_regimes${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/attn_bench.py --cases decode64,decode64_long,mix --qcols 128 > $O/att.log 2>&1 || { tail -20 $O/att.log; exit 1; }
grep '"case"' $O/att.log
timeout -k 10 300 python -u tools/attn_bench.py --small --waves 4,8 --iters 50 > $O/att_small.log 2>&1 || { tail -20 $O/att_small.log; exit 1; }
grep '"case"' $O/att_small.log | head -40
timeout -k 10 400 python -u bench.py --workers 8 > $O/w8.log 2>&1 || { tail -20 $O/w8.log; exit 1; }
grep '"metric"' $O/w8.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['step_buckets']; print('w8', d['value'], {k:v for k,v in b.items() if int(k)<=64})"
timeout -k 10 500 python -u bench.py --reply-tokens 128 > $O/r128.log 2>&1 || { tail -20 $O/r128.log; exit 1; }
grep '"metric"' $O/r128.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['step_buckets']; print('r128', d['value'], {k:v for k,v in b.items() if int(k)<=128})"

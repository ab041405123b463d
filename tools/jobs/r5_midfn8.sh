# round-5 GPU job: mid kernel 256-column tiles (fn 8) at 64-128 rows vs the other mid tiles and
# the stream kernel (tools/stream_gemm_bench.py, graph-replayed)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_midfn8${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mid" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 500 python -u tools/mid_gemm_bench.py 64,96,128 --fused-sweep --shapes qkv,o,down --fms 1,2,4 --fns 2,4,8 --splits 1,2,4,8,16 > $O/mid.jsonl 2> $O/mid.err || { tail -20 $O/mid.err; exit 1; }
python3 -c "
import json
for l in open('$O/mid.jsonl'):
    d=json.loads(l); cf={k:v for k,v in d.items() if k.startswith('v1')}
    top=sorted((v,k) for k,v in cf.items())[:4]
    print(d['shape'], d['M'], top, 'fn8', sorted((v,k) for k,v in cf.items() if 'x8' in k)[:2])"
timeout -k 10 300 python -u tools/stream_gemm_bench.py --M 64,96,128 --shapes qkv,o,down --rounds 3 > $O/stream.jsonl 2> $O/stream.err || { tail -20 $O/stream.err; exit 1; }
cut -c1-400 $O/stream.jsonl

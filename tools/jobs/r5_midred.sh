# round-5 GPU job: mid kernel split-K reduce with batched slab loads (this tree) vs the
# one-quad-at-a-time reduce (tools/jobs/alt/_C_prev.so): mid GEMM tests, then the fused
# (engine epilogue) config sweep of tools/mid_gemm_bench.py with each build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_midred${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
SO=pilottai_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/_C_new.so
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mid" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in new old; do
if [ $v = old ]; then cp tools/jobs/alt/_C_prev.so $SO; else cp /tmp/_C_new.so $SO; fi
timeout -k 10 400 python -u tools/mid_gemm_bench.py ${MS:-64,96,128,192,256} --fused-sweep > $O/sweep_$v.jsonl 2> $O/sweep_$v.err || { tail -20 $O/sweep_$v.err; exit 1; }
echo "== $v"; python3 -c "
import json
for l in open('$O/sweep_$v.jsonl'):
    d=json.loads(l); print(d['shape'], d['M'], 'best', d['best'], d.get(d['best']), 'fused', d['fused'], 'lib', d['lib'])"
done
cp /tmp/_C_new.so $SO

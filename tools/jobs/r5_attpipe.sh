# round-5 GPU job: software-pipelined wide prefill attention (this tree) vs the previous
# loop (tools/jobs/alt/_C_kvfast.so swapped in): attention tests, microbenchmark, headline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_attpipe${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
SO=pilottai_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/_C_new.so
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention or attn" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in new old; do
if [ $v = old ]; then cp tools/jobs/alt/_C_kvfast.so $SO; else cp /tmp/_C_new.so $SO; fi
timeout -k 10 200 python -u tools/attn_bench.py --cases step2048,prefill4x512,prefill2048,prefill8x256,mix --qcols 128 > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
echo "== $v"; grep '"case"' $O/bench_$v.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['case'], d['grid_items'], d['us'], d['TFLOPs'])"
done
for rep in 1 2; do
for v in new old; do
if [ $v = old ]; then cp tools/jobs/alt/_C_kvfast.so $SO; else cp /tmp/_C_new.so $SO; fi
timeout -k 10 400 python -u bench.py > $O/hb_$v.$rep.log 2>&1 || { tail -20 $O/hb_$v.$rep.log; exit 1; }
echo "$v rep=$rep $(grep '"metric"' $O/hb_$v.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['step_buckets']; print(d['value'], b.get('2048'), b.get('1024'), b.get('512'))")"
done
done
cp /tmp/_C_new.so $SO

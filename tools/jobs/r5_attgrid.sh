# round-5 GPU job: attention grid with the KV head as the fastest workgroup index (default)
# vs the item slot (PILOTTAI_ATT_GRID=item): attention tests, microbenchmark, then the
# headline bench alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_attgrid${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention or attn" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for g in kv item; do
E=""; [ $g = item ] && E=item
PILOTTAI_ATT_GRID=$E timeout -k 10 200 python -u tools/attn_bench.py --cases step2048,prefill4x512,prefill2048,prefill8x256,decode64,mix --qcols 128 > $O/bench_$g.log 2>&1 || { tail -20 $O/bench_$g.log; exit 1; }
echo "== $g"; grep '"case"' $O/bench_$g.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['case'], d['grid_items'], d['us'])"
done
for rep in 1 2; do
for g in kv item; do
E=""; [ $g = item ] && E=item
PILOTTAI_ATT_GRID=$E timeout -k 10 400 python -u bench.py > $O/hb_$g.$rep.log 2>&1 || { tail -20 $O/hb_$g.$rep.log; exit 1; }
echo "$g rep=$rep $(grep '"metric"' $O/hb_$g.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('step_buckets', ''))" | cut -c1-400)"
done
done

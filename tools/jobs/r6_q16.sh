# round-6 GPU job: the q16 two-stage exact scan -- GPU tests vs the CPU reference, then the
# config-4 store at 100M rows for both storages (one index resident at a time)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_q16${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_q16_gpu.py -x -v --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/tests.log | tail -14
for st in q16 bf16; do
  timeout -k 10 400 python -u benchmarks/semantic_store.py --rows 100000000 --storage $st --steps 10 \
    > $O/store_$st.log 2>&1 || { tail -20 $O/store_$st.log; exit 1; }
  grep '"metric"' $O/store_$st.log | cut -c1-900
done

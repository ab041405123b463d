# 32-column prefill items with the next K/V tile in flight (new) vs without (old):
# attention tests, attention microbench and 64-worker bench, alternating builds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pfpre
SO=pilottai_amd/_C.cpython-310-x86_64-linux-gnu.so
cp ab/_C_new.so $SO || exit 1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -k "attention or engine or layer_dims" --timeout 180 --timeout-method thread > gpurun_out/pfpre/pytest.log 2>&1 || exit $?
for r in 1 2; do
  for v in new old; do
    cp ab/_C_$v.so $SO || exit 1
    timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/pfpre/attn_${v}_$r.jsonl 2>&1 || exit $?
    timeout -k 10 200 python -u tools/attn_bench.py --scan > gpurun_out/pfpre/scan_${v}_$r.jsonl 2>&1 || exit $?
  done
done
for r in 1 2; do
  for v in new old; do
    cp ab/_C_$v.so $SO || exit 1
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/pfpre/w64_${v}_r${r}.json 2> gpurun_out/pfpre/w64_${v}_r${r}.err || exit $?
  done
done
cp ab/_C_new.so $SO
echo EXIT 0

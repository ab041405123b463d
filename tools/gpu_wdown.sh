# Wide-path down_proj split 8 at M <= 32 (new) vs 4 (old): wide kernel tests, 16-worker
# bench alternating builds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wdown
SO=pilottai_amd/_C.cpython-310-x86_64-linux-gnu.so
cp ab/_C_new.so $SO || exit 1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -k "wide or engine or layer_dims" --timeout 180 --timeout-method thread > gpurun_out/wdown/pytest.log 2>&1 || exit $?
for r in 1 2; do
  for v in new old; do
    cp ab/_C_$v.so $SO || exit 1
    timeout -k 10 300 python -u bench.py --workers 16 --steps 4 --warmup 1 > gpurun_out/wdown/w16_${v}_r${r}.json 2> gpurun_out/wdown/w16_${v}_r${r}.err || exit $?
  done
done
cp ab/_C_new.so $SO
echo EXIT 0

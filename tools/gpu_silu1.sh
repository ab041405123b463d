# Wide-path SwiGLU with one tile per wave (new) vs two (old): wide kernel tests, microbench,
# 16-worker bench alternating builds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/silu1
SO=pilottai_amd/_C.cpython-310-x86_64-linux-gnu.so
cp ab/_C_new.so $SO || exit 1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -k "wide or engine or layer_dims" --timeout 180 --timeout-method thread > gpurun_out/silu1/pytest.log 2>&1 || exit $?
for v in new old; do
  cp ab/_C_$v.so $SO || exit 1
  timeout -k 10 200 python -u tools/wide_gemm_bench.py 24,32,48 > gpurun_out/silu1/wide_${v}.jsonl 2>&1 || exit $?
done
for r in 1 2; do
  for v in new old; do
    cp ab/_C_$v.so $SO || exit 1
    timeout -k 10 300 python -u bench.py --workers 16 --steps 4 --warmup 1 > gpurun_out/silu1/w16_${v}_r${r}.json 2> gpurun_out/silu1/w16_${v}_r${r}.err || exit $?
  done
done
cp ab/_C_new.so $SO
echo EXIT 0

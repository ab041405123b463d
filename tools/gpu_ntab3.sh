# (1) GPU test tier on the new build (decode + wide + mid nt, mid only with one row tile);
# (2) mid microbench new vs old; (3) attention K/V nt build (attnt) vs new on the attention
# microbench; (4) 8- and 64-worker bench over old / new / attnt, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ntab3
SO=pilottai_amd/_C.cpython-310-x86_64-linux-gnu.so
cp ab/_C_new.so $SO || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > gpurun_out/ntab3/pytest.log 2>&1 || exit $?
cp ab/_C_attnt.so $SO || exit 1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -k "attention or engine" --timeout 180 --timeout-method thread > gpurun_out/ntab3/pytest_attnt.log 2>&1 || exit $?
for v in new old; do
  cp ab/_C_$v.so $SO || exit 1
  timeout -k 10 300 python -u tools/mid_gemm_bench.py 128,256 --quick > gpurun_out/ntab3/mid_${v}.jsonl 2>&1 || exit $?
done
for r in 1 2; do
  for v in attnt new; do
    cp ab/_C_$v.so $SO || exit 1
    timeout -k 10 200 python -u tools/attn_bench.py --small > gpurun_out/ntab3/attn_small_${v}_$r.jsonl 2>&1 || exit $?
    timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/ntab3/attn_${v}_$r.jsonl 2>&1 || exit $?
  done
done
for r in 1 2; do
  for v in new old attnt; do
    cp ab/_C_$v.so $SO || exit 1
    timeout -k 10 300 python -u bench.py --workers 8 --steps 6 --warmup 1 > gpurun_out/ntab3/w8_${v}_r${r}.json 2> gpurun_out/ntab3/w8_${v}_r${r}.err || exit $?
    timeout -k 10 300 python -u bench.py --workers 64 --steps 3 --warmup 1 > gpurun_out/ntab3/w64_${v}_r${r}.json 2> gpurun_out/ntab3/w64_${v}_r${r}.err || exit $?
  done
done
cp ab/_C_new.so $SO
echo EXIT 0

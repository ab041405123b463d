# Re-run the GPU test tier twice on the all-nt build, then the wide/mid microbench + bench A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ntab
SO=pilottai_amd/_C.cpython-310-x86_64-linux-gnu.so
cp ab/_C_new.so $SO || exit 1
for r in 1 2; do
  timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > gpurun_out/ntab/pytest_full_$r.log 2>&1
  echo "pytest run $r exit $?" >> gpurun_out/ntab/pytest_summary.txt
done
for r in 1 2; do
  for v in new old; do
    cp ab/_C_$v.so $SO || exit 1
    timeout -k 10 200 python -u tools/wide_gemm_bench.py 24,32,48 > gpurun_out/ntab/wide_${v}_$r.jsonl 2>&1 || exit $?
    timeout -k 10 300 python -u tools/mid_gemm_bench.py 64,128,256 --quick > gpurun_out/ntab/mid_${v}_$r.jsonl 2>&1 || exit $?
  done
done
for r in 1 2; do
  for v in new old; do
    cp ab/_C_$v.so $SO || exit 1
    timeout -k 10 300 python -u bench.py --workers 16 --steps 4 --warmup 1 > gpurun_out/ntab/w16_${v}_r${r}.json 2> gpurun_out/ntab/w16_${v}_r${r}.err || exit $?
    timeout -k 10 300 python -u bench.py --workers 64 --steps 3 --warmup 1 > gpurun_out/ntab/w64_${v}_r${r}.json 2> gpurun_out/ntab/w64_${v}_r${r}.err || exit $?
  done
done
cp ab/_C_new.so $SO
echo EXIT 0

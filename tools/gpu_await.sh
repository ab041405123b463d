# (1) Host wake-up after the step's stream synchronize: HIP's active-wait window
# (ROC_ACTIVE_WAIT_TIMEOUT, us) unset vs 20000, 8- and 64-worker bench, alternating.
# (2) Decode-GEMM config sweep with the non-temporal weight stream (M = 8, 16, 32).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/await
for r in 1 2; do
  for v in spin default; do
    if [ $v = spin ]; then export ROC_ACTIVE_WAIT_TIMEOUT=20000; else unset ROC_ACTIVE_WAIT_TIMEOUT; fi
    timeout -k 10 300 python -u bench.py --workers 8 --steps 6 --warmup 1 > gpurun_out/await/w8_${v}_r${r}.json 2> gpurun_out/await/w8_${v}_r${r}.err || exit $?
    timeout -k 10 300 python -u bench.py --workers 64 --steps 3 --warmup 1 > gpurun_out/await/w64_${v}_r${r}.json 2> gpurun_out/await/w64_${v}_r${r}.err || exit $?
  done
done
unset ROC_ACTIVE_WAIT_TIMEOUT
timeout -k 10 400 python -u tools/decode_gemm_bench.py 8,16,32 > gpurun_out/await/decode_sweep_nt.jsonl 2> gpurun_out/await/decode_sweep_nt.err || exit $?
echo EXIT 0

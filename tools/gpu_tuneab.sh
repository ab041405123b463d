# Shipped TunableOp file A/B: the merged re-tune (new) vs the previous file (old), 64 workers.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tuneab
F=pilottai_amd/tuned/gemm_llama-3-8b_tp1.csv
for r in 1 2 3; do
  for v in new old; do
    cp ab/tuned_$v.csv $F || exit 1
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/tuneab/w64_${v}_r${r}.json 2> gpurun_out/tuneab/w64_${v}_r${r}.err || exit $?
  done
done
cp ab/tuned_new.csv $F
echo EXIT 0

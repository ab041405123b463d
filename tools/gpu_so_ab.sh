# Same-box A/B of two builds of the extension (ab/_C_new.so vs ab/_C_old.so), alternating,
# on the 8-worker bench (decode-latency bound) and the attention microbench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/soab
SO=pilottai_amd/_C.cpython-310-x86_64-linux-gnu.so
for r in 1 2; do
  for v in new old; do
    cp ab/_C_$v.so $SO || exit 1
    timeout -k 10 200 python -u tools/attn_bench.py --small > gpurun_out/soab/attn_${v}_$r.jsonl 2>&1 || exit $?
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workers 8 > gpurun_out/soab/w8_${v}_$r.log 2>&1 || exit $?
  done
done
cp ab/_C_new.so $SO
echo EXIT 0

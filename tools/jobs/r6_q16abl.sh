# round-6 GPU job: q16 stage-1 timing ablations (1 = no epilogue, 2 = loads only) vs full, 100M rows
# (ablated runs answer wrongly by design: the bench's exit 1 on a wrong answer is expected there)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_q16abl${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
for v in 2 3 0; do
  PILOTTAI_Q16_STAGE1=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/v$v -o run -- \
    python3 -u benchmarks/semantic_store.py --rows 100000000 --storage q16 --steps 3 > $O/v$v.log 2>&1
  rc=$?
  if [ $rc -ne 0 ] && { [ $rc -ne 1 ] || [ $v = 0 ]; }; then tail -20 $O/v$v.log; exit 1; fi
  echo "variant $v rc $rc"; grep -h "q16::stage1" $O/v$v/run_kernel_stats.csv | cut -c1-60,200-300
done

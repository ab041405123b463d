# Session verification: GPU tier + smoke on the final tree, 8-row down_proj config A/B
# (1 tile x 8 waves vs the 16-wave default; llama.py edited in the box's scratch copy),
# 64-worker bench, kernel profiles at 8 and 64 workers (summaries only).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s5b
export TMPDIR=/tmp
P=/tmp/pilottai_prof
rm -rf $P && mkdir -p $P
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > gpurun_out/s5b/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s5b/smoke.log 2>&1 || exit $?
cp pilottai_amd/models/llama.py /tmp/llama_new.py
sed 's/if T > 8 else {"nt": 1, "waves": 8}/if T > 8 else {}/' /tmp/llama_new.py > /tmp/llama_old.py
for r in 1 2; do
  for v in new old; do
    cp /tmp/llama_$v.py pilottai_amd/models/llama.py || exit 1
    timeout -k 10 300 python -u bench.py --workers 8 --steps 6 --warmup 1 > gpurun_out/s5b/w8_${v}_r${r}.json 2> gpurun_out/s5b/w8_${v}_r${r}.err || exit $?
  done
done
cp /tmp/llama_new.py pilottai_amd/models/llama.py
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/s5b/bench.json 2> gpurun_out/s5b/bench.err || exit $?
for W in 8 64; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/w$W -o w$W -- python3 bench.py --steps 3 --warmup 1 --workers $W > gpurun_out/s5b/prof_w${W}.log 2>&1 || exit $?
  python3 tools/prof_summary.py $P/w$W/*/*.db $P/w$W/*.db --after-frac 0.5 --top 40 > gpurun_out/s5b/w${W}_kernels.md 2>&1 || exit $?
done
echo EXIT 0

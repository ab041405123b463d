# Round-2 start: every GPU test, smoke(), default bench, kernel profile of the default bench,
# and the hipBLASLt mid-M survey that the new mid-M GEMM has to beat.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2s
export TMPDIR=/tmp
P=/tmp/pilottai_prof
rm -rf $P && mkdir -p $P
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/r2s/pytest_gpu.log 2>&1 && \
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2s/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r2s/bench.log 2>&1 && \
timeout -k 10 200 python -u tools/prefill_gemm_bench.py 64,96,128,192,256,384,512 > gpurun_out/r2s/midm_hipblaslt.jsonl 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/w64 -o w64 -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/r2s/prof_run.log 2>&1 && \
python3 tools/prof_summary.py $P/w64/*/*.db $P/w64/*.db --after-frac 0.5 --top 40 > gpurun_out/r2s/w64_kernels.md 2>&1
echo EXIT $?

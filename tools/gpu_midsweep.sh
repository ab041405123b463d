# Mid-path (49-256 tokens) config sweep in the engine's epilogue form (fused), current kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/midsweep
timeout -k 10 900 python -u tools/mid_gemm_bench.py 64,96,128,160,192,256 --fused-sweep > gpurun_out/midsweep/sweep.jsonl 2> gpurun_out/midsweep/sweep.err
echo EXIT $?

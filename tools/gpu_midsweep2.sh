# Mid-path fused sweep at 160-256 rows including the 32-row tiles.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/midsweep2
timeout -k 10 900 python -u tools/mid_gemm_bench.py 160,192,256 --fused-sweep > gpurun_out/midsweep2/sweep.jsonl 2> gpurun_out/midsweep2/sweep.err
echo EXIT $?

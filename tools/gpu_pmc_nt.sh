# Counter passes over the decode GEMM's default-policy vs non-temporal weight stream.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcnt
cd /tmp && export TMPDIR=/tmp
run_pass() {
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/pmcnt/raw_$P -- python3 $R/tools/pmc_nt.py > $R/gpurun_out/pmcnt/$P.log 2>&1 && \
  python3 $R/tools/pmc_summary.py $R/gpurun_out/pmcnt/raw_$P > $R/gpurun_out/pmcnt/$P.json && rm -rf $R/gpurun_out/pmcnt/raw_$P
}
P=p1 run_pass FETCH_SIZE GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES && \
P=p2 run_pass TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
echo EXIT $?

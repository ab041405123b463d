# Hardware-counter passes over the hot kernels (tools/pmc_kernels.py), one counter set per run.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
run_pass() {
  timeout -s KILL 180 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/pmc/raw_$P -- python3 $R/tools/pmc_kernels.py > $R/gpurun_out/pmc/$P.log 2>&1 && \
  python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc/raw_$P > $R/gpurun_out/pmc/$P.json && rm -rf $R/gpurun_out/pmc/raw_$P
}
P=p1 run_pass FETCH_SIZE GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES && \
P=p2 run_pass SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES && \
P=p3 run_pass TCC_HIT_sum TCC_MISS_sum WRITE_SIZE TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
echo EXIT $?

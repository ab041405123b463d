# Hardware-counter passes over the mid-size GEMM variants and hipBLASLt (tools/pmc_mid.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcmid
cd /tmp && export TMPDIR=/tmp
run_pass() {
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/pmcmid/raw_$P -- python3 $R/tools/pmc_mid.py > $R/gpurun_out/pmcmid/$P.log 2>&1 && \
  python3 $R/tools/pmc_summary.py $R/gpurun_out/pmcmid/raw_$P > $R/gpurun_out/pmcmid/$P.json && rm -rf $R/gpurun_out/pmcmid/raw_$P
}
P=p1 run_pass SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_WAIT_INST_LDS && \
P=p2 run_pass SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE FETCH_SIZE && \
P=p3 run_pass TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_BUSY_max TCP_TOTAL_CACHE_ACCESSES_sum
echo EXIT $?

# Hardware counters of the prefill attention paths (tools/pmc_attn.py), one counter set per run.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcattn
cd /tmp && export TMPDIR=/tmp
run_pass() {
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/pmcattn/raw_$P -- python3 $R/tools/pmc_attn.py > $R/gpurun_out/pmcattn/$P.log 2>&1 && \
  python3 $R/tools/pmc_summary_disp.py $R/gpurun_out/pmcattn/raw_$P > $R/gpurun_out/pmcattn/$P.json && rm -rf $R/gpurun_out/pmcattn/raw_$P
}
P=p1 run_pass SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU && \
P=p2 run_pass SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE
echo EXIT $?

# round-6 GPU job: PMC passes over the q16 stage-1 kernel (both variants), 20M-row store
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_q16pmc${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
P1=SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_LDS
P2=SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,SQ_ACTIVE_INST_VALU,SQ_INSTS_SMEM,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_ANY,SQ_WAVES
P3=FETCH_SIZE,GRBM_GUI_ACTIVE,GRBM_COUNT
for v in 0 1; do
  for p in 1 2 3; do
    eval PM=\$P$p
    PILOTTAI_Q16_STAGE1=$v timeout -s KILL 120 rocprofv3 --pmc $PM --kernel-include-regex stage1 --output-format csv -d $O/v${v}p$p -o run -- \
      python3 -u benchmarks/semantic_store.py --rows 20000000 --storage q16 --steps 3 > $O/v${v}p$p.log 2>&1 || { tail -20 $O/v${v}p$p.log; exit 1; }
    grep '"metric"' $O/v${v}p$p.log | cut -c150-260
  done
done
ls -R $O | head -30

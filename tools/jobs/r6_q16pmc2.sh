# round-6 GPU job: PMC of the q16 bound kernel, full (1) vs no-epilogue ablation (2), 100M rows
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_q16pmc2${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
P1=SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_VALU_MFMA_BUSY_CYCLES,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU
P2=SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,SQ_INSTS_SMEM,SQ_WAVES
for v in 1 2; do
  for p in 1 2; do
    eval PM=\$P$p
    PILOTTAI_Q16_STAGE1=$v timeout -s KILL 150 rocprofv3 --pmc $PM --kernel-include-regex bound_kernel --output-format csv -d $O/v${v}p$p -o run -- \
      python3 -u benchmarks/semantic_store.py --rows 100000000 --storage q16 --steps 2 > $O/v${v}p$p.log 2>&1
    rc=$?
    if [ $rc -ne 0 ] && { [ $rc -ne 1 ] || [ $v = 1 ]; }; then tail -20 $O/v${v}p$p.log; exit 1; fi
    echo "v$v p$p rc $rc"
  done
done

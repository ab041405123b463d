# round-5 GPU job: prefill attention (128-column LDS-staged items) -- timings of the bench's
# step shapes and the counters of the step2048 / prefill2048 dispatches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_attpmc${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/attn_bench.py --cases step2048,prefill4x512,prefill2048,prefill8x256 --qcols 128 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
cat $O/bench.log
for c in step2048 prefill2048; do
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU \
  --output-format csv -d $O/pmc_$c -- python3 tools/pmc_attn.py --case $c --qcols 128 > $O/pmc_$c.log 2>&1 || { tail -20 $O/pmc_$c.log; exit 1; }
python3 tools/pmc_summary.py $O/pmc_$c > $O/pmc_$c.json
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVES SQ_ACTIVE_INST_LDS \
  --output-format csv -d $O/pmc2_$c -- python3 tools/pmc_attn.py --case $c --qcols 128 > $O/pmc2_$c.log 2>&1 || { tail -20 $O/pmc2_$c.log; exit 1; }
python3 tools/pmc_summary.py $O/pmc2_$c > $O/pmc2_$c.json
done

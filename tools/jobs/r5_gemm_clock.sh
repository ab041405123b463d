# round-5 GPU job: where the large-step GEMM loses to hipBLASLt -- in-kernel clock and cycles
# (stamp build), counters and durations of both kernels at 4096^3 and gate_up M = 2,048
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_gemm_clock${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/pp_stamps.py --shapes sq:4096,gate_up:2048 --out $O/stamps.jsonl > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
cut -c1-700 $O/stamps.jsonl
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
  --output-format csv -d $O/pmc -- python3 tools/pmc_prefill.py --shapes 4096:4096:4096,2048:28672:4096 > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python3 tools/pmc_summary.py $O/pmc > $O/pmc_summary.json
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -- python3 tools/pmc_prefill.py --shapes 4096:4096:4096,2048:28672:4096 > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
find $O/kt -name "*kernel_stats.csv" -exec cut -c1-200 {} \; | head -12
timeout -k 10 300 python -u tools/prefill_gemm_bench.py --shapes sq,gate_up,down,o --M 2048,4096 --rounds 3 \
  --variants lib,pp256w,pp256w_fused,pp128w,pp128w_fused --out $O/bench.jsonl > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
cut -c1-500 $O/bench.jsonl

# round-4 GPU job: counters of the decode attention (64 / 128 rows, ctx 600, whole-context items)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_pmcdec
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/pmc_decode_attn.py > $O/timing.log 2>&1 || { tail -20 $O/timing.log; exit 1; }
cat $O/timing.log | grep rows
i=0
for cs in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "FETCH_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  rm -rf /tmp/pmcdec_$i
  timeout -s KILL 120 rocprofv3 --pmc $cs --output-format csv -d /tmp/pmcdec_$i -- python3 tools/pmc_decode_attn.py > $O/pmc_$i.log 2>&1 || { tail -20 $O/pmc_$i.log; exit 1; }
  python3 tools/pmc_summary.py /tmp/pmcdec_$i > $O/pmc_$i.json || exit 1
  python3 - "$O/pmc_$i.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if "paged_attn" in k:
        print(k[:40], {c: round(x["mean"], 1) for c, x in v.items()})
PY
done

# round-4 GPU job: marker-bounded kernel anatomy of 32 / 64 / 128-row decode steps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_rows
mkdir -p $O
export TMPDIR=/tmp
for R in 64 128 32; do
  P=/tmp/pilottai_rows_$R
  rm -rf "$P" && mkdir -p "$P"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$P" -o r -- python3 tools/rows_anatomy.py --rows $R --ctx 600 --steps 24 --out $O/rows.jsonl > $O/rows_$R.log 2>&1 || { tail -30 $O/rows_$R.log; exit 1; }
  python3 tools/prof_summary.py "$P"/*/*.db "$P"/*.db --between-markers --top 30 > "$O/rows${R}_kernels.md" 2>&1 || { tail -20 $O/rows${R}_kernels.md; exit 1; }
  tail -1 $O/rows.jsonl
  head -16 $O/rows${R}_kernels.md
done

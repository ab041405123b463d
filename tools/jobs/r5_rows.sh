# round-5 GPU job: kernel anatomy of 8- and 64-row decode steps (marker-bounded)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_rows${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
for R in ${ROWS:-8 64}; do
timeout -s KILL 300 rocprofv3 --kernel-trace -d $O/p$R -- python3 tools/rows_anatomy.py --rows $R --ctx ${CTX:-600} --steps 24 --out $O/rows.jsonl > $O/p$R.log 2>&1 || { tail -20 $O/p$R.log; exit 1; }
python3 tools/prof_summary.py $(find $O/p$R -name "*.db" | head -1) --between-markers --top 40 > $O/rows$R.md 2>&1 || { tail -20 $O/rows$R.md; exit 1; }
done
cat $O/rows.jsonl
for R in ${ROWS:-8 64}; do head -50 $O/rows$R.md | cut -c1-200; done

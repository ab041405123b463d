# round-4 GPU job: pipelined decode tile loop -- attention numerics, engine tests, row-step anatomy, A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_attpipe
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_attn_o_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/engine_tests.log 2>&1 || { tail -40 $O/engine_tests.log; exit 1; }
tail -2 $O/engine_tests.log
for R in 64 128 32; do
  P=/tmp/pilottai_rows_$R
  rm -rf "$P" && mkdir -p "$P"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$P" -o r -- python3 tools/rows_anatomy.py --rows $R --ctx 600 --steps 24 --out $O/rows.jsonl > $O/rows_$R.log 2>&1 || { tail -30 $O/rows_$R.log; exit 1; }
  python3 tools/prof_summary.py "$P"/*/*.db "$P"/*.db --between-markers --top 12 > "$O/rows${R}_kernels.md" 2>&1 || { tail -20 $O/rows${R}_kernels.md; exit 1; }
  tail -1 $O/rows.jsonl
  grep paged_attn $O/rows${R}_kernels.md | cut -c1-60
done
timeout -k 10 420 python -u bench.py --gpus 1 --steps 3 --warmup 1 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200

# One parameterised runner for the GPU-box jobs of this repo (replaces the round-1/2
# one-off tools/gpu_*.sh scripts; they are in git history). Run through gpurun:
#
#   gpurun --timeout 900 -- 'bash tools/gpu_tasks.sh OUT_DIR TASK [TASK ...]'
#
# Every task writes under gpurun_out/OUT_DIR, runs under its own timeout, and the chain
# stops at the first failing task (no GPU step runs after a fault, abort or time-out).
# Knobs (environment): REPS, WORKERS, STEPS, WARMUP, MLIST, BENCH_ARGS.
#
# tasks:
#   tests          python -m pytest tests -m gpu (all GPU tests)
#   tests:<file>   one GPU test file, e.g. tests:tests/test_prefill_gemm_gpu.py
#   smoke          __graft_entry__.smoke()
#   bench          bench.py (driver shape: --gpus 1 --steps $STEPS --warmup $WARMUP)
#   bench_w        bench.py --workers $WORKERS (one per-rank load of the multi-GPU runs)
#   prof           rocprofv3 --kernel-trace --stats of bench.py --workers $WORKERS, summarised
#   splitk         tools/splitk_check.py --reps $REPS (hand-off stress, both consumer modes)
#   handoff_cost   tools/handoff_cost.py
#   pfbench        tools/prefill_gemm_bench.py --M $MLIST
#   anatomy        tools/step_anatomy.py
#   danat          tools/decode_anatomy.py under rocprofv3 --kernel-trace --stats (decode-step anatomy)
#   midsweep       tools/mid_gemm_bench.py $MLIST --fused-sweep (mid-path configs, engine epilogues)
#   cmd            bash -c "$CMD" (log: $CMD_NAME.log, limit $CMD_SECS s)
#   pmc            rocprofv3 --pmc passes over $PMC_SCRIPT, one pass per ';'-separated set in
#                  $PMC_SETS (each set within the per-block slot limits), summarised per kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
REPS=${REPS:-3000}
WORKERS=${WORKERS:-64}
STEPS=${STEPS:-3}
WARMUP=${WARMUP:-1}
MLIST=${MLIST:-512,768,1024,1536,2048}
run() {  # run NAME SECONDS CMD...
  local name=$1 secs=$2
  shift 2
  echo "[gpu_tasks] $name: $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[gpu_tasks] $name rc=$rc"
  tail -3 "$OUT/$name.log"
  return $rc
}
for t in "$@"; do
  case "$t" in
    tests) run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $? ;;
    tests:*) f=${t#tests:}; run "tests_$(basename "$f" .py)" 600 python -u -m pytest "$f" -m gpu -x -v --timeout 120 --timeout-method thread || exit $? ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) run bench 900 python -u bench.py --gpus 1 --steps "$STEPS" --warmup "$WARMUP" $BENCH_ARGS || exit $? ;;
    bench_w) run "bench_w$WORKERS" 600 python -u bench.py --workers "$WORKERS" --steps "$STEPS" --warmup "$WARMUP" $BENCH_ARGS || exit $? ;;
    prof)
      P=/tmp/pilottai_prof_$WORKERS
      rm -rf "$P" && mkdir -p "$P"
      run "prof_w$WORKERS" 600 rocprofv3 --kernel-trace --stats -d "$P" -o w -- python3 bench.py --steps "$STEPS" --warmup "$WARMUP" --workers "$WORKERS" $BENCH_ARGS || exit $?
      python3 tools/prof_summary.py "$P"/*/*.db "$P"/*.db --between-markers --top 40 > "$OUT/w${WORKERS}_kernels.md" 2>&1 || exit $?
      ;;
    splitk) run splitk 900 python -u tools/splitk_check.py --reps "$REPS" --out "$OUT/splitk.jsonl" $SPLITK_ARGS || exit $? ;;
    handoff_cost) run handoff_cost 300 python -u tools/handoff_cost.py --out "$OUT/handoff_cost.jsonl" || exit $? ;;
    pfbench) run pfbench 900 python -u tools/prefill_gemm_bench.py --M "$MLIST" --out "$OUT/pfbench.jsonl" $PF_ARGS || exit $? ;;
    midsweep) run midsweep 900 python -u tools/mid_gemm_bench.py "$MLIST" --fused-sweep || exit $? ;;
    cmd) run "${CMD_NAME:-cmd}" "${CMD_SECS:-600}" bash -c "$CMD" || exit $? ;;
    anatomy) run anatomy 600 python -u tools/step_anatomy.py $ANATOMY_ARGS || exit $? ;;
    danat)
      P=/tmp/pilottai_danat
      rm -rf "$P" && mkdir -p "$P"
      run danat 600 rocprofv3 --kernel-trace --stats -d "$P" -o d -- python3 -u tools/decode_anatomy.py --part engine --out "$OUT/danat.jsonl" || exit $?
      python3 tools/prof_summary.py "$P"/*/*.db "$P"/*.db --after-frac 0.5 --top 40 > "$OUT/danat_kernels.md" 2>&1 || exit $?
      run danat_proj 600 python3 -u tools/decode_anatomy.py --part proj --out "$OUT/danat.jsonl" || exit $?
      ;;
    pmc)
      i=0
      IFS=';' read -ra SETS <<< "$PMC_SETS"
      for cs in "${SETS[@]}"; do
        i=$((i + 1))
        rm -rf "/tmp/pmc_$i"
        echo "[gpu_tasks] pmc pass $i: $cs"
        timeout -s KILL 180 rocprofv3 --pmc $cs --output-format csv -d "/tmp/pmc_$i" -- python3 "$PMC_SCRIPT" > "$OUT/pmc_$i.log" 2>&1 || exit $?
        python3 tools/pmc_summary.py "/tmp/pmc_$i" > "$OUT/pmc_$i.json" || exit $?
      done
      ;;
    *) echo "[gpu_tasks] unknown task $t"; exit 2 ;;
  esac
done
echo "[gpu_tasks] done"

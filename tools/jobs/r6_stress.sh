# round-6 GPU job: the SHIPPING stream-GEMM hand-off (rel = 0) on every engine plan, 100,000
# poisoned varied-input repetitions each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_stress${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u tools/stream_handoff_stress.py --reps 100000 --rel 0 --out $O/handoff_rel0.jsonl \
  > $O/stress.log 2>&1 || { rc=$?; tail -20 $O/stress.log; exit $rc; }
cat $O/handoff_rel0.jsonl

# round-4 GPU job: 10,000-rep poisoned hand-off check of the weight-streaming kernel (rel 0 / 1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_handoff2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/splitk_check.py --reps ${REPS:-10000} --only stream --out $O/stream_handoff.jsonl > $O/log 2>&1 || { tail -20 $O/log; exit 1; }
cat $O/stream_handoff.jsonl

# round-5 GPU job: 100,000 poisoned reps of every production stream-GEMM split-K plan (shipped
# release form), then the unreleased form on the RoPE+KV and down cases for the record
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_stress${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 780 python -u tools/stream_handoff_stress.py --reps ${REPS:-100000} --rel 1 --out $O/rel1.jsonl > $O/rel1.log 2>&1 || { tail -20 $O/rel1.log; exit 1; }
cat $O/rel1.jsonl | cut -c1-200
timeout -k 10 300 python -u tools/stream_handoff_stress.py --reps ${REPS:-100000} --rel 0 --only "M32 " --out $O/rel0.jsonl > $O/rel0.log 2>&1 || { tail -20 $O/rel0.log; exit 1; }
cat $O/rel0.jsonl | cut -c1-200

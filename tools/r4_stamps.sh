set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_stamps
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/stream_stamps.py --out $O/stamps.jsonl > $O/stamps.log 2>&1 || { tail -30 $O/stamps.log; exit 1; }
cat $O/stamps.jsonl

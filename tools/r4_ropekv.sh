set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_ropekv
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ropekv_cost.py --M 256,512,1024,2048 --out $O/ropekv.jsonl > $O/ropekv.log 2>&1 || { tail -30 $O/ropekv.log; exit 1; }
cat $O/ropekv.jsonl

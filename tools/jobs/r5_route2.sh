# round-5 GPU job: in-engine A/B of the 129-256-row projection routing (rows_anatomy step times)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_route2${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
declare -A V
V[base]=''
V[pfq]='{"PF_MIDRANGE": ["gate_up", "qkv"]}'
V[pfqo]='{"PF_MIDRANGE": ["gate_up", "qkv", "o"]}'
V[pfqod]='{"PF_MIDRANGE": ["gate_up", "qkv", "o", "down"]}'
for rep in 1 2; do
for R in 256 192 144; do
for k in base pfq pfqo pfqod; do
PILOTTAI_ROUTING_JSON="${V[$k]}" timeout -k 10 240 python -u tools/rows_anatomy.py --rows $R --ctx 300 --steps 24 > $O/$k.$R.$rep.log 2>&1 || { tail -20 $O/$k.$R.$rep.log; exit 1; }
echo "$k R=$R rep=$rep $(grep -o '"step_ms": [0-9.]*' $O/$k.$R.$rep.log)"
done
done
done

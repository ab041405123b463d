# round-5 GPU job: in-engine A/B of the 64-row projection routing (rows_anatomy step times,
# alternating variants in separate engines)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_route${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
R=${ROWS:-64}
declare -A V
V[base]=''
V[sq6]='{"STREAM_CFG": {"qkv": [[32, [1,1,4,1,2,4]], [64, [1,1,6,1,4,4]]]}}'
V[sq4]='{"STREAM_CFG": {"qkv": [[32, [1,1,4,1,2,4]], [64, [1,1,4,1,4,4]]]}}'
V[mq4]='{"MID_CFG": {"qkv": [[32,1,2,2],[64,1,2,4],[128,2,2,1],[256,4,2,1],[1073741824,4,4,1]]}}'
for rep in 1 2; do
for k in base sq6 sq4 mq4; do
PILOTTAI_ROUTING_JSON="${V[$k]}" timeout -k 10 240 python -u tools/rows_anatomy.py --rows $R --ctx 600 --steps 32 > $O/$k.$rep.log 2>&1 || { tail -20 $O/$k.$rep.log; exit 1; }
echo "$k $rep $(grep step_ms $O/$k.$rep.log)"
done
done

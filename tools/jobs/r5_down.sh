# round-5 GPU job: down of 129-256-row steps on the 256x128 ping-pong kernel vs the stream kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_down${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
declare -A V
V[base]=''
V[dpf]='{"STREAM_CFG": {"down": [[32, [1,1,4,1,4,4]], [128, [1,2,4,1,8,2]]]}, "PF_MIDRANGE": ["gate_up", "down"]}'
for rep in 1 2; do
for k in base dpf; do
for R in 256 192 144; do
PILOTTAI_ROUTING_JSON="${V[$k]}" timeout -k 10 240 python -u tools/rows_anatomy.py --rows $R --ctx 300 --steps 24 > $O/$k.r$R.$rep.log 2>&1 || { tail -20 $O/$k.r$R.$rep.log; exit 1; }
echo "$k R=$R rep=$rep $(grep -o '"step_ms": [0-9.]*' $O/$k.r$R.$rep.log)"
done
done
done

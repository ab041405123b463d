# round-5 GPU job: gate_up of 65-128-row steps on the 256x128 ping-pong kernel vs the mid kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_g64${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
declare -A V
V[base]=''
V[g64]='{"PF_CFG": {"gate_up": [[64, "mid", {}], [256, "pf", {"bn": 128, "variant": 3}], [1073741824, "pf", {"bn": 256, "variant": 3}]]}}'
V[g96]='{"PF_CFG": {"gate_up": [[96, "mid", {}], [256, "pf", {"bn": 128, "variant": 3}], [1073741824, "pf", {"bn": 256, "variant": 3}]]}}'
for rep in 1 2; do
for k in base g64 g96; do
for R in 128 96 80; do
PILOTTAI_ROUTING_JSON="${V[$k]}" timeout -k 10 240 python -u tools/rows_anatomy.py --rows $R --ctx 600 --steps 24 > $O/$k.r$R.$rep.log 2>&1 || { tail -20 $O/$k.r$R.$rep.log; exit 1; }
echo "$k R=$R rep=$rep $(grep -o '"step_ms": [0-9.]*' $O/$k.r$R.$rep.log)"
done
done
done

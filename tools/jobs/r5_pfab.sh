# round-5 GPU job: in-engine A/B of the prefill-kernel family table (variant 1 3-stage 256x128
# vs the ping-pong 256x128 family) -- midrange rows_anatomy + headline bench, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_pfab${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
V3='"PF_CFG": {"qkv": [[80, "mid", {}], [1280, "pf", {"bn": 128, "variant": 3}], [2048, "pf", {"bn": 192, "variant": 3}], [3840, "pf", {"bn": 256, "variant": 3}], [1073741824, "pf", {"bn": 192, "variant": 3}]], "o": [[128, "mid", {}], [1073741824, "pf", {"bn": 128, "variant": 3}]], "gate_up": [[128, "mid", {}], [256, "pf", {"bn": 128, "variant": 3}], [1073741824, "pf", {"bn": 256, "variant": 3}]], "down": [[128, "mid", {}], [512, "pf", {"bn": 128, "variant": 3}], [1073741824, "pf", {"bn": 256, "variant": 3}]]}'
declare -A V
V[base]=''
V[v3]="{$V3}"
V[v3q]="{$V3, \"PF_MIDRANGE\": [\"gate_up\", \"qkv\"]}"
for rep in 1 2; do
for k in base v3 v3q; do
for R in 256 192; do
PILOTTAI_ROUTING_JSON="${V[$k]}" timeout -k 10 240 python -u tools/rows_anatomy.py --rows $R --ctx 300 --steps 24 > $O/$k.r$R.$rep.log 2>&1 || { tail -20 $O/$k.r$R.$rep.log; exit 1; }
echo "$k R=$R rep=$rep $(grep -o '"step_ms": [0-9.]*' $O/$k.r$R.$rep.log)"
done
done
done
for rep in 1 2 3; do
for k in base v3 v3q; do
PILOTTAI_ROUTING_JSON="${V[$k]}" timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > $O/$k.b.$rep.log 2>&1 || { tail -20 $O/$k.b.$rep.log; exit 1; }
echo "$k bench rep=$rep $(grep '"metric"' $O/$k.b.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['p50_task_latency_ms'])")"
done
done

# round-5 GPU job: stream kernel weights by plain loads (this build) vs non-temporal loads
# (tools/jobs/alt/_C_nt.so): phase stamps (member skew), then graph-timed stream bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_ntab${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
SO=pilottai_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/_C_new.so
for v in plain nt plain nt; do
if [ $v = nt ]; then cp tools/jobs/alt/_C_nt.so $SO; else cp /tmp/_C_new.so $SO; fi
timeout -k 10 300 python -u tools/stream_stamps.py --cases "down:64:4,1,1,4,1,4,4;down:128:8,1,1,8,1,8,4;qkv:64:4,1,1,6,1,4,4;o:64:4,1,1,4,1,4,4" --out $O/st_$v.jsonl > $O/st_$v.log 2>&1 || { tail -20 $O/st_$v.log; exit 1; }
done
python3 -c "
import json
for v in ('plain','nt'):
    for l in open('$O/st_'+v+'.jsonl'):
        d=json.loads(l); print(v, d['shape'], d['M'], d['us_per_call_graph'], d['loop_us'], d['barrier_wait_us'])"
cp /tmp/_C_new.so $SO

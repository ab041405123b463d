# round-4 GPU job: end-of-round marker-bounded 64-worker profile and the reply-128 bench on the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
WORKERS=64 bash tools/gpu_tasks.sh r4_endprof prof || exit 1
O=gpurun_out/r4_endprof
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --reply-tokens 128 > $O/reply128.log 2>&1 || { tail -20 $O/reply128.log; exit 1; }
grep '"metric"' $O/reply128.log | cut -c1-200

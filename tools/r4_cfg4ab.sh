# round-4 GPU job: config 4, same box, alternating: default batcher vs --memory-min-batch 16 --memory-wait-ms 10
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_cfg4ab
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for v in coal base; do
    X=""; [ $v = coal ] && X="--memory-min-batch 16 --memory-wait-ms 10"
    timeout -k 10 600 python -u bench.py --gpus 1 --steps 3 --warmup 1 --memory-rows 100000000 --embedder engine $X > $O/${v}_$rep.log 2>&1 || { tail -20 $O/${v}_$rep.log; exit 1; }
    echo "$v rep=$rep $(grep '"metric"' $O/${v}_$rep.log | tail -1 | cut -c120-175)"
  done
done

# round-4 GPU job: step-size cap A/B on the headline workload (2,048 vs 3,072 vs 4,096 tokens per step)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_mbt
mkdir -p $O
export TMPDIR=/tmp
for mbt in 4096 2048 3072; do
  timeout -k 10 420 python -u bench.py --gpus 1 --steps 3 --warmup 1 --max-batched-tokens $mbt > $O/mbt$mbt.log 2>&1 || { tail -20 $O/mbt$mbt.log; exit 1; }
  grep '"metric"' $O/mbt$mbt.log | cut -c1-200
done

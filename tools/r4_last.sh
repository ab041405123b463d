# round-4 GPU job: decode_part_target 384 vs 512 (same box, alternating), then config 4 on the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_last
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for t in 512 384; do
    PILOTTAI_DECODE_PART_TARGET=$t timeout -k 10 420 python -u bench.py --steps 3 --warmup 1 > $O/dpt${t}_$rep.log 2>&1 || { tail -20 $O/dpt${t}_$rep.log; exit 1; }
    echo "dpt=$t rep=$rep $(grep '"metric"' $O/dpt${t}_$rep.log | tail -1 | cut -c120-175)"
  done
done
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --memory-rows 100000000 --embedder engine > $O/cfg4.log 2>&1 || { tail -20 $O/cfg4.log; exit 1; }
echo "cfg4 $(grep '"metric"' $O/cfg4.log | tail -1 | cut -c120-175)"

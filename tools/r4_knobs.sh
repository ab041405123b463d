# round-4 GPU job: engine knob A/B on the headline workload, same box, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_knobs
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for k in base dpt1024 wide512 slack160; do
    E=""; X=""
    case $k in
      dpt1024) E="PILOTTAI_DECODE_PART_TARGET=1024" ;;
      wide512) X="--att-wide-min-tokens 512" ;;
      slack160) X="--align-slack 160" ;;
    esac
    env $E timeout -k 10 420 python -u bench.py --gpus 1 --steps 3 --warmup 1 $X > $O/${k}_$rep.log 2>&1 || { tail -20 $O/${k}_$rep.log; exit 1; }
    echo "$k rep=$rep $(grep '"metric"' $O/${k}_$rep.log | tail -1 | cut -c120-175)"
  done
done

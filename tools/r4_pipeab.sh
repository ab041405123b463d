# round-4 GPU job: pipelined decode tile loop (PILOTTAI_ATT_PIPE=1, default) vs the round-3 loop (0), same box, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_pipeab
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_attn_o_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PILOTTAI_ATT_PIPE=0 timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_pipe0.log 2>&1 || { tail -40 $O/tests_pipe0.log; exit 1; }
tail -1 $O/tests_pipe0.log
for rep in 1 2; do
  for p in 1 0; do
    for R in 64 128; do
      PILOTTAI_ATT_PIPE=$p timeout -k 10 300 python -u tools/rows_anatomy.py --rows $R --ctx 600 --steps 24 > $O/rows_${R}_$p_$rep.log 2>&1 || { tail -20 $O/rows_${R}_$p_$rep.log; exit 1; }
      echo "pipe=$p rep=$rep $(tail -1 $O/rows_${R}_$p_$rep.log)"
    done
  done
done
for rep in 1 2; do
  for p in 1 0; do
    PILOTTAI_ATT_PIPE=$p timeout -k 10 420 python -u bench.py --gpus 1 --steps 3 --warmup 1 > $O/bench_${p}_$rep.log 2>&1 || { tail -20 $O/bench_${p}_$rep.log; exit 1; }
    echo "bench pipe=$p rep=$rep $(tail -1 $O/bench_${p}_$rep.log | cut -c1-190)"
  done
done

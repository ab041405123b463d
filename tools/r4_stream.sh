# round-4 GPU job: stream GEMM numerics + benchmark (run through gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_stream${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_stream_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 900 python -u tools/stream_gemm_bench.py --M ${MLIST:-32,64,128,256} --sweep --rounds 3 --slabs uncached,cached_rel,cached --out $O/sweep.jsonl > $O/sweep.log 2>&1 || { tail -30 $O/sweep.log; exit 1; }
echo done

set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_stream4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_stream_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/stream_stamps.py --out $O/stamps.jsonl > $O/stamps.log 2>&1 || { tail -30 $O/stamps.log; exit 1; }
timeout -k 10 300 python -u tools/stream_stamps.py --rel 2 --out $O/stamps.jsonl > $O/stamps2.log 2>&1 || { tail -30 $O/stamps2.log; exit 1; }
timeout -k 10 900 python -u tools/stream_gemm_bench.py --M 8,16,32,64,128,256 --sweep --krot --rounds 3 --out $O/sweep.jsonl > $O/sweep.log 2>&1 || { tail -30 $O/sweep.log; exit 1; }
timeout -k 10 600 python -u tools/stream_gemm_bench.py --shapes lm_head --M 24,48,64,128,256 --sweep --rounds 3 --out $O/lm.jsonl > $O/lm.log 2>&1 || { tail -30 $O/lm.log; exit 1; }
echo done

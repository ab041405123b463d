set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_lm
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_stream_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u tools/stream_gemm_bench.py --shapes lm_head --M 144,192,256 --sweep --row-groups --rounds 3 --out $O/lm.jsonl > $O/lm.log 2>&1 || { tail -30 $O/lm.log; exit 1; }
cat $O/lm.jsonl | cut -c1-300

# round-5 GPU job: the TP step graph on custom collectives (new tests), the stream release cost
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_tp${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_custom_ar_gpu.py tests/test_tp_gpu.py tests/test_stream_gemm_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u tools/stream_gemm_bench.py --M 32,64,128,256 --shapes qkv,o,down --rel-ab --rounds 5 --out $O/rel_ab.jsonl > $O/rel_ab.log 2>&1 || { tail -20 $O/rel_ab.log; exit 1; }
cut -c1-300 $O/rel_ab.log

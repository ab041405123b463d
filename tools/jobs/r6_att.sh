# round-6 GPU job: attention (split prefill items) numerics + microbench, then the q16 scan
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_att${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k attention -x -v --timeout 200 --timeout-method thread \
  > $O/att_tests.log 2>&1 || { tail -40 $O/att_tests.log; exit 1; }
grep -E "passed|failed" $O/att_tests.log | tail -2
timeout -k 10 300 python -u tools/attn_bench.py --cases prefill2048,step2048,prefill4x512,mix --qcols 32,128 \
  --split-keys 0,512,1024 --iters 50 > $O/attn_bench.jsonl 2> $O/attn_bench.err || { tail -20 $O/attn_bench.err; exit 1; }
cat $O/attn_bench.jsonl
bash tools/jobs/r6_q16.sh

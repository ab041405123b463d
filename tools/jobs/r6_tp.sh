# round-6 GPU job: 70B dims on the hand kernels (TP=1, one packed copy), the TP engine at 2/4/8
# ranks on one GPU, config 5 at TP=1 (+ its kernel profile) and the TP=8 share-GPU rehearsal
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_tp${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -k 70b tests/test_tp_gpu.py -x -v -s --timeout 400 \
  --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED|greedy sequences|passed" $O/tests.log | tail -14
timeout -k 10 600 python -u benchmarks/workflow.py > $O/wf_tp1.log 2>&1 || { tail -20 $O/wf_tp1.log; exit 1; }
grep '"metric"' $O/wf_tp1.log > $O/wf_tp1.json && cut -c1-700 $O/wf_tp1.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_tp1 -o run -- python3 benchmarks/workflow.py \
  --workflows 8 --warmup 2 --clients 4 --no-fault > $O/prof_tp1.log 2>&1 || { tail -20 $O/prof_tp1.log; exit 1; }
find $O/prof_tp1 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/tp1_kernel_stats.csv
head -25 $O/tp1_kernel_stats.csv | cut -c1-200
PILOTTAI_DIST_BACKEND=gloo timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29551 benchmarks/workflow.py --share-gpu --clients 2 \
  --workflows 4 --warmup 1 --doc-words 120 --kv-gb 4 > $O/tp8.log 2>&1 || { tail -40 $O/tp8.log; exit 1; }
grep '"metric"' $O/tp8.log > $O/wf_tp8.json && cut -c1-900 $O/wf_tp8.json

# round-6 GPU job: config 5 (70B hierarchical workflow, TP=1 on the hand kernels) on the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_wf${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u benchmarks/workflow.py > $O/wf_tp1.log 2>&1 || { rc=$?; tail -20 $O/wf_tp1.log; exit $rc; }
grep '"metric"' $O/wf_tp1.log | tail -1 | cut -c1-400

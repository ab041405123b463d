# round-5 GPU job: the other BASELINE configs on the last tree -- config 5 (70B workflow,
# TP=1, fault injection) and HTTP serving (config 3's engine behind the OpenAI API)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_configs${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u benchmarks/workflow.py > $O/wf.log 2>&1 || { tail -20 $O/wf.log; exit 1; }
grep '"metric"' $O/wf.log | tail -1 > $O/wf.json
cut -c1-600 $O/wf.json
timeout -k 10 400 python -u benchmarks/http_serving.py > $O/http.log 2>&1 || { tail -20 $O/http.log; exit 1; }
grep '"metric"\|requests_per_s\|req' $O/http.log | tail -1 > $O/http.json
cut -c1-600 $O/http.json

# HTTP serving benchmark on one GPU (Llama-3-8B): 64 and 256 clients, free text and schema replies.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/http
timeout -k 10 300 python -u benchmarks/http_serving.py --clients 64 --requests 4 > gpurun_out/http/c64.log 2>&1 && \
timeout -k 10 300 python -u benchmarks/http_serving.py --clients 64 --requests 4 --schema > gpurun_out/http/c64_schema.log 2>&1 && \
timeout -k 10 400 python -u benchmarks/http_serving.py --clients 256 --requests 2 > gpurun_out/http/c256.log 2>&1
rc=$?
tail -qn1 gpurun_out/http/*.log
exit $rc

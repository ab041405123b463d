# round-4 GPU job: stream GEMM sweep + index checkpoint at 10M rows
set -o pipefail
cd "$GRAFT_REPO_ROOT"
RUN=2 bash tools/r4_stream.sh || exit $?
mkdir -p gpurun_out/r4_idx
df -h /tmp . > gpurun_out/r4_idx/df.txt 2>&1
timeout -k 10 600 python -u tools/index_ckpt_bench.py --rows 10000000 --out gpurun_out/r4_idx/ckpt.jsonl > gpurun_out/r4_idx/ckpt.log 2>&1 || { tail -20 gpurun_out/r4_idx/ckpt.log; exit 1; }
echo job2 done

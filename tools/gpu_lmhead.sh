# LM head (and the other decode shapes) at 48 / 64 rows: packed decode kernel vs hipBLASLt.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lmh
timeout -k 10 400 python -u tools/decode_gemm_bench.py 24,48,64 > gpurun_out/lmh/decode_sweep.jsonl 2> gpurun_out/lmh/decode_sweep.err
echo EXIT $?

# Repeat the decode-GEMM GPU tests (split-K QKV+RoPE included) to quantify the one
# mismatch seen this round in test_decode_qkv_rope[9-32-8-4096-3].
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/flake
: > gpurun_out/flake/summary.txt
for i in $(seq 1 12); do
  timeout -k 10 120 python -u -m pytest tests/test_kernels_gpu.py -q -k "decode" --timeout 60 --timeout-method thread > gpurun_out/flake/run_$i.log 2>&1
  echo "run $i exit $? $(tail -1 gpurun_out/flake/run_$i.log)" >> gpurun_out/flake/summary.txt
done
echo EXIT 0

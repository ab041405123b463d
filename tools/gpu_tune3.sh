# TunableOp for the 16-token library buckets added above 256 (272-496, odd multiples of 16).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tune3
PILOTTAI_NO_TUNED_GEMM=1 timeout -k 10 600 python -u tools/tune_gemms.py --model llama-3-8b --out gpurun_out/tune3/t.csv \
  --ms 272,304,336,368,400,432,464,496 --duration-ms 150 > gpurun_out/tune3/tune.jsonl 2> gpurun_out/tune3/tune.err
echo EXIT $?

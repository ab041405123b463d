# Re-tune the library-path projection GEMMs (steps of 288-2048 tokens) with a longer
# TunableOp search window per shape; the results are merged offline (tools/merge_tuned.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tune2
PILOTTAI_NO_TUNED_GEMM=1 timeout -k 10 900 python -u tools/tune_gemms.py --model llama-3-8b --out gpurun_out/tune2/t.csv \
  --ms 288,320,352,384,416,448,480,512,576,640,704,768,832,896,960,1024,1088,1152,1216,1280,1344,1408,1472,1536,1600,1664,1728,1792,1856,1920,1984,2048 \
  --duration-ms 150 > gpurun_out/tune2/tune.jsonl 2> gpurun_out/tune2/tune.err
echo EXIT $?

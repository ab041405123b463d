# Probe: MLP of 9-16-row decode steps on the mid kernels (PILOTTAI_DECODE_MID_MLP=1) vs the
# decode kernels: engine GPU tests with the probe on, then 8/16-worker bench alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dmlp
PILOTTAI_DECODE_MID_MLP=1 timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -q --timeout 180 --timeout-method thread > gpurun_out/dmlp/pytest.log 2>&1 || exit $?
for r in 1 2; do
  for v in 1 0; do
    PILOTTAI_DECODE_MID_MLP=$v timeout -k 10 300 python -u bench.py --workers 8 --steps 6 --warmup 1 > gpurun_out/dmlp/w8_v${v}_r${r}.json 2> gpurun_out/dmlp/w8_v${v}_r${r}.err || exit $?
    PILOTTAI_DECODE_MID_MLP=$v timeout -k 10 300 python -u bench.py --workers 16 --steps 4 --warmup 1 > gpurun_out/dmlp/w16_v${v}_r${r}.json 2> gpurun_out/dmlp/w16_v${v}_r${r}.err || exit $?
  done
done
echo EXIT 0

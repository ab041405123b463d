# 32-row mid tiles in the engine (new MID_CFG) vs the previous MID_CFG (llama.py edited in the
# box's scratch copy): 16- and 8-worker bench alternating; then the fused sweep at 96/128 rows.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fm1b
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -q --timeout 180 --timeout-method thread > gpurun_out/fm1b/pytest.log 2>&1 || exit $?
cp pilottai_amd/models/llama.py /tmp/llama_new.py
python3 - <<'PY'
s = open("/tmp/llama_new.py").read()
s = s.replace('"qkv": [(32, 1, 2, 2), (64, 1, 2, 1), ', '"qkv": [(64, 2, 2, 2), ')
s = s.replace('"o": [(32, 1, 2, 4), (64, 1, 2, 2), ', '"o": [(64, 2, 2, 4), ')
s = s.replace('"gate_up": [(32, 1, 4, 1), ', '"gate_up": [')
s = s.replace('"down": [(32, 1, 2, 4), ', '"down": [')
open("/tmp/llama_old.py", "w").write(s)
PY
for r in 1 2; do
  for v in new old; do
    cp /tmp/llama_$v.py pilottai_amd/models/llama.py || exit 1
    timeout -k 10 300 python -u bench.py --workers 16 --steps 4 --warmup 1 > gpurun_out/fm1b/w16_${v}_r${r}.json 2> gpurun_out/fm1b/w16_${v}_r${r}.err || exit $?
    timeout -k 10 300 python -u bench.py --workers 8 --steps 6 --warmup 1 > gpurun_out/fm1b/w8_${v}_r${r}.json 2> gpurun_out/fm1b/w8_${v}_r${r}.err || exit $?
  done
done
cp /tmp/llama_new.py pilottai_amd/models/llama.py
timeout -k 10 600 python -u tools/mid_gemm_bench.py 96,128 --fused-sweep > gpurun_out/fm1b/sweep96.jsonl 2> gpurun_out/fm1b/sweep96.err
echo EXIT $?

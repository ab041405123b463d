# Wide path: O projection on the decode kernel up to 32 rows (new) vs the wide kernel (old;
# llama.py edited in the box's scratch copy). GPU test tier first.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wo
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > gpurun_out/wo/pytest_gpu.log 2>&1 || exit $?
cp pilottai_amd/models/llama.py /tmp/llama_new.py
python3 - <<'PY'
s = open("/tmp/llama_new.py").read()
s = s.replace("elif T <= 32:  # O + residual on the decode kernel", "elif T <= 0:  # O + residual on the decode kernel")
open("/tmp/llama_old.py", "w").write(s)
PY
for r in 1 2; do
  for v in new old; do
    cp /tmp/llama_$v.py pilottai_amd/models/llama.py || exit 1
    timeout -k 10 300 python -u bench.py --workers 16 --steps 4 --warmup 1 > gpurun_out/wo/w16_${v}_r${r}.json 2> gpurun_out/wo/w16_${v}_r${r}.err || exit $?
  done
done
cp /tmp/llama_new.py pilottai_amd/models/llama.py
echo EXIT 0

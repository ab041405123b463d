# Graph bucket granularity: 16-token buckets from 80 to 512 (engine.py edited in the box's
# scratch copy) vs the default 32-token ones, 64 workers, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/buckets
cp pilottai_amd/engine/engine.py /tmp/engine_old.py
python3 - <<'PY'
s = open("/tmp/engine_old.py").read()
old = "DEFAULT_BUCKETS = ([8, 16, 32, 48, 64] + list(range(96, 513, 32))"
assert old in s
s = s.replace(old, "DEFAULT_BUCKETS = ([8, 16, 32, 48, 64, 80] + list(range(96, 513, 16))")
open("/tmp/engine_new.py", "w").write(s)
PY
for r in 1 2; do
  for v in new old; do
    cp /tmp/engine_$v.py pilottai_amd/engine/engine.py || exit 1
    timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/buckets/w64_${v}_r${r}.json 2> gpurun_out/buckets/w64_${v}_r${r}.err || exit $?
  done
done
cp /tmp/engine_old.py pilottai_amd/engine/engine.py
echo EXIT 0

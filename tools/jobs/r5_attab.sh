# round-5 GPU job: decode-attention latency change (first-tile page ids with the item loads,
# one-pass partition merge) -- numerics with the new build, then old / new alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_attab${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
SO=pilottai_amd/_C.cpython-310-x86_64-linux-gnu.so
cp pilottai_amd/_C_new.so $SO
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
for v in old new; do
cp pilottai_amd/_C_$v.so $SO
for R in 8 64; do
timeout -k 10 240 python -u tools/rows_anatomy.py --rows $R --ctx 600 --steps 32 > $O/$v.$R.$rep.log 2>&1 || { tail -20 $O/$v.$R.$rep.log; exit 1; }
echo "$v R=$R rep=$rep $(grep step_ms $O/$v.$R.$rep.log)"
done
done
done
cp pilottai_amd/_C_new.so $SO

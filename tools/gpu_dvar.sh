# (1) attention numerics with the page-window build, (2) decode-GEMM variant A/B (kernel
# microbench, interleaved in one process), (3) attention old/new builds on the microbench,
# (4) 8-worker bench: new attention with decode variants 0/1, old attention, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dvar
SO=pilottai_amd/_C.cpython-310-x86_64-linux-gnu.so
cp ab/_C_new.so $SO || exit 1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 180 --timeout-method thread > gpurun_out/dvar/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/decode_variant_ab.py --variants 0,1 --ms 8,16,32 > gpurun_out/dvar/kernel_ab.jsonl 2> gpurun_out/dvar/kernel_ab.err || exit $?
for r in 1 2; do
  for v in new old; do
    cp ab/_C_$v.so $SO || exit 1
    timeout -k 10 200 python -u tools/attn_bench.py --small > gpurun_out/dvar/attn_small_${v}_$r.jsonl 2>&1 || exit $?
    timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/dvar/attn_${v}_$r.jsonl 2>&1 || exit $?
  done
done
for r in 1 2; do
  for arm in new0 old0 new1; do
    v=${arm:3:1}; b=${arm:0:3}
    cp ab/_C_$b.so $SO || exit 1
    PILOTTAI_DECODE_VARIANT=$v timeout -k 10 300 python -u bench.py --workers 8 --steps 6 --warmup 1 > gpurun_out/dvar/w8_${arm}_r${r}.json 2> gpurun_out/dvar/w8_${arm}_r${r}.err || exit $?
  done
done
cp ab/_C_new.so $SO
echo EXIT 0

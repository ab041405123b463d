# 8-worker bench (per-GPU load of the 8-GPU run) under different interpreter switch
# intervals, then a kernel trace of the default for the step-boundary idle distribution.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/gil
P=/tmp/pilottai_gaps
rm -rf $P && mkdir -p $P
for sw in 0 0.0002 0.00005 0.001; do
  if [ "$sw" = "0" ]; then unset PILOTTAI_GIL_SWITCH_S; else export PILOTTAI_GIL_SWITCH_S=$sw; fi
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --workers 8 > gpurun_out/gil/w8_sw$sw.log 2>&1 || exit 1
done
unset PILOTTAI_GIL_SWITCH_S
timeout -k 10 400 rocprofv3 --kernel-trace -d $P/w8 -o w8 -- python3 bench.py --steps 3 --warmup 1 --workers 8 > gpurun_out/gil/w8_prof.log 2>&1 && \
python3 tools/gap_analysis.py "$P/w8/**/*.db" --after-frac 0.5 > gpurun_out/gil/w8_gaps_default.jsonl 2>&1 && \
export PILOTTAI_GIL_SWITCH_S=0.0002 && \
timeout -k 10 400 rocprofv3 --kernel-trace -d $P/w8b -o w8b -- python3 bench.py --steps 3 --warmup 1 --workers 8 > gpurun_out/gil/w8b_prof.log 2>&1 && \
python3 tools/gap_analysis.py "$P/w8b/**/*.db" --after-frac 0.5 > gpurun_out/gil/w8_gaps_sw0.0002.jsonl 2>&1
echo EXIT $?

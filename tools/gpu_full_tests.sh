# Full GPU test tier + smoke, then the 2,048-token prefill step anatomy profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/full gpurun_out/anat
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/full/pytest_gpu.log 2>&1 && \
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/anat/prof -o a -- python3 tools/step_anatomy.py --seqs 4 --new 512 --cached 256 --reps 6 > gpurun_out/anat/run.log 2>&1
echo EXIT $?

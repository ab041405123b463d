# Kernel anatomy of the 2,048-token prefill step (4 x 512 new tokens on a 256-token cached prefix).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/anat
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/anat/prof -o a -- python3 tools/step_anatomy.py --seqs 4 --new 512 --cached 256 --reps 6 > gpurun_out/anat/run.log 2>&1
echo EXIT $?

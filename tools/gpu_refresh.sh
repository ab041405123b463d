# Refresh: per-rank loads of the N=2/4/8 runs on one GPU, kernel profile of the 8-worker case,
# and a 2-rank shared-GPU rehearsal of the multi-rank bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_scalesim.sh | grep -q "EXIT 0" && bash tools/gpu_rehearse2.sh
echo EXIT $?

set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/splitk
timeout -k 10 300 python -u tools/splitk_check.py --reps 100 > gpurun_out/splitk/check.jsonl 2> gpurun_out/splitk/check.err
echo EXIT $?

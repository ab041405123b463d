# round-4 GPU job: marker-bounded kernel anatomy of prefill-heavy steps (2,048 / 1,024 / 512 tokens)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_stepanat
mkdir -p $O
export TMPDIR=/tmp
for SN in 4,512 2,512 8,128 1,512; do
  S=${SN%,*}; N=${SN#*,}
  P=/tmp/pilottai_step_${S}_$N
  rm -rf "$P" && mkdir -p "$P"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$P" -o s -- python3 tools/step_anatomy.py --seqs $S --new $N --cached 512 --reps 6 > $O/step_${S}_$N.log 2>&1 || { tail -30 $O/step_${S}_$N.log; exit 1; }
  python3 tools/prof_summary.py "$P"/*/*.db "$P"/*.db --between-markers --top 14 > "$O/step_${S}_${N}_kernels.md" 2>&1 || { tail -20 $O/step_${S}_${N}_kernels.md; exit 1; }
  tail -1 $O/step_${S}_$N.log | cut -c1-120
  sed -n 7,20p $O/step_${S}_${N}_kernels.md | cut -c1-120
done

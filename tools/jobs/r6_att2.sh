# round-6 GPU job: split prefill items where they can pay (few long items), then the q16 tier
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_att2${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/attn_bench.py --cases cont256x4096,cont2x256x2048,cont512x3072,prefill4x512 \
  --qcols 32,128 --split-keys 0,512,1024 > $O/attn_bench.jsonl 2> $O/attn_bench.err || { tail -20 $O/attn_bench.err; exit 1; }
cat $O/attn_bench.jsonl
bash tools/jobs/r6_q16.sh

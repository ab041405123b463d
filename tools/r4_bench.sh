# round-4 GPU job: headline bench, 8-worker bench, reply-128 bench, hybrid 8-rank rehearsal
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_bench${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 420 python -u bench.py --gpus 1 --steps 3 --warmup 1 $BENCH_ARGS > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
timeout -k 10 420 python -u bench.py --workers 8 --steps 3 --warmup 1 $BENCH_ARGS > $O/bench_w8.log 2>&1 || { tail -20 $O/bench_w8.log; exit 1; }
tail -1 $O/bench_w8.log | cut -c1-300
PILOTTAI_DIST_BACKEND=gloo timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 --steps 3 --warmup 1 --hybrid-latency 0.08 > $O/hybrid.log 2>&1 || { tail -30 $O/hybrid.log; exit 1; }
grep '"metric"' $O/hybrid.log | cut -c1-300
echo bench done

# round-5 GPU job: config 4 with the index writes and the embedding projection on their own
# streams (this tree) vs on the default stream behind the engine's steps (the previous files,
# copied in for the run), alternating; memory GPU tests first
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_memstream${RUN:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_runtime_engine.py tests/test_memory_loop.py tests/test_index_checkpoint.py -m gpu -x -q --timeout 120 --timeout-method thread -k "embed or index or memory or cosine or topk" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
F="memory/batcher.py memory/enhanced_memory.py memory/embedding.py memory/semantic_index.py"
mkdir -p /tmp/new
for f in $F; do cp pilottai_amd/$f /tmp/new/$(basename $f); done
for rep in 1 2; do
for v in new old; do
for f in $F; do b=$(basename $f .py); if [ $v = old ]; then cp tools/jobs/alt/${b}_prev.py pilottai_amd/$f; else cp /tmp/new/$b.py pilottai_amd/$f; fi; done
timeout -k 10 500 python -u bench.py --memory-rows 100000000 --embedder engine --steps 3 --warmup 1 > $O/$v.$rep.log 2>&1 || { tail -20 $O/$v.$rep.log; exit 1; }
echo "$v rep=$rep $(grep '"metric"' $O/$v.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['memory']; print(d['value'], d['p50_task_latency_ms'], m['lookup_p50_ms'], m['lookup_p99_ms'], m['passes'], m.get('lookup_anatomy_ms'))")"
done
done
for f in $F; do cp /tmp/new/$(basename $f) pilottai_amd/$f; done

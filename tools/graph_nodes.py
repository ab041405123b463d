"""Kernel launches per layer of the engine's captured step graphs (the
launch count per 70B layer in the TP step graph). Builds the engine twice -- 1 and 2 layers of
the model's exact layer shape -- captures every bucket with keep_graph=True and counts each
graph's nodes by type (utils/tracing.py graph_node_counts): per layer = N(2 layers) - N(1).

    python tools/graph_nodes.py --model llama-3-70b                   # TP = 1
    PILOTTAI_DIST_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 \\
        --master-addr 127.0.0.1 tools/graph_nodes.py --model llama-3-70b --share-gpu   # TP = 2
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="llama-3-70b")
ap.add_argument("--buckets", default="8,64,512,2048")
ap.add_argument("--share-gpu", action="store_true")
ap.add_argument("--packed", type=int, default=-1, help="1 / 0 force the packed (fused) path; -1 model default")
ap.add_argument("--out", default="")
a = ap.parse_args()

from pilottai_amd.engine.engine import EngineConfig, LLMEngine  # noqa: E402
from pilottai_amd.parallel import comm  # noqa: E402
from pilottai_amd.utils.tracing import graph_node_counts  # noqa: E402

rank, world, local = comm.init_distributed()
tp = comm.new_tp_groups(world, custom_ar=True if a.share_gpu else None)
dev = torch.device("cuda", 0 if a.share_gpu else local)
torch.cuda.set_device(dev)
buckets = [int(b) for b in a.buckets.split(",")]
counts = {}
for nl in (1, 2):
    eng = LLMEngine(EngineConfig(model=f"{a.model}-{nl}l", max_num_seqs=64, max_num_batched_tokens=max(buckets),
                                 kv_cache_gb=2.0, token_buckets=buckets, keep_graphs=True,
                                 decode_fused=None if a.packed < 0 else bool(a.packed)),
                    device=dev, tp=tp)
    counts[nl] = {b: graph_node_counts(eng._graphs[(b, False, False)]) for b in buckets}
    packed = eng.model.decode_packed
    eng.release_followers()
    del eng
    torch.cuda.empty_cache()
if rank == 0:
    for b in buckets:
        c1, c2 = counts[1][b], counts[2][b]
        rec = {"model": a.model, "tp": world, "bucket": b, "packed": packed,
               "kernels_per_layer": c2.get("kernel", 0) - c1.get("kernel", 0),
               "nodes_per_layer": sum(c2.values()) - sum(c1.values()),
               "outside_layers_kernels": 2 * c1.get("kernel", 0) - c2.get("kernel", 0),
               "graph_1l": c1, "graph_2l": c2}
        line = json.dumps(rec)
        print(line, flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(line + "\n")
if world > 1:
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()

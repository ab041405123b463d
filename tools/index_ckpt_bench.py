"""Checkpoint / resume of a large HBM semantic store (VERDICT r3 missing #1, item 7).

Fills a SemanticIndex of --rows x 1024 bf16 rows on the GPU (random unit vectors, priorities
and tag masks, as bench.py --memory-rows does), runs a batch of filtered top-k searches, saves
the index with SemanticIndex.save (chunked D2H through one pinned buffer into .npy shards),
drops it, restores it with SemanticIndex.load and repeats the searches: rows and scores must
be bit-identical. Prints one JSON line with the save / load seconds and GB/s.

    python tools/index_ckpt_bench.py [--rows 10000000] [--dir /tmp/idx_ckpt] [--out file.jsonl]
"""
import argparse
import json
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--dir", default="/tmp/pilottai_idx_ckpt")
    ap.add_argument("--queries", type=int, default=64)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import numpy as np
    import torch

    from pilottai_amd.memory.semantic_index import SemanticIndex

    dev = torch.device("cuda", 0)
    dim = 1024
    t0 = time.perf_counter()
    idx = SemanticIndex(dim=dim, capacity=a.rows, device=dev, growable=False)
    g = torch.Generator(device=dev).manual_seed(7)
    tags = [idx.tags.bit(t) for t in ("archive", "finance", "ops", "legal")]
    done = 0
    while done < a.rows:
        m = min(1 << 20, a.rows - done)
        v = torch.randn(m, dim, device=dev, generator=g, dtype=torch.float32)
        pr = torch.randint(0, 3, (m,), device=dev, dtype=torch.int32, generator=g)
        tb = (1 << tags[0]) | (1 << torch.randint(1, 4, (m,), device=dev, generator=g)).to(torch.int64)
        idx.add_device(v, pr, tb)
        done += m
    torch.cuda.synchronize(dev)
    fill_s = time.perf_counter() - t0
    rng = np.random.default_rng(3)
    q = rng.standard_normal((a.queries, dim)).astype(np.float32)
    minp = [i % 3 for i in range(a.queries)]
    qt = [("archive",) if i % 2 else ("finance",) for i in range(a.queries)]
    before = idx.search(q, 5, minp, qt)
    free = shutil.disk_usage(os.path.dirname(a.dir) or "/").free
    need = idx.count * dim * 2 + idx.count * 16
    if free < need * 1.1:
        raise SystemExit(f"not enough disk under {os.path.dirname(a.dir)}: {free / 1e9:.1f} GB free, "
                         f"{need / 1e9:.1f} GB needed")
    save = idx.save(a.dir)
    del idx
    torch.cuda.empty_cache()
    t1 = time.perf_counter()
    back = SemanticIndex.load(a.dir, device=dev, growable=False)
    load_s = time.perf_counter() - t1
    after = back.search(q, 5, minp, qt)
    rec = {"rows": a.rows, "dim": dim, "bytes": save["bytes"], "fill_s": round(fill_s, 2),
           "save_s": round(save["seconds"], 2), "save_GBps": round(save["GBps"], 2),
           "load_s": round(load_s, 2), "load_GBps": round(save["bytes"] / load_s / 1e9, 2),
           "topk_identical": after == before, "queries": a.queries}
    print(json.dumps(rec), flush=True)
    if a.out:
        with open(a.out, "a") as f:
            f.write(json.dumps(rec) + "\n")
    shutil.rmtree(a.dir, ignore_errors=True)
    if not rec["topk_identical"]:
        raise SystemExit("top-k after restore differs")


if __name__ == "__main__":
    main()

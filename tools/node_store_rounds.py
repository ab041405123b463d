"""Round overhead of NodeSemanticStore at W gloo CPU ranks.

Every rank holds a shard of ROWS/W rows (dim 1024) and submits Q queries per round (k = 64) for
R rounds; reports per-round wall time, the scan's share, and the overhead outside the scan
(collectives, packing, merge), plus what an idle round costs.

    python tools/node_store_rounds.py --world 8 --queries 64 --rounds 20
"""
import argparse
import json
import os
import socket
import time

import sys

import numpy as np
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, world, port, a, q):
    import torch
    import torch.distributed as dist

    torch.set_num_threads(1)
    from pilottai_amd.memory.node_store import NodeSemanticStore
    from pilottai_amd.memory.semantic_index import SemanticIndex

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = np.random.default_rng(rank)
    n = a.rows // world
    idx = SemanticIndex(dim=a.dim, capacity=n, device="cpu")
    idx.add(g.standard_normal((n, a.dim)).astype(np.float32), [0] * n, [()] * n, [None] * n)
    store = NodeSemanticStore(idx, group=dist.new_group(backend="gloo"), max_queries=a.queries)
    store.start()
    qs = g.standard_normal((a.queries, a.dim)).astype(np.float32)
    store.search_rows_blocking(qs, a.k, [0] * a.queries, [()] * a.queries)  # warm-up round
    dist.barrier()
    s0 = dict(store.stats)
    w0 = store._host.waited_s
    t0 = time.perf_counter()
    for _ in range(a.rounds):
        store.search_rows_blocking(qs, a.k, [0] * a.queries, [()] * a.queries)
    wall = time.perf_counter() - t0
    s1 = dict(store.stats)
    waited = store._host.waited_s - w0
    dist.barrier()
    # idle: time a burst of idle rounds (every rank idle)
    i0 = store.stats["idle_rounds"]
    time.sleep(1.0)
    idle_n = store.stats["idle_rounds"] - i0
    store.stop()
    rounds = s1["rounds"] - s0["rounds"]
    q.put((rank, {"rounds": rounds, "wall_ms_per_round": 1e3 * wall / a.rounds,
                  "round_ms": 1e3 * (s1["round_s"] - s0["round_s"]) / max(1, rounds),
                  "scan_ms": 1e3 * (s1["scan_s"] - s0["scan_s"]) / max(1, rounds),
                  "peer_wait_ms": 1e3 * waited / max(1, rounds),
                  "idle_rounds_per_s": idle_n}))
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--queries", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--rows", type=int, default=80000)
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_entry, args=(r, a.world, port, a, q)) for r in range(a.world)]
    for p in ps:
        p.start()
    got = {}
    while len(got) < a.world:
        try:
            r, v = q.get(timeout=5)
            got[r] = v
        except Exception:  # noqa: BLE001
            if any(p.exitcode not in (None, 0) for p in ps):
                raise SystemExit("a rank failed")
    for p in ps:
        p.join(60)
    per = [got[r] for r in range(a.world)]
    rec = {"world": a.world, "queries_per_rank": a.queries, "k": a.k, "rows": a.rows, "dim": a.dim,
           "round_ms_max": round(max(p["round_ms"] for p in per), 3),
           "scan_ms_max": round(max(p["scan_ms"] for p in per), 3),
           "overhead_ms_max": round(max(p["round_ms"] - p["scan_ms"] for p in per), 3),
           # the round's own host work: without the scan and without waiting for slower peers
           # (on this oversubscribed 8-CPU container the peers' CPU scans skew by 10-30 ms)
           "own_overhead_ms_max": round(max(p["round_ms"] - p["scan_ms"] - p["peer_wait_ms"] for p in per), 3),
           "transport": "shm" if os.environ.get("PILOTTAI_HOST_GATHER") != "gloo" else "gloo",
           "wall_ms_per_round": round(max(p["wall_ms_per_round"] for p in per), 3),
           "idle_rounds_per_s": min(p["idle_rounds_per_s"] for p in per), "backend": "gloo-cpu"}
    print(json.dumps(rec))
    if a.out:
        with open(a.out, "a") as f:
            f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()

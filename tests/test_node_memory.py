"""The node-wide semantic store (memory/node_store.py) over gloo ranks on
CPU: rows sharded over the ranks, lockstep rounds on a dedicated group, replicated items.

* top-k from every rank equals ONE SemanticIndex holding all rows (same global row ids, same
  scores), including the tag, priority and expiry filters;
* a write made on rank A is returned to a search from rank B;
* the asyncio API (EnhancedMemory-shaped: search_batch / store_semantic_batch) returns the
  replicated MemoryItems, ordered like EnhancedMemory, fallback text for bulk rows.
"""
import asyncio
import os
import socket
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

from pilottai_amd.memory.semantic_index import SemanticIndex

N, DIM = 1203, 64
QMIN = [0, 0, 2, 0, 3, 0, 0, 1]
QTAGS = [(), ("even",), (), ("odd",), ("even",), (), ("rare",), ("odd", "x3")]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data():
    g = np.random.default_rng(0)
    vecs = g.standard_normal((N, DIM)).astype(np.float32)
    prio = [int(i % 5) for i in range(N)]
    tags = [({"even"} if i % 2 == 0 else {"odd"}) | ({"x3"} if i % 3 == 0 else set()) |
            ({"rare"} if i % 97 == 0 else set()) for i in range(N)]
    # rows 5, 15, 25, ... expired an hour ago; the rest never expire
    exp = [time.time() - 3600 if i % 10 == 5 else None for i in range(N)]
    queries = np.random.default_rng(1).standard_normal((len(QMIN), DIM)).astype(np.float32)
    return vecs, prio, tags, exp, queries


def _entry(rank, world, port, q):
    import torch.distributed as dist

    from pilottai_amd.memory.enhanced_memory import MemoryItem
    from pilottai_amd.memory.node_store import NodeSemanticStore

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        vecs, prio, tags, exp, queries = _data()
        local = SemanticIndex(dim=DIM, capacity=64, device="cpu")
        mine = list(range(rank, N, world))  # global row g = local_row * world + rank
        local.add(vecs[mine], [prio[i] for i in mine], [tags[i] for i in mine], [exp[i] for i in mine])
        grp = dist.new_group(backend="gloo")
        store = NodeSemanticStore(local, group=grp, fallback_text=lambda g: f"archived {g}")
        store.start()
        out = {"rows": local.count}
        # 1) raw top-k from this rank (every rank asks the same queries)
        out["topk"] = store.search_rows_blocking(queries, 6, QMIN, QTAGS)
        dist.barrier()
        # 2) rank world-1 writes a finding; rank 0 finds it
        probe = queries[0] * 3.0
        if rank == world - 1:
            out["written"] = store.store_rows_blocking(
                probe[None], [MemoryItem(text="finding from the last rank", tags={"fresh"}, priority=4)])[0]
        dist.barrier()
        if rank == 0:
            out["probe"] = store.search_rows_blocking(probe[None], 3, [0], [("fresh",)])[0]

        # 3) the asyncio API from every rank at once
        async def api():
            rows = await store.store_semantic_batch([f"note from rank {rank}"], [{"r": rank}], [{"notes"}], [2])
            hits = await store.search_batch([f"note from rank {rank}"], tags=[{"notes"}], limit=world)
            any_hits = await store.search_batch(["archived document"], limit=3)
            return rows, [(h.text, h.metadata) for h in hits[0]], [h.text for h in any_hits[0]]

        out["api"] = asyncio.run(api())
        dist.barrier()
        store.stop()
        out["items"] = len(store.items)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_node_store_equals_one_index_and_shares_writes(world):
    vecs, prio, tags, exp, queries = _data()
    single = SemanticIndex(dim=DIM, capacity=2048, device="cpu")
    single.add(vecs, prio, tags, exp)
    ref = single.search(queries, 6, QMIN, QTAGS)

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # the node holds N rows in total, not N per rank
    assert sum(got[r]["rows"] for r in range(world)) == N
    for r in range(world):
        for lst_s, lst_r in zip(got[r]["topk"], ref):
            assert [row for row, _ in lst_s] == [row for row, _ in lst_r]
            np.testing.assert_allclose([s for _, s in lst_s], [s for _, s in lst_r], rtol=1e-6, atol=1e-6)
    # the filters really filtered: expired rows never, tags and priorities respected
    for qi, lst in enumerate(got[0]["topk"]):
        for row, _ in lst:
            assert row % 10 != 5 and prio[row] >= QMIN[qi] and set(QTAGS[qi]) <= tags[row]
    # a write on the last rank, read from rank 0
    w = got[world - 1]["written"]
    assert w % world == world - 1 and got[0]["probe"][0][0] == w
    # asyncio API: each rank's own note comes back with its metadata; bulk rows via fallback
    for r in range(world):
        rows, hits, any_hits = got[r]["api"]
        assert rows[0] % world == r
        assert ("note from rank %d" % r, {"r": r}) in hits
        assert len(any_hits) == 3 and all(t.startswith(("archived ", "note ", "finding ")) for t in any_hits)
    # every rank holds every replicated item (the probe + one note per rank)
    assert all(got[r]["items"] == world + 1 for r in range(world))


def test_node_store_single_rank_without_collectives():
    """world 1 (no process group): the same API over the local index."""
    from pilottai_amd.memory.enhanced_memory import MemoryItem
    from pilottai_amd.memory.node_store import NodeSemanticStore

    vecs, prio, tags, exp, queries = _data()
    idx = SemanticIndex(dim=DIM, capacity=2048, device="cpu")
    idx.add(vecs, prio, tags, exp)
    store = NodeSemanticStore(idx)
    store.start()
    try:
        assert store.search_rows_blocking(queries, 6, QMIN, QTAGS) == idx.search(queries, 6, QMIN, QTAGS)
        g = store.store_rows_blocking(queries[:1] * 2, [MemoryItem(text="mine", tags={"m"})])[0]
        assert g == N and store.search_rows_blocking(queries[:1], 1, [0], [("m",)])[0][0][0] == N
    finally:
        store.stop()


def test_both_stores_implement_the_store_protocol():
    """The batcher's keyword contract (vecs=, ...) is the same on both stores (round 5 shipped a
    node store without `vecs=`, and every node-mode write failed)."""
    from pilottai_amd.memory.enhanced_memory import EnhancedMemory
    from pilottai_amd.memory.node_store import NodeSemanticStore
    from pilottai_amd.memory.store_protocol import signature_mismatches

    assert signature_mismatches(EnhancedMemory) == []
    assert signature_mismatches(NodeSemanticStore) == []


class _FakeEngine:
    """add/remove_step_listener plus a thread that announces a heavy (2,048-token) step every
    5 ms, like LLMEngine's step listeners (the batcher's engine gate)."""

    def __init__(self):
        import threading

        self.listeners = []
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def add_step_listener(self, fn):
        self.listeners = self.listeners + [fn]

    def remove_step_listener(self, fn):
        self.listeners = [f for f in self.listeners if f is not fn]

    def _run(self):
        while not self._stop.wait(0.005):
            for fn in self.listeners:
                fn(2048)

    def close(self):
        self._stop.set()
        self._t.join(5)


def _batcher_entry(rank, world, port, q):
    import torch.distributed as dist

    from pilottai_amd.core.agent import BaseAgent
    from pilottai_amd.core.task import Task
    from pilottai_amd.memory.batcher import MemoryLookupBatcher
    from pilottai_amd.memory.embedding import HashingEmbedder
    from pilottai_amd.memory.node_store import NodeSemanticStore

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = _FakeEngine()
    try:
        emb = HashingEmbedder(DIM)
        local = SemanticIndex(dim=DIM, capacity=64, device="cpu")
        grp = dist.new_group(backend="gloo")
        store = NodeSemanticStore(local, embedder=emb, group=grp)
        store.start()
        out = {}

        async def run():
            batcher = MemoryLookupBatcher(store)
            batcher.attach_engine(eng, gate_tokens=1024, max_wait_s=0.05)
            agent = BaseAgent(role=f"worker{rank}", goal="extract findings", memory_lookup=batcher)
            task = Task(description=f"audit ledger {rank} for the quarterly revenue of unit {rank * 7 + 3}")
            # every rank's agent writes its finding through the production path (BaseAgent._remember
            # -> MemoryLookupBatcher.store -> store_semantic_batch(vecs=...) with the gate's shared
            # embedding) while lookups are pending beside it
            pend = [asyncio.ensure_future(batcher.search(f"warm up query {rank} {i}", limit=2)) for i in range(3)]
            await agent._remember(task, True, {"reasoning": f"unit {rank * 7 + 3} grew"})
            await asyncio.gather(*pend)
            await asyncio.get_running_loop().run_in_executor(None, dist.barrier)
            # now each rank looks up the NEXT rank's finding
            peer = (rank + 1) % world
            hits = await batcher.search(f"audit ledger {peer} for the quarterly revenue of unit {peer * 7 + 3}",
                                        limit=3)
            out["hits"] = [(h.text, h.metadata) for h in hits]
            out["stats"] = dict(batcher.stats)
            out["agent_errors"] = dict(agent.memory_errors)
            batcher.detach_engine()
            out["listeners_after_detach"] = len(eng.listeners)

        asyncio.run(run())
        dist.barrier()
        store.stop()
        q.put((rank, out))
    finally:
        eng.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_agent_writes_through_batcher_reach_other_ranks(world):
    """an agent's `_remember` on rank A, through MemoryLookupBatcher (engine
    gate attached) into NodeSemanticStore, is returned by a lookup on rank B; failed writes are
    counted apart from stores."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_batcher_entry, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        peer = (r + 1) % world
        st = got[r]["stats"]
        assert st["stores"] == 1 and st["store_failures"] == 0 and st["lookup_failures"] == 0, st
        assert got[r]["agent_errors"] == {"store": 0, "search": 0}
        assert got[r]["listeners_after_detach"] == 0
        texts = [t for t, _ in got[r]["hits"]]
        assert any(t.startswith(f"audit ledger {peer} ") for t in texts), (r, texts)
        md = [m for t, m in got[r]["hits"] if t.startswith(f"audit ledger {peer} ")][0]
        assert md["success"] is True and md["agent"] != ""

"""Semantic memory inside the agent loop (memory/batcher.py + core/agent.py) and the
row-sharded index (memory/semantic_index.py ShardedSemanticIndex) on gloo ranks.

Reference behaviour being reproduced: agents consult memory while they work
(pilott/memory/enhanced_memory.py:93-116, docs/examples/pdf_processing/
example_agents.py:328-331); here the lookups of concurrent agents are coalesced into
one index pass per event-loop tick.
"""
import asyncio
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest
import torch

from pilottai_amd.core.agent import BaseAgent
from pilottai_amd.core.config import AgentConfig
from pilottai_amd.core.policy import ControlPolicy
from pilottai_amd.core.task import Task
from pilottai_amd.engine.local_llm import SchemaLLM
from pilottai_amd.memory.batcher import MemoryLookupBatcher
from pilottai_amd.memory.embedding import HashingEmbedder
from pilottai_amd.memory.enhanced_memory import EnhancedMemory
from pilottai_amd.memory.semantic_index import SemanticIndex, ShardedSemanticIndex
from pilottai_amd.tools.tool import Tool, echo_tool


class _RecordingLLM(SchemaLLM):
    def __init__(self):
        super().__init__(seed=0)
        self.prompts = []

    async def generate_response(self, messages, tools=None, response_format=None):
        self.prompts.append(messages[-1]["content"])
        return await super().generate_response(messages, tools=tools, response_format=response_format)


def test_agents_consult_memory_every_step_in_batched_passes():
    async def go():
        mem = EnhancedMemory(max_size=4096, device="cpu")
        await mem.store_semantic_batch([f"prior finding {i}: quarterly revenue of unit {i} grew" for i in range(40)],
                                       tags=[{"worker"}] * 40, priorities=[1] * 40)
        lookup = MemoryLookupBatcher(mem)
        llm = _RecordingLLM()
        pol = ControlPolicy("fixed", 2)
        agents = [BaseAgent(AgentConfig(role="worker", goal="Summarize documents", max_iterations=2), llm=llm,
                            tools=[Tool(name="echo", description="identity", function=echo_tool, max_retries=1)],
                            policy=pol, memory_lookup=lookup, memory_top_k=2) for _ in range(8)]
        for a in agents:
            await a.start()
        tasks = [Task(description=f"Summarize the revenue report of unit {i}") for i in range(8)]
        res = await asyncio.gather(*(a.execute_task(t) for a, t in zip(agents, tasks)))
        return res, lookup, mem, llm

    res, lookup, mem, llm = asyncio.run(go())
    assert all(r.success for r in res)
    # 8 agents x 2 step-planning calls each; concurrent lookups share index passes
    assert lookup.stats["lookups"] == 16
    assert lookup.stats["passes"] < lookup.stats["lookups"]
    assert lookup.stats["max_batch_seen"] >= 2
    mem_prompts = [p for p in llm.prompts if "Relevant memory:" in p]
    assert len(mem_prompts) == 16
    assert any("quarterly revenue" in p for p in mem_prompts)
    # every finished task was written back (batched stores)
    assert lookup.stats["stores"] == 8 and len(mem) == 48
    assert lookup.stats["store_batches"] < 8


def test_memory_off_keeps_default_prompt():
    async def go():
        llm = _RecordingLLM()
        a = BaseAgent(AgentConfig(role="worker", goal="g", max_iterations=1), llm=llm,
                      tools=[Tool(name="echo", description="identity", function=echo_tool)],
                      policy=ControlPolicy("fixed", 1))
        await a.start()
        r = await a.execute_task(Task(description="Summarize the document"))
        return r, llm

    r, llm = asyncio.run(go())
    assert r.success and not any("Relevant memory" in p for p in llm.prompts)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rows(n, dim, seed=0):
    g = np.random.default_rng(seed)
    return g.standard_normal((n, dim)).astype(np.float32)


def _shard_entry(rank, world, port, n, dim, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        vecs = _rows(n, dim)
        prio = [int(i % 5) for i in range(n)]
        tags = [{"even"} if i % 2 == 0 else {"odd"} for i in range(n)]
        local = SemanticIndex(dim=dim, capacity=64, device="cpu")
        sh = ShardedSemanticIndex(local)
        mine = list(range(rank, n, world))  # global row g = local_row * world + rank
        ids = sh.add_local(vecs[mine], [prio[i] for i in mine], [tags[i] for i in mine], [None] * len(mine))
        assert ids == mine
        queries = _rows(6, dim, seed=1)
        res = sh.search(queries, 5, [0, 0, 2, 0, 3, 0], [(), ("even",), (), ("odd",), ("even",), ()], now=None)
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_index_topk_equals_single_index(world):
    n, dim = 203, 64
    vecs = _rows(n, dim)
    single = SemanticIndex(dim=dim, capacity=256, device="cpu")
    single.add(vecs, [int(i % 5) for i in range(n)], [{"even"} if i % 2 == 0 else {"odd"} for i in range(n)],
               [None] * n)
    queries = _rows(6, dim, seed=1)
    ref = single.search(queries, 5, [0, 0, 2, 0, 3, 0], [(), ("even",), (), ("odd",), ("even",), ()])

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_entry, args=(r, world, port, n, dim, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for r in range(world):  # every rank gets the same merged answer ...
        assert [[row for row, _ in lst] for lst in got[r]] == [[row for row, _ in lst] for lst in got[0]]
    for lst_s, lst_r in zip(got[0], ref):  # ... equal to one index holding all rows
        assert [row for row, _ in lst_s] == [row for row, _ in lst_r]
        np.testing.assert_allclose([s for _, s in lst_s], [s for _, s in lst_r], rtol=1e-5, atol=1e-5)


def test_serve_does_not_start_openings_for_custom_agents():
    """Serve's speculative opening (task analysis + tool selection) is only started for
    agents that run the standard protocol; a subclass with its own execution path must
    not have its LLM resolved (that once built a default engine per plumbing run)."""
    import sys

    sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parent.parent))
    from benchmarks.plumbing import InstantLLM, make_echo_agent_cls
    from pilottai_amd.serve import Serve

    Echo = make_echo_agent_cls()

    async def go():
        agents = [Echo(AgentConfig(role=f"echo-{i}", goal="echo")) for i in range(2)]
        serve = Serve(agents=agents, manager_llm=InstantLLM(), config={"max_concurrent_tasks": 2})
        await serve.start()
        rs = await asyncio.gather(*(serve.execute_task(Task(description=f"echo {i}")) for i in range(6)))
        await serve.stop()
        return agents, rs

    agents, rs = asyncio.run(go())
    assert all(r.success for r in rs)
    assert all(a._llm is None for a in agents)


def test_batcher_scans_beside_compute_bound_steps():
    """with an engine gate attached, an index pass waits for the engine to
    launch a compute-bound step (>= gate_tokens tokens) and starts right behind it; a lookup
    never waits longer than the latency cap when no such step comes."""
    import time as _t

    class FakeEngine:
        def __init__(self):
            self.listeners = []

        def add_step_listener(self, fn):
            self.listeners.append(fn)

        def launch(self, T):
            for fn in self.listeners:
                fn(T)

    async def run():
        mem = EnhancedMemory(device="cpu", dim=64, embedder=HashingEmbedder(64))
        await mem.store_semantic_batch(["alpha report", "beta memo", "gamma notes"])
        b = MemoryLookupBatcher(mem)
        eng = FakeEngine()
        b.attach_engine(eng, gate_tokens=1024, max_wait_s=0.2)
        loop = asyncio.get_running_loop()
        # a heavy launch 50 ms after the lookup: the pass starts beside it
        t0 = _t.perf_counter()
        loop.call_later(0.02, eng.launch, 64)     # memory-bound: not a trigger
        loop.call_later(0.05, eng.launch, 2048)   # compute-bound: the trigger
        hits = await b.search("alpha report", limit=1)
        waited = _t.perf_counter() - t0
        assert hits and hits[0].text == "alpha report"
        assert 0.045 <= waited < 0.18 and b.stats["passes_beside_heavy"] == 1
        # no heavy step: the cap releases the lookup (past the 2 ms "just launched" window)
        await asyncio.sleep(0.01)
        t0 = _t.perf_counter()
        await b.search("beta memo", limit=1)
        assert 0.18 <= _t.perf_counter() - t0 < 0.5 and b.stats["passes_capped"] == 1
        s = b.latency_summary()
        assert s["lookups"] == 2 and s["lookup_p99_ms"] >= s["lookup_p50_ms"] > 0

    asyncio.run(run())



def test_first_step_lookup_overlaps_the_opening_calls():
    """The first step plan's memory query depends only on the task, so its lookup starts with
    the opening (analysis / tool selection) calls and finishes under them: with 50 ms LLM
    calls and a 60 ms lookup the task takes about one lookup less than in sequence, the
    step-0 prompt still carries the hits, and a dropped opening cancels the lookup too."""
    import time as _t

    class SlowLookup(MemoryLookupBatcher):
        def __init__(self, mem):
            super().__init__(mem)
            self.starts = []

        async def search(self, query, limit=5, tags=None, min_priority=0):
            self.starts.append(_t.perf_counter())
            await asyncio.sleep(0.06)
            return await super().search(query, limit=limit, tags=tags, min_priority=min_priority)

    async def go():
        mem = EnhancedMemory(max_size=1024, device="cpu")
        await mem.store_semantic_batch(["prior finding: quarterly revenue grew"], tags=[{"worker"}], priorities=[1])
        lookup = SlowLookup(mem)
        llm = _RecordingLLM()
        llm.latency_s = 0.05
        a = BaseAgent(AgentConfig(role="worker", goal="Summarize documents", max_iterations=2), llm=llm,
                      tools=[Tool(name="echo", description="identity", function=echo_tool, max_retries=1)],
                      policy=ControlPolicy("fixed", 2), memory_lookup=lookup, memory_top_k=1)
        await a.start()
        t0 = _t.perf_counter()
        r = await a.execute_task(Task(description="Summarize the quarterly revenue report"))
        first_start = lookup.starts[0] - t0
        # a speculative opening that is dropped takes its lookup with it
        t2 = Task(description="Another report")
        a.prefetch_opening(t2)
        lk = a._first_lookups[t2.id]
        a.drop_opening(t2.id)
        await asyncio.sleep(0)
        return r, first_start, llm, lk, len(lookup.starts)

    r, first_start, llm, lk, nstarts = asyncio.run(go())
    assert r.success
    assert first_start < 0.02  # issued with the opening calls, not after them (>= 50 ms)
    mem_prompts = [p for p in llm.prompts if "Relevant memory:" in p]
    assert len(mem_prompts) == 2 and "quarterly revenue" in mem_prompts[0]
    assert lk.cancelled() or lk.done()


def test_writes_and_queries_share_one_embedding_call():
    """With an engine gate attached, the writes pending at a flush and the queries pending
    beside them are embedded in ONE embedder call (one engine round trip, not two), the
    writes are in the index before those queries scan it, and the answers match a plain
    lookup."""
    class FakeEngine:
        def add_step_listener(self, fn):
            pass

    class Counting(HashingEmbedder):
        def __init__(self, dim):
            super().__init__(dim)
            self.calls = []

        def __call__(self, texts):
            self.calls.append(list(texts))
            return super().__call__(texts)

    async def run():
        emb = Counting(64)
        mem = EnhancedMemory(device="cpu", dim=64, embedder=emb)
        await mem.store_semantic_batch(["alpha report", "beta memo"])
        b = MemoryLookupBatcher(mem)
        b.attach_engine(FakeEngine(), gate_tokens=1024, max_wait_s=0.0)
        emb.calls.clear()
        st = asyncio.ensure_future(b.store("gamma notes"))
        hits = await asyncio.gather(b.search("gamma notes", limit=1), b.search("beta memo", limit=1))
        await st
        return emb.calls, hits, b.stats

    calls, hits, stats = asyncio.run(run())
    assert calls == [["gamma notes", "gamma notes", "beta memo"]]
    assert [h[0].text for h in hits] == ["gamma notes", "beta memo"]
    assert stats["shared_embeds"] == 1 and stats["passes"] == 1 and stats["stores"] == 1
    # the lookup latency anatomy bench.py reports (memory.lookup_anatomy_ms)
    assert stats["embed_s"] > 0 and stats["search_s"] > 0 and stats["queued_s"] >= 0

"""Control-plane services (LB, scaling, FT, delegation), tools, knowledge, memory, checkpoints (CPU)."""
import asyncio
from datetime import datetime, timedelta
from unittest.mock import AsyncMock, patch

import pytest

from pilottai_amd import Serve
from pilottai_amd.core.agent import BaseAgent
from pilottai_amd.core.config import AgentConfig
from pilottai_amd.core.policy import ControlPolicy
from pilottai_amd.core.role import AgentStatus
from pilottai_amd.core.task import Task
from pilottai_amd.delegation.task_delegator import TaskDelegator
from pilottai_amd.engine.local_llm import SchemaLLM
from pilottai_amd.knowledge.knowledge_manager import KnowledgeManager
from pilottai_amd.memory.enhanced_memory import EnhancedMemory
from pilottai_amd.orchestration import DynamicScaling, FaultTolerance, HealthStatus, LoadBalancer
from pilottai_amd.tools.knowledge import KnowledgeSource
from pilottai_amd.tools.tool import Tool, ToolError, ToolTimeoutError

FIXED = ControlPolicy("fixed", 1)


def agent(role="w", **cfg):
    return BaseAgent(AgentConfig(role=role, goal="g", description="d", **cfg), llm=SchemaLLM(), policy=FIXED)


@pytest.fixture
def mock_orchestrator():
    m = AsyncMock()
    m.child_agents = {}
    m.config = AsyncMock()
    m.config.max_agents = 10
    m.config.min_agents = 2
    return m


# ---------------------------------------------------------------- reference tests/test_orchestration.py
async def test_load_balancer_smoke(mock_orchestrator):
    lb = LoadBalancer(mock_orchestrator, {"check_interval": 0.01})
    await lb.start()
    await lb._balance_system_load()
    await lb.stop()
    assert not lb.running


async def test_dynamic_scaling_scales_up(mock_orchestrator):
    sc = DynamicScaling(mock_orchestrator, {"check_interval": 100})
    await sc.start()
    mock_orchestrator.create_agent = AsyncMock(return_value=AsyncMock())
    with patch.object(sc, "_can_scale", return_value=True), patch.object(sc, "_get_system_load", return_value=0.9):
        await sc._check_and_adjust_scale()
        assert mock_orchestrator.create_agent.called
    await sc.stop()


async def test_fault_tolerance_recovers(mock_orchestrator):
    ft = FaultTolerance(mock_orchestrator, {"health_check_interval": 100})
    await ft.start()
    mock_agent = mock_orchestrator
    mock_agent.id = "test_agent"
    with patch.object(ft, "_check_agent_health", return_value=False):
        await ft._handle_unhealthy_agent(mock_agent)
        assert mock_agent.reset.called
    await ft.stop()


# ---------------------------------------------------------------- deeper behaviour
async def test_load_balancer_moves_tasks_between_agents():
    a, b = agent("busy", max_queue_size=10), agent("free", max_queue_size=10)
    for x in (a, b):
        await x.start()
    for i in range(8):
        await a.add_task(Task(description=f"t{i}", priority="high" if i == 7 else "low"))

    class O:
        child_agents = {a.id: a, b.id: b}

    lb = LoadBalancer(O(), {"overload_threshold": 0.5, "underload_threshold": 0.45, "balance_batch_size": 2})
    lb._calculate_load_trend = lambda aid: 1.0 if aid == a.id else -1.0
    lb._calculate_composite_load = lambda m: 0.9 if m.queue_size >= 8 else 0.1
    await lb._balance_system_load()
    assert len(a.tasks) == 6 and len(b.tasks) == 2
    assert any(t.description == "t7" for t in b.tasks.values())  # highest priority moved first
    assert lb.get_metrics()["tasks_moved"] == 2


async def test_scaling_down_respects_min_and_cooldown():
    agents = {x.id: x for x in (agent("a"), agent("b"), agent("c"))}
    for x in agents.values():
        await x.start()

    class O:
        child_agents = agents

        async def remove_child_agent(self, aid):
            agents.pop(aid)

    sc = DynamicScaling(O(), {"min_agents": 2, "cooldown_period": 1000})
    sc._get_system_load = AsyncMock(return_value=0.05)
    await sc._check_and_adjust_scale()
    assert len(agents) == 2 and sc.scale_downs == 1
    await sc._check_and_adjust_scale()  # cooldown blocks a second action
    assert len(agents) == 2


async def test_fault_tolerance_detects_and_replaces():
    s = Serve(agents=[agent("w")], manager_llm=SchemaLLM(), config={"policy": "fixed"})
    await s.start()
    ft = FaultTolerance(s, {"max_recovery_attempts": 0})
    w = next(iter(s.agents.values()))
    assert await ft._check_agent_health(w) == HealthStatus.HEALTHY
    await w.stop()  # heartbeat now fails -> CRITICAL -> replace
    st = await ft._check_agent_health(w)
    assert st == HealthStatus.CRITICAL
    await ft._handle_unhealthy_agent(w, st)
    assert w.id not in s.agents and len(s.agents) == 1 and ft.replacements == 1
    r = await s.execute_task(Task(description="after replacement"), timeout=20)
    assert r.success
    await s.stop()


async def test_fault_tolerance_gpu_probe_flags_failed_engine():
    class Eng:
        failed = RuntimeError("hip error")
        stats = {"steps": 0}

    class L:
        engine = Eng()

    a = agent("x")
    a._llm = L()
    await a.start()
    ft = FaultTolerance(AsyncMock())
    assert await ft._check_agent_health(a) == HealthStatus.CRITICAL
    assert "gpu" in ft.agent_health[a.id].details


async def test_task_delegator_decision_and_scoring(monkeypatch):
    import psutil

    monkeypatch.setattr(psutil, "cpu_percent", lambda interval=None: 10.0)  # host load must not flake the filter
    mgr = BaseAgent(AgentConfig(role="mgr", goal="g", allow_delegation=True, max_task_complexity=3),
                    llm=SchemaLLM(), policy=FIXED)
    await mgr.start()
    c1, c2 = agent("c1", specializations=["extract"]), agent("c2")
    await mgr.add_child_agent(c1)
    await mgr.add_child_agent(c2)
    d = TaskDelegator(mgr)
    ok, aid = await d.evaluate_delegation({"id": "t1", "complexity": 2})
    assert not ok
    ok, aid = await d.evaluate_delegation({"id": "t2", "complexity": 9, "type": "extract"})
    assert ok and aid == c1.id
    await d.record_delegation(aid, {"id": "t2"}, {"status": "completed", "execution_time": 1.5})
    m = d.get_agent_metrics(aid)
    assert m["success_rate"] == 1.0 and m["total_tasks"] == 1 and "t2" not in d.active_delegations
    r = await d.delegate(Task(description="hard", complexity=9))
    assert r is not None and r.success
    assert (await d.get_metrics())["history_size"] == 2


# ---------------------------------------------------------------- tools
async def test_tool_retry_timeout_metrics():
    calls = {"n": 0}

    def flaky(x=0):
        calls["n"] += 1
        if calls["n"] < 2:
            raise RuntimeError("transient")
        return x * 2

    t = Tool(name="flaky", function=flaky, retry_delay=0.0, max_retries=3)
    assert await t.execute(x=21) == 42
    assert t.metrics.success_count == 1 and t.success_rate == 1.0

    async def slow():
        await asyncio.sleep(1)

    s = Tool(name="slow", function=slow, timeout=0.05, max_retries=1, retry_delay=0)
    with pytest.raises(ToolTimeoutError):
        await s.execute()
    assert s.metrics.error_count == 1
    s.disable("maintenance")
    with pytest.raises(ToolError):
        await s.execute()
    s.enable()
    assert s.get_metrics()["enabled"]


# ---------------------------------------------------------------- knowledge
async def test_knowledge_manager_cache_and_sources(tmp_path):
    (tmp_path / "a.txt").write_text("The MI355X has 288 GB of HBM3E.")
    km = KnowledgeManager(cache_size=10, cache_ttl=60)
    assert await km.add_source(KnowledgeSource(name="docs", type="file", connection={"path": str(tmp_path)}))
    assert await km.add_source(KnowledgeSource(name="mem", type="memory",
                                               connection={"documents": ["alpha beta", "gamma HBM3E"]}))
    calls = {"n": 0}

    async def fn(q):
        calls["n"] += 1
        return {"answer": q.upper()}

    assert await km.add_source(KnowledgeSource(name="fn", type="callable", connection={"fn": fn}))
    r = await km.query_knowledge("hbm3e", ["docs", "mem", "fn"])
    assert len(r) == 3 and r[2] == {"answer": "HBM3E"}
    r2 = await km.query_knowledge("hbm3e", ["fn", "mem", "docs"])  # same sources -> cache hit
    assert r2 == r and calls["n"] == 1 and km.get_cache_stats()["hits"] == 1
    await km.invalidate_cache(source_name="fn")
    await km.query_knowledge("hbm3e", ["fn"])
    assert calls["n"] == 2
    assert km.get_source_stats()["mem"]["access_count"] >= 1
    assert not await km.add_source(KnowledgeSource(name="bad", type="file", connection={"path": "/nonexistent"}))


# ---------------------------------------------------------------- enhanced memory
async def test_enhanced_memory_semantic_and_substring():
    m = EnhancedMemory(max_size=100, device="cpu")
    assert await m.semantic_search("anything") == []  # empty store (App. A #26)
    await m.store_semantic("GPU kernels for attention on MI355X", {"k": 1}, tags={"gpu"}, priority=2)
    await m.store_semantic("quarterly revenue report for the sales team", tags={"biz"}, priority=1)
    await m.store_semantic("attention kernel tuning notes", tags={"gpu", "notes"}, priority=0, ttl=-1)
    hits = await m.semantic_search("attention kernels", limit=2)
    assert hits and hits[0].metadata == {"k": 1}  # expired item filtered out
    assert await m.semantic_search("revenue", tags={"gpu"}) == [] or \
        all("gpu" in h.tags for h in await m.semantic_search("revenue", tags={"gpu"}))
    assert [h.text for h in await m.semantic_search("REVENUE", mode="substring")] == \
        ["quarterly revenue report for the sales team"]
    assert await m.semantic_search("kernels", min_priority=3) == []
    res = await m.search_batch(["gpu attention", "sales revenue"], limit=1)
    assert res[0][0].tags == {"gpu"} and res[1][0].tags == {"biz"}
    await m.store_task("t1", {"type": "x", "v": 1})
    await m.store_task("t1", {"type": "x", "v": 2})
    recent = await m.get_recent_tasks(limit=5, task_type="x")
    assert [r["version"] for r in recent] == [2, 1]
    await m.store_pattern("p", 42, ttl=100)
    assert await m.get_pattern("p") == 42
    await m.store_interaction("agent", "msg", {"a": 1})
    await m.store_interaction("agent", "msg", {"a": 2})
    assert len(await m.get_interactions("agent")) == 2
    await m.cleanup()
    assert len(m) == 2


async def test_enhanced_memory_ring_eviction():
    m = EnhancedMemory(max_size=4, device="cpu")
    for i in range(6):
        await m.store_semantic(f"document number {i} about topic{i}")
    assert len(m) == 4
    hits = await m.semantic_search("document number 0 about topic0", limit=4)
    assert all("topic0" not in h.text for h in hits)  # evicted rows are gone, not stale


async def test_agent_enhanced_memory_documented_api():
    a = agent("x")
    await a.enhanced_memory.store_semantic("hello world", {"source": "test"})
    assert (await a.enhanced_memory.semantic_search("hello", limit=5))[0].text == "hello world"


# ---------------------------------------------------------------- checkpoint / resume
async def test_checkpoint_and_resume(tmp_path):
    s = Serve(agents=[agent("w")], manager_llm=SchemaLLM(), config={"policy": "fixed"})
    await s.start()
    r = await s.execute_task(Task(description="done before checkpoint"), timeout=20)
    assert r.success
    pending = Task(description="pending at checkpoint")
    s.tasks[pending.id] = pending
    w = next(iter(s.agents.values()))
    await w.enhanced_memory.store_semantic("remember this", tags={"t"})
    path = s.checkpoint(tmp_path / "ckpt")
    await s.stop()

    s2 = Serve(agents=[agent("w")], manager_llm=SchemaLLM(), config={"policy": "fixed"})
    n = await s2.restore(path)
    assert n == 1 and len(s2.completed_tasks) == 1 and len(s2.memory) == 1
    assert (await s2.wait_for(pending.id, timeout=20)).success
    await s2.stop()


async def test_checkpoint_save_after_interrupted_swap_keeps_a_good_copy(tmp_path, monkeypatch):
    """when an earlier save died between its renames (<path> missing, <path>.bak
    holding the last checkpoint), the next save must not delete .bak before the new
    checkpoint is in place: a crash in that window still leaves a loadable checkpoint."""
    import os
    import shutil

    from pilottai_amd.utils import checkpoint as ck

    s = Serve(agents=[agent("w")], manager_llm=SchemaLLM(), config={"policy": "fixed"})
    path = tmp_path / "ckpt"
    s.checkpoint(path)
    os.replace(path, path.with_name("ckpt.bak"))  # the interrupted state
    real_replace = os.replace

    def crash_on_publish(src, dst):
        if str(dst) == str(path):
            raise OSError("simulated crash before the new checkpoint is published")
        return real_replace(src, dst)
    monkeypatch.setattr(ck.os, "replace", crash_on_publish)
    with pytest.raises(OSError):
        s.checkpoint(path)
    monkeypatch.setattr(ck.os, "replace", real_replace)
    assert ck.load_checkpoint(path)["format_version"] == ck.FORMAT_VERSION  # from .bak
    shutil.rmtree(path.with_name("ckpt.bak"))

"""Agent runtime, factory, router and Serve orchestrator on CPU with the model-free SchemaLLM."""
import asyncio
import json
from unittest.mock import AsyncMock

import pytest

from pilottai_amd import Serve
from pilottai_amd.core.agent import BaseAgent
from pilottai_amd.core.config import AgentConfig, LLMConfig
from pilottai_amd.core.factory import AgentFactory
from pilottai_amd.core.policy import ControlPolicy
from pilottai_amd.core.role import AgentRole, AgentStatus
from pilottai_amd.core.router import TaskRouter
from pilottai_amd.core.task import Task, TaskPriority, TaskStatus
from pilottai_amd.engine.local_llm import SchemaLLM
from pilottai_amd.tools.tool import Tool, echo_tool

FIXED = ControlPolicy("fixed", steps_per_task=2)


def make_agent(role="worker", llm=None, tools=None, policy=FIXED, **cfg):
    c = AgentConfig(role=role, goal="get things done", description="test agent", **cfg)
    return BaseAgent(c, llm=llm or SchemaLLM(seed=1), tools=tools if tools is not None else
                     [Tool(name="echo", function=echo_tool, max_retries=1)], policy=policy)


# ---------------------------------------------------------------- agent
async def test_agent_executes_fixed_policy_task():
    steps = []
    a = make_agent()
    a.step_callback = lambda step, result, context: steps.append(step["tool"])
    await a.start()
    r = await a.execute_task(Task(description="summarize x", metadata={"tool_inputs": {"q": 1}}))
    assert r.success, r.error
    assert r.metadata["iterations"] == 2
    assert [s["result"]["output"] for s in r.output] == [{"echo": {"q": 1}}] * 2
    assert steps == ["echo", "echo"]
    assert a.task_metrics["completed"] == 1 and a.status == AgentStatus.IDLE
    assert a.llm.usage["calls"] == 2 + 3 + 1  # analysis, tools, 3 step plans, evaluation


async def test_agent_documented_constructor_and_dict_task():
    a = BaseAgent(AgentConfig(role="extractor", goal="extract", description="d"),
                  LLMConfig(provider="schema"), policy=FIXED)
    assert isinstance(a.llm, SchemaLLM)
    await a.start()
    r = await a.execute_task({"type": "extract", "description": "extract text"})
    assert r.success
    assert a.metrics["completed"] == 1  # documented `agent.metrics` alias


async def test_agent_reference_constructor_requires_role():
    a = BaseAgent(role="r", goal="g", llm=SchemaLLM(), max_iter=3, allow_delegation=True)
    assert a.config.max_iter == 3 and a.config.allow_delegation
    with pytest.raises(ValueError):
        BaseAgent(goal="g")


async def test_agent_timeout_and_failure_paths():
    class Slow(SchemaLLM):
        async def _complete(self, *a, **k):
            await asyncio.sleep(5)

    a = make_agent(llm=Slow())
    await a.start()
    r = await a.execute_task(Task(description="x", timeout=0.2))
    assert not r.success and "timed out" in r.error
    assert a.task_metrics["timeout"] == 1

    class Bad(SchemaLLM):
        async def _complete(self, *a, **k):
            return {"content": "not json", "usage": {"prompt_tokens": 1, "completion_tokens": 1}}

    b = make_agent(llm=Bad(retry_attempts=1) if False else Bad())
    await b.start()
    r = await b.execute_task(Task(description="x"))
    assert not r.success and "Invalid JSON" in r.error


async def test_agent_suitability_formula():
    a = make_agent(required_capabilities=["pdf"], specializations=["extract"])
    assert await a.evaluate_task_suitability({"type": "extract"}) == pytest.approx(0.9)
    assert await a.evaluate_task_suitability({"type": "other"}) == pytest.approx(0.7)
    assert await a.evaluate_task_suitability({"required_capabilities": ["gpu"]}) == 0.0
    for i in range(50):
        await a.add_task(Task(description=f"t{i}"))
    assert await a.evaluate_task_suitability({"type": "other"}) == pytest.approx(0.7 - 0.3 * 0.5)


async def test_agent_heartbeat_children_and_tool_locks():
    a = make_agent()
    await a.start()
    assert await a.send_heartbeat()
    c = make_agent("child")
    await a.add_child_agent(c)
    assert a.child_agents[c.id] is c and c.status == AgentStatus.IDLE
    assert await a.select_agent(Task(description="x")) is c
    await a.remove_child_agent(c.id)
    assert not a.child_agents
    await a.stop()
    with pytest.raises(RuntimeError):
        await a.send_heartbeat()


# ---------------------------------------------------------------- factory (reference tests/test_factory.py)
class MockAgent(BaseAgent):
    def __init__(self, config=None):
        self.config = config or AgentConfig(role="test_role", goal="g", description="d")
        self.id = f"mock-{id(self)}"
        self.status = "idle"
        self.start = AsyncMock()
        self.stop = AsyncMock()
        self.cleanup_resources = AsyncMock()


async def test_factory_registry_and_lifecycle():
    AgentFactory._agent_types.clear()
    AgentFactory.register_agent_type("test_agent", MockAgent)
    with pytest.raises(ValueError):
        AgentFactory.register_agent_type("", MockAgent)
    with pytest.raises(TypeError):
        AgentFactory.register_agent_type("invalid", object)
    with pytest.raises(ValueError):
        AgentFactory.register_agent_type("test_agent", MockAgent)
    agent = await AgentFactory.create_agent("test_agent")
    assert isinstance(agent, MockAgent) and agent.id in AgentFactory._active_agents
    with pytest.raises(ValueError):
        await AgentFactory.create_agent("")
    with pytest.raises(ValueError):
        await AgentFactory.create_agent("unknown")
    await AgentFactory.cleanup_agent(agent.id)
    assert agent.id not in AgentFactory._active_agents
    await AgentFactory.cleanup_agent("non_existent")
    async with AgentFactory.create_managed_agent("test_agent") as m:
        assert m.id in AgentFactory._active_agents
    assert m.id not in AgentFactory._active_agents
    assert "test_agent" in AgentFactory.list_available_types()


async def test_factory_creation_timeout():
    class Slow(MockAgent):
        def __init__(self, config=None):
            super().__init__(config)

            async def slow():
                await asyncio.sleep(2)

            self.start = slow

    AgentFactory._agent_types.clear()
    AgentFactory.register_agent_type("slow", Slow)
    old = AgentFactory.creation_timeout
    AgentFactory.creation_timeout = 0.05
    try:
        with pytest.raises(asyncio.TimeoutError):
            await AgentFactory.create_agent("slow")
    finally:
        AgentFactory.creation_timeout = old


async def test_factory_creates_plain_base_agent():
    AgentFactory._agent_types.clear()
    AgentFactory.register_agent_type("base", BaseAgent)
    a = await AgentFactory.create_agent("base", llm=SchemaLLM())  # App. A #36
    assert isinstance(a, BaseAgent) and a.status == AgentStatus.IDLE
    await AgentFactory.cleanup_all_agents()


# ---------------------------------------------------------------- router
async def test_router_scores_and_priority():
    class Orch:
        pass

    o = Orch()
    a1, a2 = make_agent("a1", specializations=["pdf"]), make_agent("a2")
    await a1.start()
    await a2.start()
    o.agents = [a1, a2]  # a list works (App. A #29)
    r = TaskRouter(o, {"retry_delay": 0})
    assert await r.route_task({"type": "pdf"}) == a1.id
    o.agents = {a1.id: a1, a2.id: a2}
    a1.status = AgentStatus.BUSY
    r2 = TaskRouter(o, {"retry_delay": 0})
    assert await r2.route_task({"type": "pdf"}) == a2.id
    assert TaskRouter.get_task_priority({"urgent": True}) == TaskPriority.CRITICAL
    assert TaskRouter.get_task_priority({"complexity": 9}) == TaskPriority.HIGH
    assert TaskRouter.get_task_priority({"dependencies": [1, 2, 3, 4]}) == TaskPriority.MEDIUM
    assert TaskRouter.get_task_priority({}) == TaskPriority.LOW


# ---------------------------------------------------------------- Serve
async def test_serve_documented_api_add_agent_execute_task():
    AgentFactory._agent_types.clear()
    s = Serve(name="test_pilott", llm=SchemaLLM(seed=3), config={"policy": "fixed"})
    await s.start()
    agent = await s.add_agent("test_agent", AgentConfig(role="test_agent", goal="g", description="d"),
                              LLMConfig(provider="schema"))
    assert len(s.agents) == 1 and agent.status == AgentStatus.IDLE
    r = await s.execute_task({"type": "summarize", "description": "summarize the doc"})
    assert r.success, r.error
    assert s.get_metrics()["metrics"]["successful_tasks"] == 1
    await s.stop()


async def test_serve_concurrency_priority_and_memory():
    llm = SchemaLLM(seed=5)
    agents = [make_agent(f"w{i}", llm=llm) for i in range(4)]
    s = Serve(agents=agents, manager_llm=llm, config={"max_concurrent_tasks": 4, "policy": "fixed"})
    await s.start()
    tasks = [Task(description=f"task {i}", priority=["low", "high"][i % 2]) for i in range(12)]
    ids = [await s.add_task(t) for t in tasks]
    results = await asyncio.gather(*(s.wait_for(i, timeout=30) for i in ids))
    assert all(r.success for r in results)
    assert len(s.completed_tasks) == 12 and s.memory is not None and len(s.memory) == 12
    assert (await s.get_result(ids[0])).success
    assert s.latency.pct(50) > 0
    await s.stop()


async def test_serve_reference_constructor_and_validation():
    a = make_agent()
    with pytest.raises(ValueError):
        Serve(agents=[a], manager_llm=SchemaLLM(), manager_agent=make_agent("m"))
    s = Serve(agents=[a], manager_llm=SchemaLLM(), config={"max_concurrent_tasks": 2, "policy": "fixed"})
    tid = await s.add_task(Task(description="x"))
    r = await s.wait_for(tid, timeout=10)
    assert r.success
    await s.stop()


async def test_serve_decomposition_parent_completes():
    llm = SchemaLLM(seed=7)
    s = Serve(agents=[make_agent(f"w{i}", llm=llm) for i in range(2)], manager_llm=llm,
              config={"max_concurrent_tasks": 2, "policy": "fixed"})
    await s.start()
    r = await s.execute_task(Task(description="big job", metadata={"decompose": True}), timeout=30)
    assert r.success  # parent aggregates its subtasks (App. A #23)
    parent = [t for t in s.tasks.values() if t.subtasks][0]
    assert len(parent.subtasks) == 2 and s.metrics["decomposed_tasks"] == 1
    await s.stop()


async def test_serve_retry_on_failed_evaluation_and_dependencies():
    class Flaky(SchemaLLM):
        n = 0

        async def _complete(self, messages, rf, tools):
            r = await super()._complete(messages, rf, tools)
            if rf and rf.get("schema") == "agent.result_evaluation":
                Flaky.n += 1
                obj = json.loads(r["content"])
                obj["success"] = Flaky.n > 1  # first attempt fails, retry succeeds
                r["content"] = json.dumps(obj)
            return r

    llm = Flaky(seed=1)
    s = Serve(agents=[make_agent("w", llm=llm, policy=ControlPolicy("model", 1)),
                      make_agent("v", llm=llm, policy=ControlPolicy("model", 1))],
              manager_llm=SchemaLLM(), config={"max_concurrent_tasks": 2, "policy": "fixed"})
    await s.start()
    r = await s.execute_task(Task(description="flaky"), timeout=30)
    assert r.success and s.metrics["retried_tasks"] == 1
    a = Task(description="first")
    b = Task(description="second", dependencies=[a.id])
    bid = await s.add_task(b)
    await s.add_task(a)
    assert (await s.wait_for(bid, timeout=30)).success
    await s.stop()


async def test_serve_queue_overflow_evicts_lower_priority():
    s = Serve(agents=[], manager_llm=SchemaLLM(), config={"max_queue_size": 2, "max_concurrent_tasks": 1,
                                                          "analyze_tasks": False, "agent_wait_timeout": 0.2})
    await s.start()
    for w in s._workers:  # freeze consumers so the queue fills
        w.cancel()
    await asyncio.sleep(0)
    await s.add_task(Task(description="l1", priority="low"))
    await s.add_task(Task(description="l2", priority="low"))
    await s.add_task(Task(description="h", priority="high"))
    assert len(s.failed_tasks) == 1
    victim = next(iter(s.failed_tasks.values()))
    assert "overflow" in victim.error
    assert [t.description for _, _, t in sorted(s._queue._queue)][0] == "h"
    with pytest.raises(RuntimeError):
        await s.add_task(Task(description="l3", priority="low"))
    await s.stop()


async def test_serve_orchestrator_protocol():
    llm = SchemaLLM()
    s = Serve(agents=[make_agent("w", llm=llm)], manager_llm=llm, config={"policy": "fixed"})
    await s.start()
    n = await s.create_agent(role="w2")
    await s.add_child_agent(n)
    assert n.id in s.child_agents and s.verbose is False
    await s.remove_child_agent(n.id)
    assert n.id not in s.child_agents
    await s.stop()


def test_complex_workflow_steps_go_to_specialised_children():
    """README.md:143-146 of the reference: manager.execute_task({"type": "complex_workflow", "steps": [...]})."""
    import asyncio

    from pilottai_amd.core.agent import BaseAgent
    from pilottai_amd.core.config import AgentConfig, LLMConfig
    from pilottai_amd.core.policy import ControlPolicy
    from pilottai_amd.core.task import TaskResult
    from pilottai_amd.engine.local_llm import SchemaLLM

    seen = []

    class Worker(BaseAgent):
        async def _execute_task_internal(self, task):
            seen.append((self.config.role, task.metadata["type"], task.metadata["previous_output"]))
            return TaskResult(success=True, output=f"{self.config.role}-out")

    async def main():
        llm = SchemaLLM(LLMConfig(provider="schema"))
        mgr = BaseAgent(AgentConfig(role="manager", goal="g", max_child_agents=4), llm=llm, policy=ControlPolicy("fixed"))
        for s in ("extract", "analyze", "summarize"):
            await mgr.add_child_agent(Worker(AgentConfig(role=s, goal=s, specializations=[s]), llm=llm))
        return await mgr.execute_task({"type": "complex_workflow", "steps": ["extract", "analyze", "summarize"]})

    r = asyncio.run(main())
    assert r.success and r.output == {"extract": "extract-out", "analyze": "analyze-out", "summarize": "summarize-out"}
    assert seen == [("extract", "extract", None), ("analyze", "analyze", "extract-out"),
                    ("summarize", "summarize", "analyze-out")]


async def test_agent_analysis_and_tool_selection_overlap():
    """The two independent opening calls of an agent task are in flight together
    (one continuous-batch step for both), and a "cannot execute" analysis still
    fails the task (reference pilott/core/agent.py:176-182)."""
    class SlowLLM(SchemaLLM):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            self.inflight, self.peak = 0, 0

        async def generate_response(self, messages, tools=None, **kw):
            self.inflight += 1
            self.peak = max(self.peak, self.inflight)
            await asyncio.sleep(0.02)
            try:
                return await super().generate_response(messages, tools, **kw)
            finally:
                self.inflight -= 1

    llm = SlowLLM(seed=3)
    a = make_agent(llm=llm)
    await a.start()
    r = await a.execute_task(Task(description="summarize y"))
    assert r.success, r.error
    assert llm.peak == 2

    class NoLLM(SlowLLM):
        async def generate_response(self, messages, tools=None, **kw):
            out = await super().generate_response(messages, tools, **kw)
            text = json.dumps(messages)
            if "can_execute" in text:
                obj = json.loads(out["content"])
                obj["can_execute"] = False
                obj["reason"] = "no"
                out["content"] = json.dumps(obj)
            return out

    b = make_agent(llm=NoLLM(seed=4), policy=ControlPolicy("model"))
    await b.start()
    r = await b.execute_task(Task(description="summarize z"))
    assert not r.success and "Cannot execute" in (r.error or "")


class _CountingLLM(SchemaLLM):
    """SchemaLLM with a small per-call latency that records peak concurrency."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.inflight, self.peak, self.total = 0, 0, 0

    async def _complete(self, messages, response_format, tools):
        self.inflight += 1
        self.total += 1
        self.peak = max(self.peak, self.inflight)
        await asyncio.sleep(0.02)
        try:
            return await super()._complete(messages, response_format, tools)
        finally:
            self.inflight -= 1


async def test_serve_speculative_agent_start_overlaps_orchestrator_analysis():
    """The orchestrator's analysis and the agent's two opening calls (analysis, tool
    selection) run together; the task still makes exactly the same LLM calls."""
    llm = _CountingLLM(seed=8)
    s = Serve(agents=[make_agent("w", llm=llm)], manager_llm=llm, config={"policy": "fixed"})
    await s.start()
    r = await s.execute_task(Task(description="summarize q"))
    assert r.success, r.error
    assert llm.peak == 3
    # orchestrator analysis + evaluation; agent analysis, tools, 3 step plans (FIXED: 2 steps + done), evaluation
    assert llm.total == 2 + 2 + 3 + 1
    assert all(str(a.status) == "idle" for a in s.agents.values())
    assert not any(a._openings for a in s.agents.values())
    await s.stop()


async def test_serve_speculation_dropped_on_decomposition():
    """A speculatively started agent is released and its opening calls dropped when
    the orchestrator decomposes the task; the subtasks then run normally."""
    llm = _CountingLLM(seed=9)
    s = Serve(agents=[make_agent(f"w{i}", llm=llm) for i in range(2)], manager_llm=llm,
              config={"max_concurrent_tasks": 2, "policy": "fixed"})
    await s.start()
    r = await s.execute_task(Task(description="big job", metadata={"decompose": True}))
    assert r.success
    parent = [t for t in s.tasks.values() if t.subtasks][0]
    assert len(parent.subtasks) == 2 and s.metrics["decomposed_tasks"] == 1
    await asyncio.sleep(0.1)
    assert all(str(a.status) == "idle" for a in s.agents.values())
    assert not any(a._openings for a in s.agents.values())
    await s.stop()

"""Fault-injection hooks drive the failure-detection paths deterministically."""
import asyncio
import time

from pilottai_amd.core.agent import BaseAgent
from pilottai_amd.core.config import AgentConfig, LLMConfig
from pilottai_amd.engine.local_llm import SchemaLLM
from pilottai_amd.orchestration.fault_tolerance import FaultTolerance, GPUHealthProbe, HealthStatus
from pilottai_amd.utils.faults import FaultInjector


def test_dropped_heartbeat_is_critical_then_heals():
    async def main():
        mgr = BaseAgent(AgentConfig(role="mgr", goal="g", max_child_agents=4), llm=SchemaLLM(LLMConfig(provider="schema")))
        kid = BaseAgent(AgentConfig(role="kid", goal="g"), llm=SchemaLLM(LLMConfig(provider="schema")))
        await mgr.add_child_agent(kid)
        ft = FaultTolerance(mgr, {"resource_threshold": 1.0})
        inj = FaultInjector()
        inj.drop_heartbeat(kid, seconds=0.2)
        bad = await ft._check_agent_health(kid)
        await asyncio.sleep(0.25)
        good = await ft._check_agent_health(kid)
        inj.restore()
        return bad, good, inj.log

    bad, good, log = asyncio.run(main())
    assert bad == HealthStatus.CRITICAL and good == HealthStatus.HEALTHY
    assert log[0][1] == "drop_heartbeat"


def test_llm_failures_are_retried_by_agent_steps():
    async def main():
        llm = SchemaLLM(LLMConfig(provider="schema"))
        inj = FaultInjector()
        inj.fail_llm(llm, times=1)
        try:
            await llm.apredict("x", response_format={"schema": "agent.result_evaluation"})
            first = "ok"
        except RuntimeError as e:
            first = str(e)
        second = await llm.apredict("x", response_format={"schema": "agent.result_evaluation"})
        inj.restore()
        return first, second

    first, second = asyncio.run(main())
    assert "injected" in first and second


def test_engine_stall_detected_by_gpu_probe():
    from pilottai_amd.engine.engine import EngineConfig, LLMEngine

    eng = LLMEngine(EngineConfig(model="tiny", max_num_seqs=4, max_num_batched_tokens=64, max_model_len=256,
                                 num_kv_blocks=64, use_graphs=False), device="cpu")
    inj = FaultInjector()
    inj.stall_engine(eng, seconds=1.0)
    eng.start()
    eng.submit([1, 2, 3], lambda o: None, max_tokens=4)
    agent = BaseAgent(AgentConfig(role="a", goal="g"), llm=SchemaLLM(LLMConfig(provider="schema")))
    agent._llm.engine = eng
    probe = GPUHealthProbe(stall_timeout=0.3)
    assert probe.check(agent) is None
    time.sleep(0.5)
    msg = probe.check(agent)
    inj.restore()
    eng.stop()
    assert msg and "stalled" in msg

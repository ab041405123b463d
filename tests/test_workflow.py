"""Hierarchical document workflow (BASELINE config 5 on CPU): delegation to the
matching replica, context passed between stages, crash of a replica ->
FaultTolerance replacement, in-flight stage re-delegated, no failed workflow."""
import asyncio

from pilottai_amd.core.config import LLMConfig
from pilottai_amd.engine.local_llm import SchemaLLM
from pilottai_amd.orchestration.fault_tolerance import FaultTolerance
from pilottai_amd.serve import Serve
from pilottai_amd.workflows import STAGES, build_document_workflow


class SlowSchemaLLM(SchemaLLM):
    async def apredict(self, prompt, response_format=None):
        await asyncio.sleep(0.01)
        return await super().apredict(prompt, response_format=response_format)


def test_workflow_delegation_and_fault_tolerance():
    async def main():
        llm = SlowSchemaLLM(LLMConfig(model_name="x", provider="schema"))
        mgr, kids = await build_document_workflow(llm, replicas=2)
        serve = Serve(agents=[mgr], config={"max_concurrent_tasks": 8, "analyze_tasks": False,
                                            "evaluate_results": False})
        await serve.start()
        ft = FaultTolerance(mgr, {"health_check_interval": 0.05, "heartbeat_timeout": 1.0,
                                  "resource_threshold": 1.0})
        await ft.start()

        async def one(i):
            return await serve.execute_task({"type": "document_workflow", "document": f"doc {i} revenue grew"})

        first = await asyncio.gather(*(one(i) for i in range(8)))
        victim = next(k for k in kids if k.stage == "analyze")
        await victim.stop()  # crash
        second = await asyncio.gather(*(one(i) for i in range(8, 24)))
        await asyncio.sleep(0.3)
        m = ft.get_health_metrics()
        await ft.stop()
        await mgr.delegator.stop()
        await serve.stop()
        return first + second, m, mgr, victim

    results, m, mgr, victim = asyncio.run(main())
    assert all(r.success for r in results), [r.error for r in results if not r.success]
    for r in results:
        assert set(r.output) == set(STAGES)
        assert r.output["analyze"]["risk"] in ("low", "medium", "high")
        assert len(r.output["summarize"]["action_items"]) == 2
    assert m["replacements"] >= 1
    assert victim.id not in mgr.child_agents
    assert sum(1 for k in mgr.child_agents.values() if k.stage == "analyze") == 2

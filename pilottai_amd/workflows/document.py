"""Hierarchical document workflow: extract -> analyze -> summarize (BASELINE
config 5; the reference's hierarchical example is
docs/examples/pdf_processing/example_agents.py:13-112).

    Serve ──► WorkflowManager (orchestrator, can_delegate)
                 │ TaskDelegator: per stage, the best live child whose
                 │ specialisation matches (suitability x load x success rate)
                 ├── StageAgent "extract"   x replicas
                 ├── StageAgent "analyze"   x replicas
                 └── StageAgent "summarize" x replicas

Each stage is one schema-constrained LLM call (source/rules.yaml `workflow:`)
whose prompt starts with the document, so the document's KV blocks are computed
once and shared by all stages through the engine's prefix cache. A stage that
fails (e.g. its agent crashed mid-task) is re-delegated to another replica; a
dead child is replaced by FaultTolerance through `WorkflowManager.create_agent`.
"""
from __future__ import annotations

import asyncio
import json
import time
from typing import Any, Dict, List, Optional, Tuple

from pilottai_amd.core.agent import BaseAgent
from pilottai_amd.core.config import AgentConfig
from pilottai_amd.core.prompts import PromptManager, parse_json_response
from pilottai_amd.core.role import AgentRole
from pilottai_amd.core.task import Task, TaskResult
from pilottai_amd.delegation.task_delegator import TaskDelegator

STAGES = ("extract", "analyze", "summarize")
_PROMPTS: Optional[PromptManager] = None


def _prompts() -> PromptManager:
    global _PROMPTS
    if _PROMPTS is None:
        _PROMPTS = PromptManager("workflow")
    return _PROMPTS


class StageAgent(BaseAgent):
    """One workflow stage = one structured LLM call."""

    def __init__(self, stage: str, *a, **kw):
        if stage not in STAGES:
            raise ValueError(f"unknown stage {stage!r}")
        self.stage = stage
        super().__init__(*a, **kw)

    async def execute_task(self, task) -> TaskResult:
        task = Task.from_any(task)
        if self.status == "stopped":
            return TaskResult(success=False, error=f"agent {self.id} is stopped")
        t0 = time.perf_counter()
        self.active_tasks.add(task.id)
        try:
            md = task.metadata
            prompt = _prompts().format_prompt(self.stage, task_description=task.description, role=self.config.role,
                                              facts=json.dumps(md.get("facts", [])),
                                              analysis=json.dumps(md.get("analysis", {})))
            resp = await self.llm.apredict(prompt, response_format={"schema": f"workflow.{self.stage}"})
            out = parse_json_response(resp.get("content") if isinstance(resp, dict) else resp)
            if self.status == "stopped":  # crashed while the call was in flight
                raise RuntimeError(f"agent {self.id} stopped during {self.stage}")
            self.task_metrics["completed"] += 1
            return TaskResult(success=True, output=out, execution_time=time.perf_counter() - t0)
        except Exception as e:  # noqa: BLE001 — reported to the delegator
            self.task_metrics["failed"] += 1
            self.last_error = str(e)
            return TaskResult(success=False, error=str(e), execution_time=time.perf_counter() - t0)
        finally:
            self.active_tasks.discard(task.id)


class WorkflowManager(BaseAgent):
    concurrent_safe = True  # delegates: many workflows may run through one manager

    def __init__(self, *a, stage_retries: int = 3, **kw):
        super().__init__(*a, **kw)
        self.delegator = TaskDelegator(self)
        self.stage_retries = stage_retries
        self.stage_failures = 0

    async def evaluate_task_suitability(self, task) -> float:
        return 1.0

    async def _run_stage(self, stage: str, doc: str, ctx: Dict[str, Any],
                         wait_s: float = 120.0) -> Tuple[TaskResult, Optional[str]]:
        last: Optional[TaskResult] = None
        failures = 0
        deadline = time.monotonic() + wait_s
        while failures < self.stage_retries and time.monotonic() < deadline:
            sub = Task(description=doc, required_skills=[stage], metadata={"type": stage, **ctx})
            res = await self.delegator.delegate(sub)
            if res is None:  # no live replica of this stage right now (e.g. being replaced)
                await asyncio.sleep(0.02)
                continue
            if res.success:
                return res, None
            failures += 1
            self.stage_failures += 1
            last = res
        return last or TaskResult(success=False, error=f"no agent for stage {stage}"), stage

    async def execute_task(self, task) -> TaskResult:
        task = Task.from_any(task)
        t0 = time.perf_counter()
        doc = task.metadata.get("document") or task.description
        out: Dict[str, Any] = {}
        ctx: Dict[str, Any] = {}
        for stage in STAGES:
            res, failed = await self._run_stage(stage, doc, ctx)
            if failed:
                return TaskResult(success=False, error=f"{stage} failed: {res.error}", output=out,
                                  execution_time=time.perf_counter() - t0)
            out[stage] = res.output
            if stage == "extract":
                ctx["facts"] = (res.output or {}).get("facts", [])
            elif stage == "analyze":
                ctx["analysis"] = res.output
        self.task_metrics["completed"] += 1
        return TaskResult(success=True, output=out, execution_time=time.perf_counter() - t0)

    async def create_agent(self, role: Optional[str] = None, agent_type: Optional[str] = None, **kw) -> BaseAgent:
        """FaultTolerance replacement hook: a fresh replica of the failed stage."""
        stage = next((s for s in STAGES if role and role.startswith(s)), "extract")
        return _stage_agent(stage, f"{stage}-r{int(time.time() * 1000) % 100000}", self._llm)


def _stage_agent(stage: str, role: str, llm) -> StageAgent:
    cfg = AgentConfig(role=role, role_type=AgentRole.WORKER, goal=f"{stage} documents",
                      specializations=[stage], max_queue_size=1000, max_concurrent_tasks=1024)
    return StageAgent(stage, cfg, llm=llm)


async def build_document_workflow(llm, replicas: int = 2) -> Tuple[WorkflowManager, List[StageAgent]]:
    mgr = WorkflowManager(AgentConfig(role="workflow-manager", role_type=AgentRole.ORCHESTRATOR,
                                      goal="Run extract -> analyze -> summarize", can_delegate=True,
                                      max_child_agents=64, max_concurrent_tasks=1024), llm=llm)
    kids = []
    for stage in STAGES:
        for r in range(replicas):
            a = _stage_agent(stage, f"{stage}-{r}", llm)
            await mgr.add_child_agent(a)
            kids.append(a)
    await mgr.delegator.start()
    return mgr, kids

"""Control policy: which reply fields the caller pins instead of the model.

Every control decision of the orchestrator/agent loop is read from an LLM JSON
reply. Two policies:

* ``model`` (default) — the model decides all control fields; only fields that
  must name existing entities (tool names) are pinned by the caller.
* ``fixed`` — deterministic control flow for benchmarks and reproducible runs
  (random-init weights): no decomposition, `steps_per_task` tool steps, success
  verdicts, no orchestrator retry. The amount of LLM work per task is then fixed:
  7 calls (orchestrator analysis + evaluation, agent analysis, tool selection,
  steps_per_task+1 step plans, agent evaluation), each bounded by its schema.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict, List, Sequence


@dataclass
class ControlPolicy:
    mode: str = "model"
    steps_per_task: int = 1
    decompose: bool = False

    @property
    def fixed_mode(self) -> bool:
        return self.mode == "fixed"

    def orchestrator_analysis(self, task_meta: Dict[str, Any]) -> Dict[str, Any]:
        if "decompose" in task_meta:
            return {"requires_decomposition": bool(task_meta["decompose"])}
        return {"requires_decomposition": self.decompose} if self.fixed_mode else {}

    def orchestrator_evaluation(self, success: bool) -> Dict[str, Any]:
        return {"success": bool(success), "requires_retry": not success} if self.fixed_mode else {}

    def agent_analysis(self) -> Dict[str, Any]:
        return {"can_execute": True} if self.fixed_mode else {}

    def tool_selection(self, tools: Sequence[str]) -> Dict[str, Any]:
        names: List[str] = list(tools)
        return {"selected_tools": names, "execution_sequence": names} if names else {}

    def step_planning(self, step_index: int, tool: str) -> Dict[str, Any]:
        fixed: Dict[str, Any] = {"next_step.tool": tool}
        if self.fixed_mode:
            fixed["task_complete"] = step_index >= self.steps_per_task
            fixed["next_step.inputs"] = {}
        return fixed

    def agent_evaluation(self) -> Dict[str, Any]:
        return {"success": True} if self.fixed_mode else {}


DEFAULT_POLICY = ControlPolicy()


# The agent a task is bound to (speculatively reserved or executing), visible to the
# manager-side LLM calls the orchestrator makes for that task (its analysis and its
# evaluation): the node plane's DistributedLLM sends them to that agent's rank, where the
# task's prompt prefix is already in the engine's prefix cache.
from contextvars import ContextVar  # noqa: E402

TASK_AGENT: ContextVar = ContextVar("pilottai_task_agent", default=None)

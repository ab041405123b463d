"""Score-based task router (reference: pilott/core/router.py:15-145).

score = 0.4*suitability + 0.3*(1 - load_penalty) + 0.2*specialisation + 0.1*success_rate
load_penalty = min(1, 0.5*queue_util + 0.3*cpu + 0.2*mem); an agent is viable
while queue_util < load_threshold; scores are cached for load_check_interval s.
Works with `agents` as a dict or a list (the reference never returned an agent
for either, App. A #29). The per-agent load inputs can come from the GPU side:
an agent backed by the local engine reports KV-cache utilisation, which is
folded into `mem`.
"""
from __future__ import annotations

import asyncio
import logging
import time
from typing import Any, Dict, Iterable, Optional

from pydantic import BaseModel, Field

from .task import TaskPriority


class RouterConfig(BaseModel):
    load_check_interval: float = Field(default=5, ge=0)
    max_queue_size: int = Field(default=100, gt=0)
    routing_timeout: float = Field(default=30, gt=0)
    max_retry_attempts: int = Field(default=3, ge=0)
    load_threshold: float = Field(default=0.8, ge=0.0, le=1.0)
    retry_delay: float = Field(default=1.0, ge=0.0)


def _agents_of(owner: Any) -> Iterable[Any]:
    agents = getattr(owner, "child_agents", None)
    if not agents:
        agents = getattr(owner, "agents", None)
    if agents is None:
        return []
    if isinstance(agents, dict):
        return list(agents.values())
    return list(agents)


class TaskRouter:
    def __init__(self, pilott: Any, config: Optional[Dict] = None):
        self.pilott = pilott
        self.config = RouterConfig(**(config or {}))
        self.agent_scores: Dict[str, float] = {}
        self.last_check: Dict[str, float] = {}
        self._metrics_cache: Dict[str, Any] = {}
        self._lock = asyncio.Lock()
        self.logger = logging.getLogger("pilottai_amd.router")
        self.routed = 0

    async def _metrics(self, agent) -> Dict[str, Any]:
        now = time.monotonic()
        hit = self._metrics_cache.get(agent.id)
        if hit and now - hit[0] < self.config.load_check_interval:
            return hit[1]
        m = await agent.get_metrics()
        self._metrics_cache[agent.id] = (now, m)
        return m

    async def route_task(self, task: Dict[str, Any]) -> Optional[str]:
        async def attempt_all():
            for attempt in range(max(1, self.config.max_retry_attempts)):
                aid = await self._attempt_routing(task)
                if aid:
                    self.routed += 1
                    return aid
                if attempt < self.config.max_retry_attempts - 1:
                    await asyncio.sleep(self.config.retry_delay)
            return None

        try:
            async with self._lock:
                return await asyncio.wait_for(attempt_all(), self.config.routing_timeout)
        except asyncio.TimeoutError:
            raise RuntimeError("Task routing timed out")

    async def select_agent(self, task: Dict[str, Any]):
        aid = await self._attempt_routing(task)
        if aid is None:
            return None
        for a in _agents_of(self.pilott):
            if a.id == aid:
                return a
        return None

    async def _attempt_routing(self, task: Dict[str, Any]) -> Optional[str]:
        scores = await self._calculate_agent_scores(task)
        best, best_s = None, -1.0
        for aid, s in scores.items():
            if s > best_s:
                best, best_s = aid, s
        return best

    async def _calculate_agent_scores(self, task: Dict[str, Any]) -> Dict[str, float]:
        now = time.monotonic()
        scores: Dict[str, float] = {}
        for agent in _agents_of(self.pilott):
            if str(getattr(agent, "status", "idle")) in ("busy", "stopped", "error"):
                continue
            try:
                m = await self._metrics(agent)
                if m.get("queue_utilization", 1.0) >= self.config.load_threshold:
                    continue
                if agent.id in self.agent_scores and now - self.last_check.get(agent.id, -1e9) < \
                        self.config.load_check_interval:
                    scores[agent.id] = self.agent_scores[agent.id]
                    continue
                base = await agent.evaluate_task_suitability(task)
                s = (0.4 * base + 0.3 * (1.0 - self._load_penalty(m)) + 0.2 * self._spec_bonus(agent, task)
                     + 0.1 * float(m.get("success_rate", 0.5)))
                scores[agent.id] = s
                self.agent_scores[agent.id] = s
                self.last_check[agent.id] = now
            except Exception as e:  # noqa: BLE001
                self.logger.debug("score failed for %s: %s", getattr(agent, "id", "?"), e)
        return scores

    @staticmethod
    def _load_penalty(m: Dict[str, Any]) -> float:
        mem = max(float(m.get("memory_usage", 1.0)), float(m.get("kv_cache_utilization", 0.0)))
        return min(1.0, 0.5 * float(m.get("queue_utilization", 1.0)) + 0.3 * float(m.get("cpu_usage", 1.0)) + 0.2 * mem)

    @staticmethod
    def _spec_bonus(agent, task: Dict[str, Any]) -> float:
        specs = set(getattr(agent, "specializations", []) or [])
        if not specs:
            return 0.0
        if task.get("type") in specs:
            return 0.3
        return 0.1 * len(set(task.get("tags", [])) & specs)

    @staticmethod
    def get_task_priority(task: Dict[str, Any]) -> TaskPriority:
        if task.get("urgent", False):
            return TaskPriority.CRITICAL
        c = task.get("complexity", 1) or 1
        d = len(task.get("dependencies", []) or [])
        if c > 8 or d > 5:
            return TaskPriority.HIGH
        if c > 5 or d > 3:
            return TaskPriority.MEDIUM
        return TaskPriority.LOW

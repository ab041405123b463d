"""Dynamic agent-pool scaling (reference: pilott/orchestration/orchestration.py:10-337,
duplicated in scaling.py:425-666 — one implementation here).

load  = min(1, 0.35*avg_queue_util + 0.25*cpu + 0.25*mem + 0.15*total_queue/(n*100))
trend = sum(i*load_i)/sum(i) over the last 5 samples (linearly weighted)
trend > up  -> create_agent() + add_child_agent() x scale_up_increment (<= max_agents)
trend < down-> retire idle agents with the lowest success rate (>= min_agents)
with a cooldown between scaling actions (total seconds, not timedelta.seconds, App. A #35).
On the GPU path `mem` includes the serving engine's KV-cache utilisation, so the
pool grows when agents queue on the continuous batch, not only on host load.
"""
from __future__ import annotations

import asyncio
import logging
from datetime import datetime, timedelta
from typing import Any, Dict, List, Optional

import psutil
from pydantic import BaseModel, Field


class ScalingMetrics(BaseModel):
    timestamp: datetime = Field(default_factory=datetime.now)
    system_load: float = 0.0
    num_agents: int = 0
    queue_size: int = 0
    avg_queue_utilization: float = 0.0


class ScalingConfig(BaseModel):
    scale_up_threshold: float = Field(default=0.8, ge=0, le=1)
    scale_down_threshold: float = Field(default=0.3, ge=0, le=1)
    min_agents: int = Field(default=2, ge=1)
    max_agents: int = Field(default=10, ge=1)
    cooldown_period: float = Field(default=300, ge=0)
    check_interval: float = Field(default=60, gt=0)
    scale_up_increment: int = Field(default=1, ge=1)
    scale_down_increment: int = Field(default=1, ge=1)
    metrics_retention_period: float = Field(default=3600, gt=0)


class DynamicScaling:
    def __init__(self, orchestrator: Any, config: Optional[Dict[str, Any]] = None):
        self.orchestrator = orchestrator
        self.config = ScalingConfig(**(config or {}))
        self.running = False
        self._task: Optional[asyncio.Task] = None
        self.metrics_history: List[ScalingMetrics] = []
        self.last_scaling_time = datetime.min
        self.scale_ups = 0
        self.scale_downs = 0
        self._lock = asyncio.Lock()
        self.logger = logging.getLogger("pilottai_amd.scaling")

    def _agents(self) -> Dict[str, Any]:
        ca = getattr(self.orchestrator, "child_agents", None)
        return ca if isinstance(ca, dict) else {}

    async def start(self):
        if not self.running:
            self.running = True
            self._task = asyncio.create_task(self._scaling_loop())

    async def stop(self):
        self.running = False
        if self._task:
            self._task.cancel()
            try:
                await self._task
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
            self._task = None

    async def _scaling_loop(self):
        while self.running:
            try:
                await self._check_and_adjust_scale()
            except asyncio.CancelledError:
                raise
            except Exception as e:  # noqa: BLE001
                self.logger.error("scaling error: %s", e)
            await asyncio.sleep(self.config.check_interval)

    async def _get_system_load(self) -> float:
        agents = [a for a in self._agents().values() if str(getattr(a, "status", "")) not in ("stopped", "error")]
        n = len(agents)
        cpu = psutil.cpu_percent(interval=None) / 100.0
        mem = psutil.virtual_memory().percent / 100.0
        if n == 0:
            return min(1.0, 0.25 * cpu + 0.25 * mem)
        qu, total_q = 0.0, 0
        for a in agents:
            try:
                m = await a.get_metrics()
            except Exception:  # noqa: BLE001
                continue
            qu += float(m.get("queue_utilization", 0.0))
            total_q += int(m.get("queue_size", 0))
            mem = max(mem, float(m.get("kv_cache_utilization", 0.0)))
        return min(1.0, 0.35 * qu / n + 0.25 * cpu + 0.25 * mem + 0.15 * total_q / (n * 100))

    def _analyze_load_trend(self) -> float:
        h = self.metrics_history[-5:]
        if not h:
            return 0.0
        w = list(range(1, len(h) + 1))
        return sum(wi * m.system_load for wi, m in zip(w, h)) / sum(w)

    def _can_scale(self) -> bool:
        return (datetime.now() - self.last_scaling_time).total_seconds() >= self.config.cooldown_period

    async def _check_and_adjust_scale(self):
        async with self._lock:
            load = await self._get_system_load()
            self.metrics_history.append(ScalingMetrics(system_load=load, num_agents=len(self._agents())))
            cutoff = datetime.now() - timedelta(seconds=self.config.metrics_retention_period)
            self.metrics_history = [m for m in self.metrics_history if m.timestamp > cutoff]
            if not self._can_scale():
                return
            trend = self._analyze_load_trend()
            if trend > self.config.scale_up_threshold:
                await self._scale_up()
            elif trend < self.config.scale_down_threshold:
                await self._scale_down()

    async def _scale_up(self):
        n = len(self._agents())
        added = 0
        for _ in range(self.config.scale_up_increment):
            if n + added >= self.config.max_agents:
                break
            agent = await self.orchestrator.create_agent()
            await self.orchestrator.add_child_agent(agent)
            added += 1
        if added:
            self.scale_ups += added
            self.last_scaling_time = datetime.now()
            self.logger.info("scaled up by %d agents", added)

    async def _scale_down(self):
        agents = self._agents()
        removable = len(agents) - self.config.min_agents
        if removable <= 0:
            return
        idle = []
        for aid, a in list(agents.items()):
            if str(getattr(a, "status", "")) == "idle" and not getattr(a, "active_tasks", None):
                m = await a.get_metrics()
                idle.append((float(m.get("success_rate", 0.0)), aid, a))
        idle.sort(key=lambda x: x[0])
        removed = 0
        for _, aid, a in idle[: min(removable, self.config.scale_down_increment)]:
            await self._safely_remove_agent(aid, a)
            removed += 1
        if removed:
            self.scale_downs += removed
            self.last_scaling_time = datetime.now()
            self.logger.info("scaled down by %d agents", removed)

    async def _safely_remove_agent(self, aid: str, agent):
        if hasattr(agent, "pause_task_acceptance"):
            await agent.pause_task_acceptance()
        if hasattr(agent, "wait_for_tasks"):
            try:
                await agent.wait_for_tasks(timeout=60)
            except Exception:  # noqa: BLE001
                pass
        await agent.stop()
        await self.orchestrator.remove_child_agent(aid)

    def get_scaling_metrics(self) -> Dict[str, Any]:
        cur = self.metrics_history[-1] if self.metrics_history else None
        return {"current_load": cur.system_load if cur else 0.0, "num_agents": len(self._agents()),
                "load_trend": self._analyze_load_trend(), "scale_ups": self.scale_ups,
                "scale_downs": self.scale_downs,
                "last_scaling_time": None if self.last_scaling_time == datetime.min else self.last_scaling_time.isoformat(),
                "running": self.running}

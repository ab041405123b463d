"""Load balancer (reference: pilott/orchestration/load_balancer.py:13-391).

Every `check_interval` s: sample each agent, pause agents over the overload
threshold (and resume them once they cool down — the reference never resumed),
classify agents as overloaded (composite load > 0.8 and rising) or underloaded
(< 0.2 and falling), and move up to `balance_batch_size` queued, unlocked tasks
(highest priority first) from each overloaded agent to the best underloaded one,
with backup/restore on failure.

composite load = 0.3*cpu + 0.3*mem + 0.2*queue/max_tasks_per_agent + 0.2*error_rate
target score   = 0.4*suitability + 0.3*(1-load) + 0.2*(1-error_rate) + 0.1*(1-max(cpu,mem))
(SURVEY App. C). On the GPU path `mem` is max(host memory, KV-cache utilisation)
of the engine that serves the agent. Host CPU/memory are sampled once per tick
without blocking (the reference blocked the event loop 1 s per agent, App. A #33).
"""
from __future__ import annotations

import asyncio
import logging
from datetime import datetime, timedelta
from typing import Any, Dict, List, Optional, Tuple

import psutil
from pydantic import BaseModel, Field


class LoadMetrics(BaseModel):
    cpu_usage: float = 0.0
    memory_usage: float = 0.0
    queue_size: int = 0
    active_tasks: int = 0
    total_tasks: int = 0
    error_rate: float = 0.0
    timestamp: datetime = Field(default_factory=datetime.now)


class LoadBalancerConfig(BaseModel):
    check_interval: float = Field(default=30, gt=0)
    overload_threshold: float = Field(default=0.8, ge=0, le=1)
    underload_threshold: float = Field(default=0.2, ge=0, le=1)
    max_tasks_per_agent: int = Field(default=10, gt=0)
    balance_batch_size: int = Field(default=3, gt=0)
    min_load_difference: float = Field(default=0.3, ge=0, le=1)
    metrics_retention_period: float = Field(default=3600, gt=0)
    task_move_timeout: float = Field(default=30, gt=0)


def _agents(orch) -> Dict[str, Any]:
    ca = getattr(orch, "child_agents", None)
    return ca if isinstance(ca, dict) else {}


class LoadBalancer:
    def __init__(self, orchestrator: Any, config: Optional[Dict[str, Any]] = None):
        self.orchestrator = orchestrator
        self.config = LoadBalancerConfig(**(config or {}))
        self.running = False
        self._task: Optional[asyncio.Task] = None
        self._lock = asyncio.Lock()
        self._history: Dict[str, List[LoadMetrics]] = {}
        self._paused: set = set()
        self._last_balance: Optional[datetime] = None
        self.moves = 0
        self.logger = logging.getLogger("pilottai_amd.load_balancer")

    async def start(self):
        if self.running:
            return
        self.running = True
        self._task = asyncio.create_task(self._balancing_loop())

    async def stop(self):
        self.running = False
        if self._task:
            self._task.cancel()
            try:
                await self._task
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
            self._task = None

    async def _balancing_loop(self):
        while self.running:
            try:
                async with self._lock:
                    await self._balance_system_load()
            except asyncio.CancelledError:
                raise
            except Exception as e:  # noqa: BLE001
                self.logger.error("balancing error: %s", e)
            await asyncio.sleep(self.config.check_interval)

    async def _balance_system_load(self):
        metrics = await self._collect_system_metrics()
        self._update_metrics_history(metrics)
        over, under = self._analyze_agent_loads(metrics)
        if over and under:
            await self._redistribute_tasks(over, under, metrics)

    async def _collect_system_metrics(self) -> Dict[str, LoadMetrics]:
        sys_cpu = psutil.cpu_percent(interval=None) / 100.0
        sys_mem = psutil.virtual_memory().percent / 100.0
        out: Dict[str, LoadMetrics] = {}
        for aid, agent in list(_agents(self.orchestrator).items()):
            if str(getattr(agent, "status", "")) in ("stopped", "error"):
                continue
            try:
                m = await agent.get_metrics()
                lm = LoadMetrics(cpu_usage=max(sys_cpu, float(m.get("cpu_usage", 0.0))),
                                 memory_usage=max(sys_mem, float(m.get("memory_usage", 0.0)),
                                                  float(m.get("kv_cache_utilization", 0.0))),
                                 queue_size=int(m.get("queue_size", 0)), active_tasks=int(m.get("active_tasks", 0)),
                                 total_tasks=int(m.get("total_tasks", 0)),
                                 error_rate=1.0 - float(m.get("success_rate", 1.0)) if m.get("total_tasks") else 0.0)
                out[aid] = lm
                if max(lm.cpu_usage, lm.memory_usage) > self.config.overload_threshold:
                    await self._handle_overload(aid)
                elif aid in self._paused:
                    await self._resume(aid)
            except Exception as e:  # noqa: BLE001
                self.logger.error("metrics for %s failed: %s", aid, e)
        return out

    async def _handle_overload(self, aid: str):
        agent = _agents(self.orchestrator).get(aid)
        if agent is not None and aid not in self._paused:
            await agent.pause_task_acceptance()
            self._paused.add(aid)
            self.logger.warning("agent %s paused (resource overload)", aid)

    async def _resume(self, aid: str):
        agent = _agents(self.orchestrator).get(aid)
        self._paused.discard(aid)
        if agent is not None and hasattr(agent, "resume_task_acceptance"):
            await agent.resume_task_acceptance()

    def _update_metrics_history(self, metrics: Dict[str, LoadMetrics]):
        cutoff = datetime.now() - timedelta(seconds=self.config.metrics_retention_period)
        for aid, m in metrics.items():
            h = self._history.setdefault(aid, [])
            h.append(m)
            self._history[aid] = [x for x in h if x.timestamp > cutoff]

    def _calculate_composite_load(self, m: LoadMetrics) -> float:
        return (0.3 * m.cpu_usage + 0.3 * m.memory_usage + 0.2 * (m.queue_size / self.config.max_tasks_per_agent)
                + 0.2 * m.error_rate)

    def _calculate_load_trend(self, aid: str) -> float:
        h = self._history.get(aid, [])[-5:]
        if len(h) < 2:
            return 0.0
        loads = [self._calculate_composite_load(m) for m in h]
        return (loads[-1] - loads[0]) / len(loads)

    def _analyze_agent_loads(self, metrics: Dict[str, LoadMetrics]) -> Tuple[List[str], List[str]]:
        over, under = [], []
        for aid, m in metrics.items():
            load, trend = self._calculate_composite_load(m), self._calculate_load_trend(aid)
            if load > self.config.overload_threshold and trend > 0:
                over.append(aid)
            elif load < self.config.underload_threshold and trend < 0:
                under.append(aid)
        return over, under

    @staticmethod
    def _is_task_moveable(task) -> bool:
        st = getattr(task, "status", None) if not isinstance(task, dict) else task.get("status")
        locked = task.get("locked") if isinstance(task, dict) else getattr(task, "metadata", {}).get("locked")
        return str(getattr(st, "value", st)) in ("pending", "None") and not locked

    async def _get_moveable_tasks(self, aid: str) -> List[Any]:
        agent = _agents(self.orchestrator).get(aid)
        if agent is None:
            return []
        active = getattr(agent, "active_tasks", set())
        return [t for tid, t in list(getattr(agent, "tasks", {}).items())
                if tid not in active and self._is_task_moveable(t)]

    async def _find_best_agent(self, task, candidates: List[str], metrics: Dict[str, LoadMetrics]) -> Optional[str]:
        best, best_s = None, -1.0
        for aid in candidates:
            agent = _agents(self.orchestrator).get(aid)
            m = metrics.get(aid)
            if agent is None or m is None or not self._can_accept_task(agent, m):
                continue
            suit = await agent.evaluate_task_suitability(task if isinstance(task, dict) else task)
            load = self._calculate_composite_load(m)
            s = 0.4 * suit + 0.3 * (1 - load) + 0.2 * (1 - m.error_rate) + 0.1 * (1 - max(m.cpu_usage, m.memory_usage))
            if s > best_s:
                best, best_s = aid, s
        return best

    def _can_accept_task(self, agent, m: LoadMetrics) -> bool:
        return (str(getattr(agent, "status", "")) not in ("stopped", "error")
                and m.queue_size < self.config.max_tasks_per_agent
                and self._calculate_composite_load(m) < self.config.overload_threshold)

    async def _redistribute_tasks(self, over: List[str], under: List[str], metrics: Dict[str, LoadMetrics]):
        for src in over:
            tasks = await self._get_moveable_tasks(src)
            tasks.sort(key=lambda t: getattr(getattr(t, "priority", None), "rank", 0), reverse=True)
            moved = 0
            for t in tasks:
                if moved >= self.config.balance_batch_size:
                    break
                dst = await self._find_best_agent(t, under, metrics)
                if dst is None:
                    continue
                try:
                    await asyncio.wait_for(self._move_task(t, src, dst), self.config.task_move_timeout)
                    moved += 1
                except Exception as e:  # noqa: BLE001
                    self.logger.error("move of %s failed: %s", getattr(t, "id", "?"), e)
            if moved:
                self._last_balance = datetime.now()
                self.moves += moved

    async def _move_task(self, task, src: str, dst: str):
        agents = _agents(self.orchestrator)
        a, b = agents[src], agents[dst]
        tid = task["id"] if isinstance(task, dict) else task.id
        meta = task if isinstance(task, dict) else task.metadata
        meta["locked"] = True
        removed = False
        try:
            await a.remove_task(tid)
            removed = True
            await b.add_task(task)
            meta.update(moved_at=datetime.now().isoformat(), moved_from=src, moved_to=dst)
        except Exception:
            if removed:
                try:
                    await a.add_task(task)  # restore on the source agent
                except Exception as e:  # noqa: BLE001
                    self.logger.error("restore of %s failed: %s", tid, e)
            raise
        finally:
            meta["locked"] = False

    def get_metrics(self) -> Dict[str, Any]:
        latest = {aid: h[-1] for aid, h in self._history.items() if h}
        loads = [self._calculate_composite_load(m) for m in latest.values()]
        return {"running": self.running, "agents": len(latest),
                "average_load": sum(loads) / len(loads) if loads else 0.0,
                "max_load": max(loads) if loads else 0.0, "paused_agents": sorted(self._paused),
                "tasks_moved": self.moves,
                "last_balance": self._last_balance.isoformat() if self._last_balance else None}

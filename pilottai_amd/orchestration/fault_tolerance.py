"""Failure detection and recovery (reference: pilott/orchestration/scaling.py:34-423).

Every `health_check_interval` s each registered agent is classified:
    heartbeat missing / older than heartbeat_timeout -> CRITICAL
    resource usage > resource_threshold              -> CRITICAL
    serving GPU engine failed / wedged               -> CRITICAL   (GPU probe)
    stuck tasks (non-terminal older than task_timeout) -> DEGRADED
    error count > error_threshold                    -> UNHEALTHY
Non-healthy agents are recovered in place (stop -> reset -> start -> re-check)
while attempts < max_recovery_attempts, the fresh status is not CRITICAL and the
cooldown has passed; otherwise they are replaced: a new agent of the same role is
created through the orchestrator, pending and in-progress tasks are transferred,
and the registration is swapped. Agents implement `send_heartbeat` (missing in
the reference, App. A #30) and the decision uses the fresh status (App. A #31).
"""
from __future__ import annotations

import asyncio
import logging
import threading
import time
from datetime import datetime, timedelta
from enum import Enum
from typing import Any, Dict, List, Optional

from pydantic import BaseModel, Field, model_validator


class HealthStatus(str, Enum):
    HEALTHY = "healthy"
    DEGRADED = "degraded"
    UNHEALTHY = "unhealthy"
    CRITICAL = "critical"


class AgentHealth(BaseModel):
    agent_id: str
    status: HealthStatus = HealthStatus.HEALTHY
    last_heartbeat: datetime = Field(default_factory=datetime.now)
    error_count: int = 0
    recovery_attempts: int = 0
    last_recovery: Optional[datetime] = None
    resource_usage: float = 0.0
    details: Dict[str, Any] = Field(default_factory=dict)


class FaultToleranceConfig(BaseModel):
    health_check_interval: float = Field(default=30, gt=0)
    max_recovery_attempts: int = Field(default=3, ge=0)
    recovery_attempts: Optional[int] = Field(default=None, ge=0)  # README spelling (App. A #42)
    recovery_cooldown: float = Field(default=300, ge=0)
    heartbeat_timeout: float = Field(default=60, gt=0)
    resource_threshold: float = Field(default=0.9, ge=0, le=1)
    task_timeout: float = Field(default=1800, gt=0)
    error_threshold: int = Field(default=5, ge=0)
    metrics_retention: float = Field(default=3600, gt=0)
    engine_stall_timeout: float = Field(default=120, gt=0)

    @model_validator(mode="after")
    def _alias(self):
        if self.recovery_attempts is not None:
            self.max_recovery_attempts = self.recovery_attempts
        return self


class GPUHealthProbe:
    """Liveness of the local inference engine behind an agent.

    CRITICAL when the engine loop crashed (`engine.failed`), or when it holds
    work but has not completed a step for `stall_timeout` s (a wedged kernel or
    collective). `device_ok()` runs a tiny kernel + synchronize in a watchdog
    thread so a hung GPU cannot block the event loop.
    """

    def __init__(self, stall_timeout: float = 120.0):
        self.stall_timeout = stall_timeout
        self._last: Dict[int, tuple] = {}

    def engine_of(self, agent) -> Any:
        llm = vars(agent).get("_llm") if hasattr(agent, "__dict__") else None  # never trigger lazy LLM creation
        return getattr(llm, "engine", None)

    def check(self, agent) -> Optional[str]:
        eng = self.engine_of(agent)
        if eng is None:
            return None
        if getattr(eng, "failed", None) is not None:
            return f"engine failed: {eng.failed!r}"
        steps = eng.stats.get("steps", 0)
        busy = (eng.sched.has_work() if hasattr(eng, "sched") else False) or \
            not getattr(eng, "_inbox", None) is None and not eng._inbox.empty()
        now = time.monotonic()
        prev = self._last.get(id(eng))
        if prev is None or prev[0] != steps or not busy:
            self._last[id(eng)] = (steps, now)
        elif now - prev[1] > self.stall_timeout:
            return f"engine stalled for {now - prev[1]:.0f}s with work pending"
        return None

    @staticmethod
    def device_ok(timeout: float = 10.0) -> bool:
        import torch

        if not torch.cuda.is_available():
            return True
        ok = {"v": False}

        def probe():
            try:
                x = torch.ones(16, device="cuda")
                torch.cuda.synchronize()
                ok["v"] = float(x.sum().item()) == 16.0
            except Exception:  # noqa: BLE001
                ok["v"] = False

        t = threading.Thread(target=probe, daemon=True)
        t.start()
        t.join(timeout)
        return ok["v"] and not t.is_alive()


class FaultTolerance:
    def __init__(self, orchestrator: Any, config: Optional[Dict[str, Any]] = None):
        self.orchestrator = orchestrator
        self.config = FaultToleranceConfig(**(config or {}))
        self.agent_health: Dict[str, AgentHealth] = {}
        self.recovery_history: List[Dict[str, Any]] = []
        self.running = False
        self._task: Optional[asyncio.Task] = None
        self._lock = asyncio.Lock()
        self.gpu_probe = GPUHealthProbe(self.config.engine_stall_timeout)
        self.replacements = 0
        self.recoveries = 0
        self.logger = logging.getLogger("pilottai_amd.fault_tolerance")

    def _agents(self) -> Dict[str, Any]:
        ca = getattr(self.orchestrator, "child_agents", None)
        return ca if isinstance(ca, dict) else {}

    async def start(self):
        if not self.running:
            self.running = True
            self._task = asyncio.create_task(self._monitoring_loop())

    async def stop(self):
        self.running = False
        if self._task:
            self._task.cancel()
            try:
                await self._task
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
            self._task = None

    async def register_agent(self, agent):
        self.agent_health[agent.id] = AgentHealth(agent_id=agent.id)

    async def unregister_agent(self, agent_id: str):
        self.agent_health.pop(agent_id, None)

    async def _monitoring_loop(self):
        while self.running:
            try:
                await self._check_system_health()
            except asyncio.CancelledError:
                raise
            except Exception as e:  # noqa: BLE001
                self.logger.error("health check error: %s", e)
            await asyncio.sleep(self.config.health_check_interval)

    async def _check_system_health(self):
        agents = self._agents()
        for aid, a in agents.items():
            if aid not in self.agent_health:
                await self.register_agent(a)
        for aid in list(self.agent_health):
            agent = agents.get(aid)
            if agent is None:
                await self.unregister_agent(aid)
                continue
            status = await self._check_agent_health(agent)
            if status is not HealthStatus.HEALTHY and status != HealthStatus.HEALTHY:
                await self._handle_unhealthy_agent(agent, status)

    async def _check_agent_health(self, agent) -> HealthStatus:
        h = self.agent_health.setdefault(agent.id, AgentHealth(agent_id=agent.id))
        details: Dict[str, Any] = {}
        hb_ok = await self._check_heartbeat(agent)
        if hb_ok:
            h.last_heartbeat = datetime.now()
        else:
            details["heartbeat"] = "missing"
        try:
            m = await agent.get_metrics()
        except Exception as e:  # noqa: BLE001
            m = {}
            details["metrics_error"] = str(e)
        h.resource_usage = float(m.get("resource_usage", max(m.get("cpu_usage", 0.0), m.get("memory_usage", 0.0))))
        h.error_count = int(m.get("error_count", 0))
        gpu = self.gpu_probe.check(agent)
        if gpu:
            details["gpu"] = gpu
        stuck = self._check_stuck_tasks(agent)
        details["stuck_tasks"] = stuck
        status = self._determine_health_status(hb_ok, h.resource_usage, stuck, h.error_count, gpu)
        h.status = status
        h.details = details
        return status

    def _determine_health_status(self, hb_ok: bool, resource: float, stuck: int, errors: int,
                                 gpu_problem: Optional[str]) -> HealthStatus:
        if not hb_ok or gpu_problem:
            return HealthStatus.CRITICAL
        if resource > self.config.resource_threshold:
            return HealthStatus.CRITICAL
        if stuck > 0:
            return HealthStatus.DEGRADED
        if errors > self.config.error_threshold:
            return HealthStatus.UNHEALTHY
        return HealthStatus.HEALTHY

    async def _check_heartbeat(self, agent) -> bool:
        hb = getattr(agent, "send_heartbeat", None)
        if hb is None:
            return False
        try:
            ts = await asyncio.wait_for(hb(), timeout=min(5.0, self.config.heartbeat_timeout))
            if isinstance(ts, datetime):
                return datetime.now() - ts < timedelta(seconds=self.config.heartbeat_timeout)
            return bool(ts) or ts is None
        except Exception:  # noqa: BLE001
            return False

    def _check_stuck_tasks(self, agent) -> int:
        n = 0
        now = datetime.now()
        tasks = getattr(agent, "tasks", None)
        for t in list(tasks.values()) if isinstance(tasks, dict) else []:
            if self._is_task_stuck(t, now):
                n += 1
        return n

    def _is_task_stuck(self, task, now: datetime) -> bool:
        if isinstance(task, dict):
            st, created = task.get("status"), task.get("created_at")
            if isinstance(created, str):
                created = datetime.fromisoformat(created)
        else:
            st, created = getattr(task, "status", None), getattr(task, "started_at", None) or getattr(task, "created_at", None)
        st = str(getattr(st, "value", st))
        if st in ("completed", "failed", "cancelled", "timeout") or created is None:
            return False
        return (now - created).total_seconds() > self.config.task_timeout

    def _should_attempt_recovery(self, aid: str, status: HealthStatus) -> bool:
        h = self.agent_health.get(aid)
        if h is None or status == HealthStatus.CRITICAL:
            return False
        if h.recovery_attempts >= self.config.max_recovery_attempts:
            return False
        if h.last_recovery and (datetime.now() - h.last_recovery).total_seconds() < self.config.recovery_cooldown:
            return False
        return True

    async def _handle_unhealthy_agent(self, agent, status: Optional[HealthStatus] = None):
        async with self._lock:
            if status is None:
                status = await self._check_agent_health(agent)
            if not isinstance(status, HealthStatus):  # mocked / boolean health checks
                status = HealthStatus.HEALTHY if status else HealthStatus.UNHEALTHY
            if status == HealthStatus.HEALTHY:
                return
            self.agent_health.setdefault(agent.id, AgentHealth(agent_id=agent.id))
            if self._should_attempt_recovery(agent.id, status):
                ok = await self._recover_agent(agent)
                if ok:
                    return
            await self._replace_agent(agent)

    async def _recover_agent(self, agent) -> bool:
        h = self.agent_health[agent.id]
        h.recovery_attempts += 1
        h.last_recovery = datetime.now()
        ok = False
        try:
            await agent.stop()
            await agent.reset()
            await agent.start()
            st = await self._check_agent_health(agent)
            ok = st == HealthStatus.HEALTHY if isinstance(st, HealthStatus) else bool(st)
        except Exception as e:  # noqa: BLE001
            self.logger.error("recovery of %s failed: %s", agent.id, e)
        self._record(agent.id, "recover", ok)
        if ok:
            self.recoveries += 1
        return ok

    async def _replace_agent(self, agent) -> Optional[Any]:
        try:
            role = getattr(getattr(agent, "config", None), "role", None)
            new = await self.orchestrator.create_agent(role=role, agent_type=type(agent).__name__)
            await self._transfer_tasks(agent, new)
            try:
                await agent.stop()
            except Exception:  # noqa: BLE001
                pass
            await self.orchestrator.remove_child_agent(agent.id)
            await self.orchestrator.add_child_agent(new)
            await self.unregister_agent(agent.id)
            await self.register_agent(new)
            self.replacements += 1
            self._record(agent.id, "replace", True, new_agent=new.id)
            return new
        except Exception as e:  # noqa: BLE001
            self.logger.error("replacement of %s failed: %s", getattr(agent, "id", "?"), e)
            self._record(getattr(agent, "id", "?"), "replace", False)
            return None

    async def _transfer_tasks(self, old, new):
        tasks = getattr(old, "tasks", None)
        if not isinstance(tasks, dict):  # the agent protocol's task map; mocks / proxies without one: nothing to move
            return
        for tid, t in list(tasks.items()):
            if not self._is_task_recoverable(t):
                continue
            try:
                if hasattr(old, "remove_task") and tid not in getattr(old, "active_tasks", set()):
                    await old.remove_task(tid)
                await new.add_task(t)
            except Exception as e:  # noqa: BLE001
                self.logger.error("task transfer %s failed: %s", tid, e)

    @staticmethod
    def _is_task_recoverable(task) -> bool:
        st = task.get("status") if isinstance(task, dict) else getattr(task, "status", None)
        return str(getattr(st, "value", st)) in ("pending", "in_progress", "retry", "None")

    def _record(self, aid: str, action: str, ok: bool, **kw):
        self.recovery_history.append({"agent_id": aid, "action": action, "success": ok,
                                      "timestamp": datetime.now().isoformat(), **kw})
        cutoff = datetime.now() - timedelta(seconds=self.config.metrics_retention)
        self.recovery_history = [r for r in self.recovery_history
                                 if datetime.fromisoformat(r["timestamp"]) > cutoff]

    def get_health_metrics(self) -> Dict[str, Any]:
        counts: Dict[str, int] = {s.value: 0 for s in HealthStatus}
        for h in self.agent_health.values():
            counts[h.status.value] += 1
        return {"total_agents": len(self.agent_health), "status": counts, "recoveries": self.recoveries,
                "replacements": self.replacements, "recent_actions": self.recovery_history[-20:],
                "running": self.running}

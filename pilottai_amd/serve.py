"""`Serve` — the orchestrator (reference: pilott/pilott.py:17-697).

Per task: LLM analysis -> (optional) LLM decomposition into subtasks -> priority
queue -> worker pool -> agent reservation -> agent.execute_task -> LLM result
evaluation -> one retry (possibly on another agent) -> memory -> callback.

Both API surfaces of the reference are served:
    Serve(agents=[...], manager_llm=..., config={...});  await add_task(Task) / get_result(id)
    Serve(name=..., verbose=...);  await add_agent(type, config, llm_config);  await execute_task({...})
and Serve implements the orchestrator protocol the control-plane services expect
(child_agents / create_agent / add_child_agent / remove_child_agent),
so LoadBalancer, DynamicScaling, FaultTolerance and TaskDelegator run against it.

Design fixes vs. the reference: concurrency is a real worker pool
bounded by max_concurrent_tasks (#11), agents are reserved atomically (#12), a
failing task never stalls the queue (#13), the queue orders by priority rank
(#16), decomposed parents complete when their subtasks do (#23), every config
field is honoured (#24).
"""
from __future__ import annotations

import asyncio
import itertools
import json
import logging
import time
from collections import defaultdict, deque
from datetime import datetime, timedelta
from typing import Any, Callable, Deque, Dict, List, Optional, Sequence, Union

from pydantic import BaseModel, Field

from .core.agent import BaseAgent, _content, _is_workflow as _is_workflow_task, _resolve_default_llm
from .core.config import AgentConfig, LLMConfig
from .core.errors import AgentLostError
from .core.factory import AgentFactory
from .core.memory import Memory
from .core.policy import DEFAULT_POLICY, TASK_AGENT, ControlPolicy
from .core.prompts import PromptManager, parse_json_response
from .core.role import AgentStatus
from .core.router import TaskRouter
from .core.task import Task, TaskPriority, TaskResult, TaskStatus
from .utils.timeouts import with_timeout


class ServeConfig(BaseModel):
    name: str = "Pilott"
    memory_enabled: bool = True
    verbose: bool = False
    max_concurrent_tasks: int = Field(default=5, gt=0)
    task_timeout: float = Field(default=300, gt=0)
    max_queue_size: int = Field(default=1000, gt=0)
    cleanup_interval: float = Field(default=3600, gt=0)
    task_retention_period: float = Field(default=86400, gt=0)
    max_retry_attempts: int = Field(default=3, ge=0)
    # extensions
    policy: str = "model"            # "model" | "fixed" (core/policy.py)
    steps_per_task: int = Field(default=1, ge=0)
    routing: str = "first_idle"      # "first_idle" | "scored" (TaskRouter)
    analyze_tasks: bool = True       # orchestrator LLM analysis per task
    # start a simple task's agent opening calls (analysis + tool selection: LLM calls
    # without side effects) while the orchestrator analyses the task; dropped if it decomposes
    speculative_start: bool = True
    evaluate_results: bool = True    # orchestrator LLM evaluation per task
    agent_wait_timeout: float = Field(default=60.0, gt=0)
    enable_load_balancer: bool = False
    enable_scaling: bool = False
    enable_fault_tolerance: bool = False
    load_balancer: Dict[str, Any] = Field(default_factory=dict)
    scaling: Dict[str, Any] = Field(default_factory=dict)
    fault_tolerance: Dict[str, Any] = Field(default_factory=dict)
    min_agents: int = 1
    max_agents: int = 1024
    latency_window: int = 100000


class _LatencyStats:
    def __init__(self, n: int):
        self.v: Deque[float] = deque(maxlen=n)

    def add(self, x: float):
        self.v.append(x)

    def pct(self, p: float) -> float:
        if not self.v:
            return 0.0
        s = sorted(self.v)
        return s[min(len(s) - 1, int(p / 100.0 * len(s)))]


class Serve:
    def __init__(self, agents: Optional[Sequence[BaseAgent]] = None, manager_llm: Any = None,
                 manager_agent: Optional[BaseAgent] = None, memory: bool = True,
                 task_callback: Optional[Callable] = None, step_callback: Optional[Callable] = None,
                 config: Optional[Union[Dict[str, Any], ServeConfig]] = None, *, name: Optional[str] = None,
                 verbose: Optional[bool] = None, llm: Any = None):
        if manager_llm is not None and manager_agent is not None:
            raise ValueError("Cannot specify both manager_llm and manager_agent")
        cfg = config if isinstance(config, ServeConfig) else ServeConfig(**(config or {}))
        if name is not None:
            cfg.name = name
        if verbose is not None:
            cfg.verbose = verbose
        self.config = cfg
        self.policy = ControlPolicy(cfg.policy, cfg.steps_per_task)
        self._manager_llm = manager_llm or llm
        self.manager_agent = manager_agent
        self.memory = Memory() if (memory and cfg.memory_enabled) else None
        self.prompts = PromptManager("orchestrator")
        self.task_callback = task_callback
        self.step_callback = step_callback
        self.agents: Dict[str, BaseAgent] = {}
        self._started = False
        self._idle: Deque[str] = deque()
        self._inflight: Dict[str, int] = {}  # tasks running per agent (capacity accounting)
        self.agent_rank: Optional[Callable[[Any], int]] = None  # node-wide pool: agent -> rank
        self.node = None  # parallel.node_plane.NodeManager when the pool spans ranks
        for a in agents or []:
            self._register_agent(a)
        self.tasks: Dict[str, Task] = {}
        self.completed_tasks: Dict[str, TaskResult] = {}
        self.failed_tasks: Dict[str, TaskResult] = {}
        self.running_tasks: Dict[str, str] = {}  # task id -> agent id
        self._futures: Dict[str, asyncio.Future] = {}
        self._queue: Optional[asyncio.PriorityQueue] = None
        self._seq = itertools.count()
        self._agent_cv: Optional[asyncio.Condition] = None
        self._waiting_on: Dict[str, List[Task]] = defaultdict(list)
        self._workers: List[asyncio.Task] = []
        self._active = 0  # tasks executing (worker loop + caller-runs path)
        self._cleanup_task: Optional[asyncio.Task] = None
        self._services: List[Any] = []
        self._shutting_down = False
        self.router = TaskRouter(self) if cfg.routing == "scored" else None
        self.metrics: Dict[str, int] = defaultdict(int)
        self.latency = _LatencyStats(cfg.latency_window)
        self.last_cleanup = datetime.now()
        self.logger = logging.getLogger(f"pilottai_amd.serve.{cfg.name}")
        self.logger.setLevel(logging.DEBUG if cfg.verbose else logging.INFO)

    # ------------------------------------------------------------------ protocol
    @property
    def child_agents(self) -> Dict[str, BaseAgent]:
        return self.agents

    @property
    def verbose(self) -> bool:
        return self.config.verbose

    @property
    def manager_llm(self):
        if self._manager_llm is None and self.manager_agent is None:
            self._manager_llm = _resolve_default_llm()
        return self._manager_llm

    def _register_agent(self, agent: BaseAgent):
        # a Serve-level control policy applies to agents that did not pick one
        if self.config.policy != "model" and getattr(agent, "policy", None) is DEFAULT_POLICY:
            agent.policy = self.policy
        self.agents[agent.id] = agent
        if step := self.step_callback:
            if getattr(agent, "step_callback", None) is None:
                agent.step_callback = step
        if self._started and self._is_available(agent):
            self._idle.append(agent.id)

    async def add_agent(self, agent: Union[BaseAgent, str], config: Optional[Union[AgentConfig, dict]] = None,
                        llm_config: Optional[Union[LLMConfig, dict]] = None, **kwargs) -> BaseAgent:
        """Documented API: add an agent instance or create one through AgentFactory."""
        if isinstance(agent, str):
            if agent not in AgentFactory._agent_types:
                AgentFactory.register_agent_type(agent, BaseAgent)
            if llm_config is not None:
                kwargs["llm_config"] = llm_config if isinstance(llm_config, LLMConfig) else LLMConfig(**llm_config)
            agent = await AgentFactory.create_agent(agent, config, **kwargs)
        elif self._started and str(getattr(agent, "status", "")) == "stopped":
            await agent.start()
        if getattr(agent, "policy", None) is not None and self.config.policy != "model":
            agent.policy = self.policy  # agents created for this Serve follow its policy
        self._register_agent(agent)
        await self._notify_agents()
        return agent

    async def remove_agent(self, agent_id: str) -> Optional[BaseAgent]:
        a = self.agents.pop(agent_id, None)
        try:
            self._idle.remove(agent_id)
        except ValueError:
            pass
        return a

    # orchestrator protocol used by DynamicScaling / FaultTolerance
    async def create_agent(self, **kw) -> BaseAgent:
        node = getattr(self, "node", None)
        if node is not None:  # node-wide pool: the new worker goes to the least-loaded rank
            remote = await node.create_agent(**kw)
            if remote is not None:
                return remote
        template = next((a for a in self.agents.values() if isinstance(a, BaseAgent)), None)
        role = kw.get("role") or (template.config.role if template else "worker")
        agent_type = kw.get("agent_type")
        if agent_type and agent_type in AgentFactory._agent_types:
            return await AgentFactory.create_agent(agent_type, template.config if template else None)
        cfg = template.config.model_copy(update={"role": role}) if template else AgentConfig(role=role, goal="work")
        cls = type(template) if template else BaseAgent
        agent = cls(cfg, llm=getattr(template, "_llm", None),
                    tools=list(getattr(template, "tools", {}).values()) if template else None,
                    policy=getattr(template, "policy", None))
        await agent.start()
        return agent

    async def add_child_agent(self, agent: BaseAgent):
        await self.add_agent(agent)

    async def remove_child_agent(self, agent_id: str):
        await self.remove_agent(agent_id)

    # ------------------------------------------------------------------ lifecycle
    async def start(self):
        if self._started:
            return
        self._shutting_down = False
        self._queue = asyncio.PriorityQueue(maxsize=self.config.max_queue_size)
        self._agent_cv = asyncio.Condition()
        for a in list(self.agents.values()):
            try:
                if str(getattr(a, "status", "stopped")) == "stopped":
                    await a.start()
            except Exception as e:  # noqa: BLE001
                self.logger.error("failed to start agent %s: %s", a.id, e)
        self._idle = deque(aid for aid, a in self.agents.items() if self._is_available(a))
        self._workers = [asyncio.create_task(self._worker(i)) for i in range(self.config.max_concurrent_tasks)]
        self._cleanup_task = asyncio.create_task(self._cleanup_loop())
        self._started = True
        await self._start_services()

    async def _start_services(self):
        c = self.config
        if c.enable_load_balancer:
            from .orchestration.load_balancer import LoadBalancer

            self._services.append(LoadBalancer(self, c.load_balancer))
        if c.enable_scaling:
            from .orchestration.scaling import DynamicScaling

            self._services.append(DynamicScaling(self, c.scaling))
        if c.enable_fault_tolerance:
            from .orchestration.fault_tolerance import FaultTolerance

            ft = FaultTolerance(self, c.fault_tolerance)
            self._services.append(ft)
        for s in self._services:
            await s.start()
            if hasattr(s, "register_agent"):
                for a in self.agents.values():
                    await s.register_agent(a)

    async def stop(self):
        self._shutting_down = True
        for s in self._services:
            try:
                await s.stop()
            except Exception as e:  # noqa: BLE001
                self.logger.error("service stop failed: %s", e)
        self._services.clear()
        for w in self._workers:
            w.cancel()
        for w in self._workers:
            try:
                await w
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
        self._workers.clear()
        if self._cleanup_task:
            self._cleanup_task.cancel()
            try:
                await self._cleanup_task
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
        for a in list(self.agents.values()):
            try:
                await a.stop()
            except Exception as e:  # noqa: BLE001
                self.logger.error("error stopping agent %s: %s", getattr(a, "id", "?"), e)
        for tid, fut in list(self._futures.items()):
            if not fut.done():
                fut.set_result(TaskResult(success=False, error="orchestrator stopped"))
        await self._cleanup_resources()
        self._started = False

    async def __aenter__(self):
        await self.start()
        return self

    async def __aexit__(self, *exc):
        await self.stop()

    # ------------------------------------------------------------------ submit
    async def add_task(self, task: Union[Task, Dict[str, Any], str]) -> str:
        return await self._submit(task, inline=False)

    async def _submit(self, task: Union[Task, Dict[str, Any], str], inline: bool) -> str:
        if self._shutting_down:
            raise RuntimeError("Orchestrator is shutting down")
        if not self._started:
            await self.start()
        task = Task.from_any(task)
        self.tasks[task.id] = task
        self._futures.setdefault(task.id, asyncio.get_running_loop().create_future())
        task.metadata.setdefault("_t_submit", time.perf_counter())
        spec = await self._speculative_agent(task) if inline else None
        tok = TASK_AGENT.set(spec.id if spec is not None else None)
        try:
            analysis = await self._analyze_task(task) if self.config.analyze_tasks else {}
        except BaseException:
            await self._drop_speculation(task, spec)
            raise
        finally:
            TASK_AGENT.reset(tok)
        if analysis.get("requires_decomposition", False):
            await self._drop_speculation(task, spec)
            spec = None
            subtasks = await self._decompose_task(task)
            if len(subtasks) > 1 or (subtasks and subtasks[0].id != task.id):
                task.update_status(TaskStatus.DELEGATED)
                for st in subtasks:
                    task.add_subtask(st)
                    self.tasks[st.id] = st
                    self._futures.setdefault(st.id, asyncio.get_running_loop().create_future())
                    st.metadata.setdefault("_t_submit", time.perf_counter())
                self.metrics["decomposed_tasks"] += 1
                for st in subtasks:
                    await self._enqueue(st)
                return task.id
        if inline:
            # yield the loop once per task before running it in the caller's coroutine: when the
            # LLM and tool calls complete without suspending, a caller-runs client would
            # otherwise run its whole batch before any other client, heartbeat or plane RPC got
            # a turn (the reference's single queue consumer interleaves clients,
            # pilott/pilott.py:272-303); the slot test below then sees the state after the yield
            await asyncio.sleep(0)
        if inline and self._queue.empty() and self._active < self.config.max_concurrent_tasks \
                and not any(d in self.tasks and d not in self.completed_tasks for d in task.dependencies):
            # caller-runs: a free concurrency slot and nothing queued ahead — run the
            # task in the caller's coroutine (no queue hop, no worker wake-up); the
            # slot accounting, timeout, evaluation and callbacks are the worker's
            self._active += 1
            try:
                await self._run(task, agent=spec)
            except Exception as e:  # noqa: BLE001 — as the worker loop
                self._finish(task, TaskResult(success=False, error=str(e)))
            finally:
                self._active -= 1
            return task.id
        await self._drop_speculation(task, spec)
        await self._enqueue(task)
        return task.id

    async def _speculative_agent(self, task: Task) -> Optional[BaseAgent]:
        """Reserve an idle agent and start the task's opening agent calls now, so they
        overlap the orchestrator's own analysis call (which only decides whether to
        decompose: the reference, pilott/pilott.py:184-231, runs the two back to
        back). Only where the caller-runs path will take the task and the plain
        first-idle pick applies (no manager agent, no scored router)."""
        if not (self.config.speculative_start and self.config.analyze_tasks) or self.manager_agent is not None \
                or self.router is not None or _is_workflow_task(task):
            return None
        if not self._queue.empty() or self._active >= self.config.max_concurrent_tasks or \
                any(d in self.tasks and d not in self.completed_tasks for d in task.dependencies):
            return None
        async with self._agent_cv:
            agent = self._pick_idle(task, None)
            if agent is None:
                return None
            n = self._inflight.get(agent.id, 0) + 1
            self._inflight[agent.id] = n
            if n >= self._capacity(agent):
                agent.status = AgentStatus.BUSY
        prefetch = getattr(agent, "prefetch_opening", None)
        if prefetch is not None:
            prefetch(task)
        return agent

    async def _drop_speculation(self, task: Task, agent: Optional[BaseAgent]):
        if agent is None:
            return
        drop = getattr(agent, "drop_opening", None)
        if drop is not None:
            drop(task.id)
        await self._release_agent(agent)

    async def execute_task(self, task: Union[Task, Dict[str, Any], str], timeout: Optional[float] = None) -> TaskResult:
        """Documented API: submit and wait for the TaskResult."""
        tid = await self._submit(task, inline=timeout is None)
        return await self.wait_for(tid, timeout)

    async def wait_for(self, task_id: str, timeout: Optional[float] = None) -> TaskResult:
        fut = self._futures.get(task_id)
        if fut is None:
            r = await self.get_result(task_id)
            if r is None:
                raise KeyError(task_id)
            return r
        if timeout is None:
            return await asyncio.shield(fut)
        return await asyncio.wait_for(asyncio.shield(fut), timeout)

    async def _enqueue(self, task: Task):
        unmet = [d for d in task.dependencies if d in self.tasks and d not in self.completed_tasks]
        if unmet:
            for d in unmet:
                self._waiting_on[d].append(task)
            return
        item = (-task.priority.rank, next(self._seq), task)
        if self._queue.full():
            await self._handle_queue_overflow(task, item)
            return
        self._queue.put_nowait(item)

    async def _handle_queue_overflow(self, task: Task, item):
        """Evict the lowest-priority queued task if the newcomer outranks it."""
        q = self._queue._queue  # heap of (-rank, seq, task)
        worst = max(q) if q else None
        if worst is not None and (-worst[0]) < task.priority.rank:
            q.remove(worst)
            import heapq

            heapq.heapify(q)
            victim = worst[2]
            self._finish(victim, TaskResult(success=False, error="Removed due to queue overflow"))
            self._queue.put_nowait(item)
            return
        self.tasks.pop(task.id, None)
        raise RuntimeError("Task queue is full")

    # ------------------------------------------------------------------ workers
    async def _worker(self, idx: int):
        while True:
            _, _, task = await self._queue.get()
            self._active += 1
            try:
                if task.id in self.tasks and task.status not in (TaskStatus.CANCELLED,):
                    await self._run(task)
            except asyncio.CancelledError:
                raise
            except Exception as e:  # noqa: BLE001 — never stall the queue (App. A #13)
                self.logger.error("task %s failed: %s", task.id, e)
                self._finish(task, TaskResult(success=False, error=str(e)))
            finally:
                self._active -= 1
                self._queue.task_done()

    async def _run(self, task: Task, agent: Optional[BaseAgent] = None):
        t_start = time.perf_counter()
        try:
            result = await with_timeout(self._execute_task(task, agent), self.config.task_timeout)
        except asyncio.TimeoutError:
            self.metrics["timeout_tasks"] += 1
            result = TaskResult(success=False, error="Task execution timed out",
                                execution_time=time.perf_counter() - t_start)
        self._finish(task, result)

    def _finish(self, task: Task, result: TaskResult):
        self.metrics["processed_tasks"] += 1
        if result.success:
            self.completed_tasks[task.id] = result
            self.metrics["successful_tasks"] += 1
            task.status = TaskStatus.COMPLETED
        else:
            self.failed_tasks[task.id] = result
            self.metrics["failed_tasks"] += 1
            task.status = TaskStatus.FAILED
        task.result = result
        task.completed_at = datetime.now()
        t0 = task.metadata.get("_t_submit")
        if t0 is not None:
            self.latency.add(time.perf_counter() - t0)
        fut = self._futures.pop(task.id, None)
        if fut is not None and not fut.done():
            fut.set_result(result)
        for dep in self._waiting_on.pop(task.id, []):
            if result.success:
                asyncio.ensure_future(self._enqueue(dep))
            else:
                self._finish(dep, TaskResult(success=False, error=f"dependency {task.id} failed"))
        if task.parent_task_id:
            self._maybe_finish_parent(task.parent_task_id)

    def _maybe_finish_parent(self, pid: str):
        parent = self.tasks.get(pid)
        if parent is None or pid in self.completed_tasks or pid in self.failed_tasks:
            return
        results = []
        for sid in parent.subtasks:
            r = self.completed_tasks.get(sid) or self.failed_tasks.get(sid)
            if r is None:
                return
            results.append(r)
        ok = all(r.success for r in results)
        agg = TaskResult(success=ok, output=[r.output for r in results],
                         error=None if ok else "; ".join(r.error or "" for r in results if not r.success),
                         execution_time=sum(r.execution_time for r in results),
                         metadata={"subtasks": list(parent.subtasks)})
        self._finish(parent, agg)

    async def _run_on_agent(self, task: Task, agent: Optional[BaseAgent], prefer: Optional[str] = None) -> TaskResult:
        """Execute on `agent` (or a newly acquired one). If the agent is lost mid-task (its
        rank died: AgentLostError), the task did not complete there: re-queue it on another
        agent — not a retry, and each task still completes exactly once."""
        while True:
            if agent is None:
                agent = await self._acquire_agent(task, prefer=prefer)
            try:
                self.running_tasks[task.id] = agent.id
                task.metadata["_agent_id"] = agent.id
                return await agent.execute_task(task)
            except AgentLostError as e:
                self.metrics["requeued_tasks"] += 1
                self.logger.warning("task %s re-queued: %s", task.id, e)
            finally:
                self.running_tasks.pop(task.id, None)
                await self._release_agent(agent)
            agent, prefer = None, None

    async def _execute_task(self, task: Task, agent: Optional[BaseAgent] = None) -> TaskResult:
        """`agent`: already reserved (speculative start in _submit)."""
        task.mark_started() if task.status in (TaskStatus.PENDING, TaskStatus.RETRY) else None
        result = await self._run_on_agent(task, agent)
        tok = TASK_AGENT.set(task.metadata.get("_agent_id"))
        try:
            evaluation = await self._evaluate_result(task, result) if self.config.evaluate_results else \
                {"success": result.success, "requires_retry": not result.success}
        finally:
            TASK_AGENT.reset(tok)
        if not evaluation.get("success", result.success):
            if evaluation.get("requires_retry", False) and task.retry_count < max(1, self.config.max_retry_attempts):
                self.metrics["retried_tasks"] += 1
                task.retry_count += 1
                result = await self._retry_task(task, evaluation)
            elif result.success:
                result = result.model_copy(update={"success": False,
                                                   "error": evaluation.get("failure_reason", "rejected by evaluation")})
        if self.memory is not None:
            await self._update_memory(task, result)
        if self.task_callback:
            await self._execute_callback(self.task_callback, task=task, result=result, agent=agent)
        return result

    async def _retry_task(self, task: Task, evaluation: Dict[str, Any]) -> TaskResult:
        mods = evaluation.get("task_modifications") or {}
        if isinstance(mods, dict) and mods:
            for k, v in mods.items():
                if k in ("description", "priority", "tools", "config", "metadata"):
                    setattr(task, k, v)
        return await self._run_on_agent(task, None, prefer=evaluation.get("agent"))

    # ------------------------------------------------------------------ agents
    def _is_available(self, a: BaseAgent) -> bool:
        st = str(getattr(a, "status", "idle"))
        return st == "idle" and getattr(a, "accepting_tasks", True)

    @staticmethod
    def _capacity(a: BaseAgent) -> int:
        """Tasks an agent may run at once: 1 (the reference's busy/idle model) unless
        the agent declares `concurrent_safe` (e.g. a delegating workflow manager,
        whose work happens in its children), then its config.max_concurrent_tasks."""
        if getattr(a, "concurrent_safe", False):
            return max(1, int(getattr(getattr(a, "config", None), "max_concurrent_tasks", 1)))
        return 1

    async def _notify_agents(self):
        if self._agent_cv is not None:
            async with self._agent_cv:
                self._agent_cv.notify_all()

    async def _acquire_agent(self, task: Task, prefer: Optional[str] = None) -> BaseAgent:
        if self.manager_agent is not None:
            a = await self.manager_agent.select_agent(task)
            if a is not None:
                return a
        deadline = time.monotonic() + self.config.agent_wait_timeout
        async with self._agent_cv:
            while True:
                agent = self._pick_idle(task, prefer)
                if agent is not None:
                    n = self._inflight.get(agent.id, 0) + 1
                    self._inflight[agent.id] = n
                    if n >= self._capacity(agent):
                        agent.status = AgentStatus.BUSY  # reserved atomically (App. A #12)
                    return agent
                left = deadline - time.monotonic()
                if left <= 0:
                    raise RuntimeError("No suitable agent found for task")
                try:
                    await asyncio.wait_for(self._agent_cv.wait(), timeout=left)
                except asyncio.TimeoutError:
                    pass

    def _pick_idle(self, task: Task, prefer: Optional[str]) -> Optional[BaseAgent]:
        if prefer:
            for aid in list(self._idle):
                a = self.agents.get(aid)
                if a is not None and (aid == prefer or a.config.role == prefer):
                    self._idle.remove(aid)
                    return a
        if self.agent_rank is not None:
            return self._pick_idle_balanced()
        n = len(self._idle)
        for _ in range(n):
            aid = self._idle.popleft()
            a = self.agents.get(aid)
            if a is None:
                continue
            if self._is_available(a):
                if self._inflight.get(aid, 0) + 1 < self._capacity(a):
                    self._idle.append(aid)  # still has free capacity: stays schedulable
                return a
            if str(a.status) not in ("stopped", "error"):
                self._idle.append(aid)  # paused (LoadBalancer): keep it, skip it
        return None

    def _pick_idle_balanced(self) -> Optional[BaseAgent]:
        """Node-wide pool (parallel/node_plane.py): the available agent on the rank with
        the fewest tasks in flight, so work spreads evenly over the GPUs whatever the
        submission pattern."""
        per_rank: Dict[int, int] = defaultdict(int)
        for aid in self.running_tasks.values():
            a = self.agents.get(aid)
            if a is not None:
                per_rank[self.agent_rank(a)] += 1
        for aid, n in self._inflight.items():  # reserved but not yet running
            a = self.agents.get(aid)
            if a is not None and aid not in self.running_tasks.values():
                per_rank[self.agent_rank(a)] += n
        best, best_key = None, None
        for aid in list(self._idle):
            a = self.agents.get(aid)
            if a is None or not self._is_available(a) or self._inflight.get(aid, 0) >= self._capacity(a):
                continue
            key = (per_rank[self.agent_rank(a)], self.agent_rank(a))
            if best_key is None or key < best_key:
                best, best_key = a, key
        if best is not None and self._inflight.get(best.id, 0) + 1 >= self._capacity(best):
            self._idle.remove(best.id)
        return best

    async def _release_agent(self, agent: BaseAgent):
        n = self._inflight.get(agent.id, 1) - 1
        if n > 0:
            self._inflight[agent.id] = n
        else:
            self._inflight.pop(agent.id, None)
        if agent.id in self.agents:
            if str(agent.status) == "busy" and getattr(agent, "accepting_tasks", True) and not agent.active_tasks:
                agent.status = AgentStatus.IDLE
            if agent.id not in self._idle:
                self._idle.append(agent.id)
        async with self._agent_cv:
            self._agent_cv.notify()

    # ------------------------------------------------------------------ LLM steps
    async def _llm_json(self, kind: str, fixed: Dict[str, Any], **kw) -> Dict[str, Any]:
        prompt = self.prompts.format_prompt(kind, **kw)
        rf = {"schema": f"orchestrator.{kind}", "fixed": fixed}
        llm = self.manager_llm
        try:
            resp = await llm.apredict(prompt, response_format=rf)
        except TypeError:
            resp = await llm.apredict(prompt)
        return parse_json_response(_content(resp) if isinstance(resp, dict) else resp)

    async def _analyze_task(self, task: Task) -> Dict[str, Any]:
        if self.manager_agent is not None and hasattr(self.manager_agent, "analyze_task"):
            return await self.manager_agent.analyze_task(task)
        try:
            res = await self._llm_json("task_analysis", self.policy.orchestrator_analysis(task.metadata),
                                       task_description=task.description)
        except Exception as e:  # noqa: BLE001
            self.logger.warning("task analysis failed (%s); executing without decomposition", e)
            return {"requires_decomposition": False}
        for k, typ in (("requires_decomposition", bool), ("complexity", str), ("estimated_resources", dict)):
            if k in res and not isinstance(res[k], typ):
                raise ValueError(f"Field {k} should be of type {typ.__name__}")
        return res

    async def _decompose_task(self, task: Task) -> List[Task]:
        try:
            res = await self._llm_json("task_decomposition", {}, task_description=task.description)
            subs = []
            for i, sd in enumerate(res.get("subtasks") or []):
                desc = str(sd.get("description") or "").strip() or f"{task.description} (part {i + 1})"
                subs.append(Task(description=desc, priority=sd.get("priority", task.priority),
                                 parent_task_id=task.id, metadata={k: v for k, v in task.metadata.items()
                                                                   if not k.startswith("_")}))
            return subs or [task]
        except Exception as e:  # noqa: BLE001
            self.logger.error("decomposition failed: %s", e)
            return [task]

    async def _evaluate_result(self, task: Task, result: TaskResult) -> Dict[str, Any]:
        if self.manager_agent is not None:
            return await self.manager_agent.evaluate_result(task, result)
        try:
            return await self._llm_json(
                "result_evaluation", self.policy.orchestrator_evaluation(result.success),
                task_description=task.description,
                result=json.dumps({"success": result.success, "output": str(result.output)[:500],
                                   "error": result.error, "execution_time": result.execution_time}))
        except Exception as e:  # noqa: BLE001
            self.logger.warning("result evaluation failed: %s", e)
            return {"success": result.success, "requires_retry": False}

    async def _update_memory(self, task: Task, result: TaskResult):
        try:
            self.memory.store_nowait({"type": "task_execution", "task_id": task.id, "description": task.description,
                                      "result": result.model_dump(mode="json"),
                                      "timestamp": datetime.now().isoformat()}, tags=["task_execution"])
        except Exception as e:  # noqa: BLE001
            self.logger.error("memory update failed: %s", e)

    async def _execute_callback(self, cb: Callable, **kw):
        try:
            if asyncio.iscoroutinefunction(cb):
                await cb(**kw)
            else:
                await asyncio.to_thread(cb, **kw)
        except Exception as e:  # noqa: BLE001
            self.logger.error("callback failed: %s", e)

    # ------------------------------------------------------------------ housekeeping
    async def _cleanup_loop(self):
        while True:
            await asyncio.sleep(self.config.cleanup_interval)
            await self._cleanup_resources()

    async def _cleanup_resources(self):
        now = datetime.now()
        keep = timedelta(seconds=self.config.task_retention_period)
        for d in (self.completed_tasks, self.failed_tasks):
            for tid in [t for t, r in d.items() if now - r.completion_time > keep]:
                d.pop(tid, None)
                self.tasks.pop(tid, None)
        self.last_cleanup = now

    async def get_result(self, task_id: str) -> Optional[TaskResult]:
        return self.completed_tasks.get(task_id) or self.failed_tasks.get(task_id)

    async def broadcast_context(self, text: Optional[str] = None, src: int = 0) -> Dict[str, Any]:
        """Shared-context broadcast. Collective over the world group:
        every rank calls it; rank `src` supplies `text`. The text travels as token
        ids (RCCL over xGMI), each rank's engines pre-compute its KV into their
        prefix caches, and every LLM of this Serve puts it at the front of its
        prompts, so all later agent calls on every GPU reuse those blocks."""
        from .engine.local_llm import encode_chat
        from .engine.tokenizer import get_tokenizer
        from .parallel import comm

        llms = [self.manager_llm] + [vars(a).get("_llm") for a in self.agents.values()]
        llms = list({id(x): x for x in llms if x is not None}.values())
        engines = list({id(e): e for e in (getattr(x, "engine", None) for x in llms) if e is not None}.values())
        tok = engines[0].tok if engines else get_tokenizer()
        rank = comm.env_rank_world()[0] if comm.dist.is_initialized() else 0
        ids = comm.broadcast_tokens(tok.encode(text or "") if rank == src else None, src=src)
        ctx = tok.decode(ids)
        for x in llms:
            if hasattr(x, "shared_context"):
                x.shared_context = ctx or None
        prewarmed = 0
        if ctx:
            msg = encode_chat(tok, [{"role": "system", "content": ctx}])
            for e in engines:
                await asyncio.to_thread(e.prewarm, msg)
                prewarmed += 1
        self.shared_context = ctx
        return {"tokens": len(ids), "prewarmed_engines": prewarmed}

    def get_metrics(self) -> Dict[str, Any]:
        m = {
            "name": self.config.name,
            "active_agents": sum(1 for a in self.agents.values() if str(a.status) != "stopped"),
            "idle_agents": len(self._idle),
            "queue_size": self._queue.qsize() if self._queue else 0,
            "running_tasks": len(self.running_tasks),
            "completed_tasks": len(self.completed_tasks),
            "failed_tasks": len(self.failed_tasks),
            "metrics": dict(self.metrics),
            "latency_p50_s": self.latency.pct(50),
            "latency_p99_s": self.latency.pct(99),
            "last_cleanup": self.last_cleanup.isoformat(),
        }
        llm = self._manager_llm
        eng = getattr(llm, "engine", None)
        if eng is not None:
            m["engine"] = eng.metrics()
        return m

    # ------------------------------------------------------------------ checkpoint
    def checkpoint(self, path) -> str:
        from .utils.checkpoint import save_serve_checkpoint

        return save_serve_checkpoint(self, path)

    async def restore(self, path, requeue: bool = True) -> int:
        from .utils.checkpoint import restore_serve_checkpoint

        return await restore_serve_checkpoint(self, path, requeue=requeue)

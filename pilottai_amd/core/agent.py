"""LLM-driven agent (reference: pilott/core/agent.py:59-627).

Per task: validate -> task analysis (LLM) -> tool selection (LLM) -> ordered
tool-lock acquisition -> step loop (LLM plans the next step, the tool or the
function-calling LLM executes it; at most `max_iter` steps) -> self-evaluation
(LLM) -> TaskResult. Every LLM call carries its reply schema
(`response_format`), so a local engine constrains decoding and every reply parses.

Fixes relative to the reference: prompts format (#1/#2), the LLM
reply is read as a string or a dict (#3), the step schema is
{"task_complete", "next_step": {"tool", "inputs", ...}} (#4), tools are a
name->Tool mapping (#5), timeouts use asyncio.wait_for (#6), the step counter is
per task (#7), suitability reads the merged AgentConfig (#8), `child_agents`
exists (#9), `send_heartbeat` exists (#30). Both constructor styles work:
`BaseAgent(role=..., goal=..., llm=...)` and the documented
`BaseAgent(agent_config, llm_config)` (docs example).
"""
from __future__ import annotations

import asyncio
import json
import logging
import time
import uuid
from collections import deque
from datetime import datetime
from typing import Any, Callable, Deque, Dict, List, Optional, Sequence, Union

import psutil

_PROC = psutil.Process()
_NCPU = max(1, len(_PROC.cpu_affinity()) if hasattr(_PROC, "cpu_affinity") else (psutil.cpu_count() or 1))
_CPU_SAMPLE = [0.0, 0.0]  # [monotonic time, value]


def _process_cpu_share() -> float:
    """This process's CPU share in [0, 1], sampled at most every 0.5 s (psutil's
    interval-free reading is garbage when calls are microseconds apart, which is
    exactly what many agents reporting metrics back to back produce)."""
    now = time.monotonic()
    if now - _CPU_SAMPLE[0] >= 0.5:
        _CPU_SAMPLE[1] = min(1.0, max(0.0, _PROC.cpu_percent(interval=None) / (100.0 * _NCPU)))
        _CPU_SAMPLE[0] = now
    return _CPU_SAMPLE[1]

from .config import AgentConfig, LLMConfig
from .policy import DEFAULT_POLICY, ControlPolicy
from .prompts import PromptManager, parse_json_response
from .role import AgentRole, AgentStatus
from .task import Task, TaskResult, TaskStatus
from ..utils.timeouts import with_timeout

_DEFAULT_LLM: Dict[str, Any] = {"llm": None, "factory": None}


def set_default_llm(llm: Any = None, factory: Optional[Callable[[], Any]] = None):
    """Process-wide LLM used by agents created without one (e.g. by AgentFactory)."""
    _DEFAULT_LLM["llm"] = llm
    _DEFAULT_LLM["factory"] = factory


def _resolve_default_llm():
    if _DEFAULT_LLM["llm"] is None:
        if _DEFAULT_LLM["factory"] is not None:
            _DEFAULT_LLM["llm"] = _DEFAULT_LLM["factory"]()
        else:
            from pilottai_amd.engine.local_llm import make_llm

            _DEFAULT_LLM["llm"] = make_llm(LLMConfig())
    return _DEFAULT_LLM["llm"]


def _content(resp: Any) -> str:
    if isinstance(resp, dict):
        return resp.get("content") or ""
    return "" if resp is None else str(resp)


def _short(x: Any, n: int = 400) -> Any:
    s = json.dumps(x, default=str)
    return x if len(s) <= n else s[:n] + "..."


def _is_workflow(task: Task) -> bool:
    return (task.type or task.metadata.get("type")) == "complex_workflow" and bool(task.metadata.get("steps"))


class BaseAgent:
    TASK_TIMEOUT = 300.0
    MAX_HISTORY_SIZE = 100

    def __init__(self, role: Union[str, AgentConfig, None] = None, goal: Optional[Union[str, LLMConfig, dict]] = None,
                 backstory: Optional[str] = None, knowledge: Optional[List[str]] = None,
                 config: Optional[Union[Dict[str, Any], AgentConfig]] = None, llm: Any = None,
                 function_calling_llm: Any = None, max_iter: Optional[int] = None, verbose: bool = False,
                 allow_delegation: Optional[bool] = None, tools: Optional[Sequence[Any]] = None,
                 step_callback: Optional[Callable] = None, *, agent_config: Optional[AgentConfig] = None,
                 llm_config: Optional[Union[LLMConfig, dict]] = None, policy: Optional[ControlPolicy] = None,
                 memory: Any = None, memory_lookup: Any = None, memory_top_k: int = 3):
        # --- accept BaseAgent(agent_config, llm_config) and factory-style cls(config)
        if isinstance(role, AgentConfig):
            agent_config, role = role, None
        if isinstance(config, AgentConfig):
            agent_config, config = config, None
        if isinstance(goal, (LLMConfig, dict)) and agent_config is not None:
            llm_config, goal = goal, None
        if agent_config is None:
            if not role:
                raise ValueError("Agent role is required")
            agent_config = AgentConfig(role=role, goal=goal or f"Complete tasks as {role}", backstory=backstory,
                                       knowledge=knowledge or [], max_iterations=max_iter or 10,
                                       verbose=verbose, can_delegate=bool(allow_delegation),
                                       additional_config=dict(config or {}))
        else:
            upd = {}
            if max_iter:
                upd["max_iter"] = max_iter
            if allow_delegation is not None:
                upd["allow_delegation"] = allow_delegation
            if upd:
                agent_config = agent_config.model_copy(update=upd)
                agent_config._sync_aliases()
        self.config: AgentConfig = agent_config
        self.agent_config = agent_config  # documented alias (docs example)
        self.id = str(uuid.uuid4())
        self._llm = llm
        self._llm_config = LLMConfig(**llm_config) if isinstance(llm_config, dict) else llm_config
        self.function_calling_llm = function_calling_llm
        self.tools: Dict[str, Any] = {}
        for t in tools or []:
            self.add_tool(t)
        self.policy = policy or DEFAULT_POLICY
        self.prompts = PromptManager("agent")
        self.step_callback = step_callback
        self.status = AgentStatus.STOPPED
        self.current_task: Optional[Task] = None
        self.iteration_count = 0
        self.conversation_history: Deque[Dict[str, str]] = deque(maxlen=self.MAX_HISTORY_SIZE)
        self.execution_locks: Dict[str, asyncio.Lock] = {}
        self._openings: Dict[str, "asyncio.Future"] = {}  # prefetched opening calls by task id
        self._first_lookups: Dict[str, "asyncio.Future"] = {}  # step 0's memory lookup, by task id
        self._tool_locks: Dict[str, asyncio.Lock] = {}
        self.tasks: Dict[str, Task] = {}
        self.active_tasks: set = set()
        self.task_history: Deque[Dict[str, Any]] = deque(maxlen=1000)
        self.task_metrics: Dict[str, int] = {"completed": 0, "failed": 0, "timeout": 0}
        self.metrics = self.task_metrics  # documented alias `agent.metrics[...]`
        self.memory_errors: Dict[str, int] = {"store": 0, "search": 0}  # failed memory calls
        self.child_agents: Dict[str, "BaseAgent"] = {}
        self.parent: Optional["BaseAgent"] = None
        self._memory = memory
        # per-step semantic memory (memory/batcher.py MemoryLookupBatcher, shared by the
        # agents of a Serve): every step-planning call carries the top-k hits for the
        # task + last result, and each finished task is written back
        self.memory_lookup = memory_lookup
        self.memory_top_k = int(memory_top_k)
        self.last_error: Optional[str] = None
        self.last_heartbeat = datetime.now()
        self._accepting = True
        self.llm_usage = {"calls": 0, "prompt_tokens": 0, "completion_tokens": 0}
        self.logger = logging.getLogger(f"pilottai_amd.agent.{self.config.role}")
        self.logger.setLevel(logging.DEBUG if self.config.verbose else logging.INFO)

    # ------------------------------------------------------------------ properties
    @property
    def llm(self):
        if self._llm is None:
            if self._llm_config is not None:
                from pilottai_amd.engine.local_llm import make_llm

                self._llm = make_llm(self._llm_config)
            else:
                self._llm = _resolve_default_llm()
        return self._llm

    @llm.setter
    def llm(self, v):
        self._llm = v

    @property
    def role(self) -> str:
        return self.config.role

    @property
    def specializations(self) -> List[str]:
        return list(self.config.specializations)

    @property
    def max_concurrent_tasks(self) -> int:
        return self.config.max_concurrent_tasks

    @property
    def enhanced_memory(self):
        """Per-agent semantic memory (documented API: agent.enhanced_memory.store_semantic)."""
        if self._memory is None:
            from pilottai_amd.memory.enhanced_memory import EnhancedMemory

            self._memory = EnhancedMemory()
        return self._memory

    def add_tool(self, tool: Any):
        from pilottai_amd.tools.tool import Tool

        if isinstance(tool, Tool):
            self.tools[tool.name] = tool
        elif callable(tool):
            t = Tool.from_callable(tool)
            self.tools[t.name] = t
        elif isinstance(tool, str):
            self.tools[tool] = None  # name-only placeholder: an LLM-only step
        else:
            raise TypeError(f"unsupported tool {tool!r}")

    # ------------------------------------------------------------------ lifecycle
    async def start(self):
        self.status = AgentStatus.IDLE
        self._accepting = True
        self.last_heartbeat = datetime.now()

    async def stop(self):
        self.status = AgentStatus.STOPPED
        for lock in list(self.execution_locks.values()):
            if lock.locked():
                try:
                    lock.release()
                except RuntimeError:
                    pass
        self.execution_locks.clear()
        self.conversation_history.clear()
        self.current_task = None
        self.iteration_count = 0

    async def reset(self):
        self.status = AgentStatus.IDLE
        self.current_task = None
        self.iteration_count = 0
        self.conversation_history.clear()
        self._tool_locks.clear()
        self.tasks.clear()
        self.active_tasks.clear()
        self.task_metrics.update(completed=0, failed=0, timeout=0)
        self.last_error = None
        self._accepting = True

    async def cleanup_resources(self):
        for lock in self._tool_locks.values():
            if lock.locked():
                try:
                    lock.release()
                except RuntimeError:
                    pass
        self._tool_locks.clear()
        self.conversation_history.clear()
        if self._memory is not None and hasattr(self._memory, "stop"):
            await self._memory.stop()

    async def send_heartbeat(self) -> datetime:
        """Liveness probe used by FaultTolerance (missing in the reference, App. A #30)."""
        if self.status == AgentStatus.STOPPED:
            raise RuntimeError(f"agent {self.id} is stopped")
        self.last_heartbeat = datetime.now()
        return self.last_heartbeat

    # ------------------------------------------------------------------ task queue
    async def add_task(self, task: Union[Task, Dict[str, Any]]) -> str:
        t = Task.from_any(task)
        if t.id in self.tasks:
            raise ValueError(f"Task {t.id} already exists")
        if len(self.tasks) >= self.config.max_queue_size:
            raise RuntimeError("agent task queue is full")
        self.tasks[t.id] = t
        return t.id

    async def remove_task(self, task_id: str) -> Optional[Task]:
        if task_id in self.active_tasks:
            raise ValueError(f"Cannot remove active task {task_id}")
        return self.tasks.pop(task_id, None)

    async def wait_for_tasks(self, poll: float = 0.05, timeout: Optional[float] = None):
        t0 = time.monotonic()
        while self.active_tasks:
            if timeout is not None and time.monotonic() - t0 > timeout:
                raise asyncio.TimeoutError("tasks still active")
            await asyncio.sleep(poll)

    async def pause_task_acceptance(self):
        self._accepting = False
        if self.status == AgentStatus.IDLE:
            self.status = AgentStatus.BUSY

    async def resume_task_acceptance(self):
        self._accepting = True
        if self.status == AgentStatus.BUSY and not self.active_tasks:
            self.status = AgentStatus.IDLE

    @property
    def accepting_tasks(self) -> bool:
        return self._accepting and self.status not in (AgentStatus.STOPPED, AgentStatus.ERROR)

    # ------------------------------------------------------------------ children
    async def add_child_agent(self, agent: "BaseAgent"):
        if len(self.child_agents) >= self.config.max_child_agents:
            raise RuntimeError("max_child_agents reached")
        agent.parent = self
        self.child_agents[agent.id] = agent
        if agent.status == AgentStatus.STOPPED:
            await agent.start()

    async def remove_child_agent(self, agent_id: str) -> Optional["BaseAgent"]:
        a = self.child_agents.pop(agent_id, None)
        if a is not None:
            a.parent = None
        return a

    async def create_agent(self, **kw) -> "BaseAgent":
        """Orchestrator-protocol hook (used by DynamicScaling on manager agents)."""
        role = kw.get("role") or f"{self.config.role}-child"
        cfg = AgentConfig(role=role, goal=kw.get("goal", self.config.goal), description=kw.get("description", ""),
                          role_type=AgentRole.WORKER)
        return type(self)(cfg, llm=self._llm, tools=list(self.tools.values()), policy=self.policy)

    # ------------------------------------------------------------------ execution
    async def execute_task(self, task: Union[Task, Dict[str, Any]]) -> TaskResult:
        task = Task.from_any(task)
        if task.id in self.active_tasks:
            raise ValueError(f"Task {task.id} is already being executed")
        self.status = AgentStatus.BUSY
        self.current_task = task
        self.active_tasks.add(task.id)
        self.tasks.setdefault(task.id, task)
        t0 = time.perf_counter()
        timeout = task.timeout or float(self.config.task_timeout or self.TASK_TIMEOUT)
        lock = self.execution_locks.setdefault(task.id, asyncio.Lock())
        try:
            async with lock:
                try:
                    body = self._execute_workflow(task) if _is_workflow(task) else self._execute_task_internal(task)
                    result = await with_timeout(body, timeout)
                except asyncio.TimeoutError:
                    self.task_metrics["timeout"] += 1
                    self.task_metrics["failed"] += 1
                    self.last_error = "Task execution timed out"
                    task.update_status(TaskStatus.TIMEOUT)
                    return TaskResult(success=False, error="Task execution timed out",
                                      execution_time=time.perf_counter() - t0)
            if result.success:
                self.task_metrics["completed"] += 1
                task.update_status(TaskStatus.COMPLETED)
            else:
                self.task_metrics["failed"] += 1
                self.last_error = result.error
                task.update_status(TaskStatus.FAILED)
            task.result = result
            self.task_history.append({"task_id": task.id, "success": result.success,
                                      "execution_time": result.execution_time, "ts": datetime.now().isoformat()})
            return result
        finally:
            self.active_tasks.discard(task.id)
            self.tasks.pop(task.id, None)
            self.execution_locks.pop(task.id, None)
            self.current_task = None
            if self.status == AgentStatus.BUSY and not self.active_tasks:
                self.status = AgentStatus.IDLE if self._accepting else AgentStatus.BUSY
            self.last_heartbeat = datetime.now()

    async def _execute_workflow(self, task: Task) -> TaskResult:
        """Documented orchestration form (reference README.md:143-146):
        `execute_task({"type": "complex_workflow", "steps": ["extract", "analyze", ...]})`.
        Steps run in order; each goes to the child agent specialised in it (or the
        most suitable child), else this agent runs it; a step sees the previous
        step's output in its metadata. Output: {step: output}."""
        t0 = time.perf_counter()
        outputs: Dict[str, Any] = {}
        prev: Any = None
        for i, step in enumerate(task.metadata.get("steps") or []):
            name = step if isinstance(step, str) else str(step.get("type", f"step{i}"))
            sub = Task(description=f"{name}: {task.description}",
                       metadata={"type": name, "previous_output": prev, "workflow_id": task.id})
            child = self._child_for(name)
            res = await (child.execute_task(sub) if child is not None else self._execute_task_internal(sub))
            if not res.success:
                return TaskResult(success=False, output=outputs, error=f"step {name} failed: {res.error}",
                                  execution_time=time.perf_counter() - t0)
            outputs[name] = prev = res.output
        return TaskResult(success=True, output=outputs, execution_time=time.perf_counter() - t0)

    def _child_for(self, step: str) -> Optional["BaseAgent"]:
        live = [a for a in self.child_agents.values() if str(a.status) not in ("stopped", "error")]
        for a in live:
            if step in (a.config.specializations or []) or a.config.role == step:
                return a
        return None

    async def _execute_task_internal(self, task: Task) -> TaskResult:
        t0 = time.perf_counter()
        held: List[str] = []
        iterations = 0
        try:
            opening = self._openings.pop(task.id, None)
            first_lookup = self._first_lookups.pop(task.id, None)
            try:
                self._validate_task(task)
            except BaseException:
                for f in (opening, first_lookup):
                    if f is not None:
                        f.cancel()
                raise
            if first_lookup is None:
                first_lookup = self._start_first_lookup(task)
            if opening is None:
                opening = self.prefetch_opening(task, _store=False)
            analysis, selection = await opening
            if analysis.get("can_execute", True) is False:
                raise ValueError(f"Cannot execute task: {analysis.get('reason')}")
            chosen = [t for t in selection.get("selected_tools", []) if t in self.tools]
            for name in sorted(set(chosen)):  # fixed order -> no deadlock
                lock = self._tool_locks.setdefault(name, asyncio.Lock())
                await lock.acquire()
                held.append(name)
            steps, iterations = await self._execute_steps(task, chosen, first_lookup)
            first_lookup = None
            evaluation = await self._evaluate_result(task, steps)
            ok = bool(evaluation.get("success", False))
            await self._remember(task, ok, evaluation)
            return TaskResult(success=ok, output=steps, error=None if ok else evaluation.get("reasoning", "evaluation failed"),
                              execution_time=time.perf_counter() - t0,
                              metadata={"analysis": analysis, "tools_used": selection, "evaluation": evaluation,
                                        "iterations": iterations, "agent_id": self.id, "agent_role": self.config.role})
        except Exception as e:  # noqa: BLE001
            return TaskResult(success=False, output=None, error=str(e), execution_time=time.perf_counter() - t0,
                              metadata={"agent_id": self.id, "iterations": iterations})
        finally:
            if first_lookup is not None and not first_lookup.done():
                first_lookup.cancel()
            for name in reversed(sorted(held)):
                lock = self._tool_locks.get(name)
                if lock is not None and lock.locked():
                    lock.release()

    def prefetch_opening(self, task: Task, _store: bool = True) -> Optional["asyncio.Future"]:
        """Start a task's two opening LLM calls — task analysis and tool selection.

        They are independent (the reference's _select_tools, pilott/core/agent.py:
        259-268, does not read the analysis; it runs them back to back, :176-179),
        so both go into the continuous batch at once. Neither has side effects: the
        orchestrator may start them speculatively while it analyses the task itself
        (Serve._submit) and drop them (drop_opening) if it decomposes the task."""
        if _store and type(self)._execute_task_internal is not BaseAgent._execute_task_internal:
            # a subclass with its own execution path never consumes the opening: starting
            # it would spend two LLM calls per task (and resolve a default LLM) for nothing
            return None

        async def both():
            sel = asyncio.ensure_future(self._select_tools(task))
            try:
                ana = await self._analyze_task(task)
            except BaseException:
                sel.cancel()
                raise
            if ana.get("can_execute", True) is False:
                sel.cancel()
                return ana, {}
            return ana, await sel

        fut = asyncio.ensure_future(both())
        if _store:
            self._openings[task.id] = fut
            lk = self._start_first_lookup(task)
            if lk is not None:
                self._first_lookups[task.id] = lk
        return fut

    def drop_opening(self, task_id: str):
        for d in (self._openings, self._first_lookups):
            fut = d.pop(task_id, None)
            if fut is not None and not fut.done():
                fut.cancel()

    def _start_first_lookup(self, task: Task) -> Optional["asyncio.Future"]:
        """The first step plan's memory lookup depends only on the task (no step result
        yet), so it starts with the opening calls instead of after them: its batched index
        pass and query embedding overlap the analysis / tool-selection round trips rather
        than adding to the task's critical path. Later steps' lookups read the previous
        step's result and stay in the loop."""
        if self.memory_lookup is None or self.memory_top_k <= 0:
            return None
        return asyncio.ensure_future(self._memory_context(task, json.dumps(_short(None))))

    def _validate_task(self, task: Task):
        if not task.description:
            raise ValueError("Task must have a description")
        for dep in task.dependencies:
            d = self.tasks.get(dep)
            if d is not None and d.status != TaskStatus.COMPLETED:
                raise ValueError(f"Dependency {dep} not yet completed")
        if task.max_retries < 0:
            raise ValueError("Task max_retries must be a non-negative integer")
        if task.is_expired():
            raise ValueError("Task deadline has passed")

    # ------------------------------------------------------------------ LLM calls
    def _compose_messages(self, system: str, prompt: str) -> List[Dict[str, str]]:
        """Chat messages for one agent call.

        Against the on-node engine (LLMs with `prefix_cache_layout`), the task
        text goes FIRST and the agent's identity block after it: every call of a
        task — the orchestrator's and every agent's — then starts with the same
        "Task: ..." tokens, so its KV blocks are prefilled once per task and
        reused by the prefix cache (the reference sends system-then-user to a
        remote API, pilott/core/agent.py; same content, different order)."""
        if getattr(self.llm, "prefix_cache_layout", False) and prompt.startswith("Task:"):
            head, sep, tail = prompt.partition("\n\n")
            if sep:
                return [{"role": "user", "content": f"{head}\n\n{system.rstrip()}\n\n{tail}"}]
        return [{"role": "system", "content": system}, {"role": "user", "content": prompt}]

    async def _llm_json(self, kind: str, fixed: Optional[Dict[str, Any]] = None, schema: Optional[str] = None,
                        **kw) -> Dict[str, Any]:
        prompt = self.prompts.format_prompt(kind, **kw)
        system = self.prompts.format_prompt("system_base", role=self.config.role, goal=self.config.goal,
                                            backstory=self.config.backstory or "No specific backstory.")
        messages = self._compose_messages(system, prompt)
        rf = {"schema": f"agent.{schema or kind}", "fixed": fixed or {}}
        try:
            resp = await self.llm.generate_response(messages, response_format=rf)
        except TypeError:  # a third-party LLM without structured-output support
            resp = await self.llm.generate_response(messages)
        text = _content(resp)
        if not text and not isinstance(resp, dict):
            raise ValueError("Empty response from LLM")
        if isinstance(resp, dict) and "usage" in resp:
            u = resp["usage"]
            self.llm_usage["calls"] += 1
            self.llm_usage["prompt_tokens"] += u.get("prompt_tokens", 0)
            self.llm_usage["completion_tokens"] += u.get("completion_tokens", 0)
        self.conversation_history.extend(messages + [{"role": "assistant", "content": text}])
        return parse_json_response(resp if isinstance(resp, dict) and "content" not in resp else text)

    async def _analyze_task(self, task: Task) -> Dict[str, Any]:
        return await self._llm_json("task_analysis", self.policy.agent_analysis(), role=self.config.role,
                                    goal=self.config.goal, task_description=task.description)

    async def _select_tools(self, task: Task) -> Dict[str, Any]:
        names = [n for n in self.tools]
        return await self._llm_json("tool_selection", self.policy.tool_selection(names),
                                    tools=json.dumps(names), task_description=task.description)

    async def _execute_steps(self, task: Task, tools: List[str], first_lookup: Optional["asyncio.Future"] = None):
        completed: List[Dict[str, Any]] = []
        step_inputs = task.metadata.get("tool_inputs", {}) if isinstance(task.metadata, dict) else {}
        iterations = 0
        while iterations < self.config.max_iter:
            tool = tools[iterations % len(tools)] if tools else "none"
            fixed = self.policy.step_planning(iterations, tool)
            if self.policy.fixed_mode:
                fixed["next_step.inputs"] = step_inputs
            last = json.dumps(_short(completed[-1] if completed else None))
            common = dict(task_description=task.description, completed_steps=json.dumps(_short(completed, 800)),
                          available_tools=json.dumps(tools), last_result=last)
            if self.memory_lookup is not None and self.memory_top_k > 0:
                if iterations == 0 and first_lookup is not None:
                    ctx = await first_lookup  # started with the opening calls (same query)
                else:
                    ctx = await self._memory_context(task, last)
                plan = await self._llm_json("step_planning_memory", fixed, schema="step_planning",
                                            memory_context=ctx, **common)
            else:
                plan = await self._llm_json("step_planning", fixed, **common)
            if plan.get("task_complete", False):
                break
            step = plan.get("next_step") or {k: plan[k] for k in ("tool", "inputs") if k in plan}
            result = await self._execute_step(step)
            completed.append({"step": step, "result": result})
            iterations += 1
            self.iteration_count += 1
            if self.step_callback:
                await self._execute_callback(self.step_callback, step=step, result=result,
                                             context={"task": task.id, "completed_steps": completed})
        return completed, iterations

    async def _memory_context(self, task: Task, last_result: str) -> str:
        """Top-k memory hits for this step (one batched index pass per event-loop tick
        across all agents), as a short text block for the step-planning prompt."""
        query = f"{task.description[:400]} {last_result[:200]}"
        try:
            hits = await self.memory_lookup.search(query, limit=self.memory_top_k)
        except Exception as e:  # noqa: BLE001 — memory is advisory (reference: warn and go on)
            self.memory_errors["search"] += 1
            self.logger.warning("memory search failed: %s", e)
            return "none"
        return "; ".join(h.text[:160] for h in hits) or "none"

    async def _remember(self, task: Task, ok: bool, evaluation: Dict[str, Any]):
        if self.memory_lookup is None or self.memory_top_k <= 0:
            return
        try:
            await self.memory_lookup.store(
                f"{task.description[:300]} => {'done' if ok else 'failed'}: {str(evaluation.get('reasoning', ''))[:200]}",
                metadata={"task_id": task.id, "agent": self.id, "success": ok}, tags={self.config.role},
                priority=1 if ok else 0)
        except Exception as e:  # noqa: BLE001 -- advisory, but counted: get_metrics() reports it
            self.memory_errors["store"] += 1
            n = self.memory_errors["store"]
            (self.logger.error if n >= 3 else self.logger.warning)("memory store failed (%d so far): %s", n, e)

    async def _execute_step(self, step: Dict[str, Any]) -> Any:
        name = step.get("tool")
        inputs = step.get("inputs") or {}
        tool = self.tools.get(name)
        if tool is None:
            # no executable tool for this step: an LLM-only reasoning step
            return {"status": "llm_only", "output": step.get("expected_outcome")}
        if step.get("requires_llm") and self.function_calling_llm is not None:
            resp = await asyncio.wait_for(self.function_calling_llm.generate_response(
                messages=[{"role": "user", "content": json.dumps(step)}], tools=[tool.spec()]), 60)
            calls = (resp or {}).get("tool_calls") or []
            if calls:
                args = json.loads(calls[0]["function"].get("arguments") or "{}")
                inputs = {**inputs, **args}
        try:
            out = await asyncio.wait_for(tool.execute(**inputs), 30)
            return {"status": "success", "output": out}
        except asyncio.TimeoutError:
            raise TimeoutError(f"Step execution timed out for tool {name}")

    async def _evaluate_result(self, task: Task, steps: Any) -> Dict[str, Any]:
        return await self._llm_json("result_evaluation", self.policy.agent_evaluation(), role=self.config.role,
                                    goal=self.config.goal, task_description=task.description,
                                    result=json.dumps(_short(steps, 800)))

    async def _execute_callback(self, cb: Callable, **kw):
        try:
            if asyncio.iscoroutinefunction(cb):
                await cb(**kw)
            else:
                await asyncio.to_thread(cb, **kw)
        except Exception as e:  # noqa: BLE001
            self.logger.error("callback failed: %s", e)

    # ------------------------------------------------------------------ metrics
    async def get_metrics(self) -> Dict[str, Any]:
        done = self.task_metrics["completed"] + self.task_metrics["failed"]
        # this process's CPU share, not the whole machine's (the reference used
        # system-wide psutil, so load from unrelated processes marked agents busy)
        cpu = _process_cpu_share()
        mem = psutil.virtual_memory().percent / 100.0
        m = {
            "queue_size": len(self.tasks),
            "active_tasks": len(self.active_tasks),
            "success_rate": self.task_metrics["completed"] / done if done else 0.0,
            "queue_utilization": len(self.tasks) / self.config.max_queue_size,
            "cpu_usage": cpu,
            "memory_usage": mem,
            "total_tasks": done,
            "error_count": self.task_metrics["failed"],
            "last_error": self.last_error,
            "resource_usage": max(cpu, mem),
            "llm_usage": dict(self.llm_usage),
            "memory_store_failures": self.memory_errors["store"],
            "memory_search_failures": self.memory_errors["search"],
        }
        eng = getattr(getattr(self._llm, "engine", None), "metrics", None)
        if callable(eng):
            em = eng()
            # a full KV cache throttles delegation (TaskDelegator) but is not a fault:
            # it stays out of resource_usage, which FaultTolerance acts on
            m["kv_cache_utilization"] = 1.0 - em["free_kv_blocks"] / max(1, em["total_kv_blocks"])
        return m

    async def get_health(self) -> Dict[str, Any]:
        return {"status": self.status, "active_tasks": len(self.active_tasks), "total_tasks": len(self.tasks),
                "metrics": dict(self.task_metrics), "memory_usage": len(self.conversation_history),
                "last_heartbeat": self.last_heartbeat.isoformat(),
                "locks": {k: v.locked() for k, v in self.execution_locks.items()}}

    async def evaluate_task_suitability(self, task: Union[Dict[str, Any], Task]) -> float:
        """0 if capabilities missing; 0.7 (+0.2 specialisation) - 0.3 queue_util."""
        try:
            if isinstance(task, Task):
                task = {"type": task.type or task.metadata.get("type"), "required_capabilities": task.required_skills}
            req = set(task.get("required_capabilities") or [])
            if req - set(self.config.required_capabilities) - set(self.config.specializations):
                return 0.0
            score = 0.7
            if task.get("type") and task["type"] in self.config.specializations:
                score += 0.2
            score -= 0.3 * (len(self.tasks) / self.config.max_queue_size)
            return max(0.0, min(1.0, score))
        except Exception:  # noqa: BLE001
            return 0.0

    # ------------------------------------------------------------------ manager hooks
    async def determine_strategy(self, task: Task) -> Dict[str, Any]:
        return {"parallel_execution": True, "priority_level": task.priority,
                "resource_allocation": {"max_agents": 1, "time_allocation": 30, "tool_requirements": []},
                "coordination_needs": [], "monitoring_points": [], "abort_conditions": []}

    async def select_agent(self, task: Task) -> Optional["BaseAgent"]:
        best, best_s = None, -1.0
        for a in self.child_agents.values():
            if a.status in (AgentStatus.BUSY, AgentStatus.STOPPED, AgentStatus.ERROR):
                continue
            s = await a.evaluate_task_suitability(task)
            if s > best_s:
                best, best_s = a, s
        return best

    async def evaluate_result(self, task: Task, result: TaskResult) -> Dict[str, Any]:
        return {"success": result.success, "quality_score": 5, "matches_requirements": True, "goal_alignment": 5,
                "improvements": [], "next_actions": [], "requires_retry": not result.success,
                "reasoning": str(result.error) if not result.success else "Task completed"}

    def __repr__(self) -> str:
        return f"<{type(self).__name__} role={self.config.role!r} id={self.id[:8]} status={self.status}>"

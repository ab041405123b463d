"""Node-global orchestration plane for agent-DP (the reference's single
agent pool, pilott/pilott.py:93, spread over the GPUs of a node).

One process per GPU. Rank 0 hosts the ONE manager `Serve` (the orchestrator of BASELINE
config 3, "Manager + 64 workers"); every rank hosts worker agents next to its own engine.
Rank 0's Serve sees the whole node as one agent pool: the agents of rank r > 0 appear
there as `RemoteAgent` proxies, so the orchestrator, TaskRouter, LoadBalancer,
DynamicScaling and FaultTolerance act on the node-wide pool exactly as the reference's
act on one process (pilott/orchestration/load_balancer.py:180-251 moves tasks between any
agents, pilott/orchestration/orchestration.py:169-218 grows and shrinks the pool).

Transport: a small asyncio TCP control plane (length-prefixed JSON, 127.0.0.1 on one
node). The model tensors never cross it — each agent's LLM calls run on its own rank's
engine; only task descriptions, results and load counters travel. The manager's own LLM
calls (task analysis / evaluation) go through `DistributedLLM`, which sends each call to
the least-loaded live rank, so rank 0's GPU is not a hotspot.

Failure handling (SURVEY §5 "failure detection"; reference replace-and-transfer,
pilott/orchestration/scaling.py:323-372): worker ranks heartbeat every `hb_interval`
seconds with their load vector; a rank whose connection drops or whose heartbeat is older
than `hb_timeout` is declared lost. Every request in flight on it fails with
`AgentLostError`, its proxies leave the pool, and Serve re-queues those tasks on the
survivors (each submitted task completes exactly once; a late reply from a rank that was
declared lost is ignored).
"""
from __future__ import annotations

import asyncio
import hmac
import itertools
import json
import logging
import os
import secrets
import struct
import time
from datetime import datetime
from typing import Any, Callable, Dict, List, Optional, Sequence

from ..core.errors import AgentLostError
from ..core.policy import TASK_AGENT
from ..core.role import AgentStatus
from ..core.task import Task, TaskResult

log = logging.getLogger("pilottai_amd.node_plane")

_HDR = struct.Struct(">I")
MAX_MSG = 64 << 20


def plane_port() -> int:
    """Control-plane port: PILOTTAI_PLANE_PORT, else MASTER_PORT + 7."""
    if os.environ.get("PILOTTAI_PLANE_PORT"):
        return int(os.environ["PILOTTAI_PLANE_PORT"])
    return int(os.environ.get("MASTER_PORT", "29511")) + 7


def plane_secret() -> str:
    """Shared secret every worker's hello must carry (the plane had no
    authentication). PILOTTAI_PLANE_SECRET when set (launchers export it to every rank);
    otherwise, inside an initialised torch.distributed job, a token that rank 0 draws and
    broadcasts to the job's ranks; otherwise a per-process token (a lone rank 0)."""
    env = os.environ.get("PILOTTAI_PLANE_SECRET")
    if env:
        return env
    try:
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            box = [secrets.token_hex(16) if dist.get_rank() == 0 else None]
            dist.broadcast_object_list(box, src=0)
            os.environ["PILOTTAI_PLANE_SECRET"] = box[0]
            return box[0]
    except Exception:  # noqa: BLE001 — no usable process group: fall through
        pass
    tok = secrets.token_hex(16)
    os.environ["PILOTTAI_PLANE_SECRET"] = tok
    return tok


async def _send(writer: asyncio.StreamWriter, obj: Dict[str, Any]):
    data = json.dumps(obj, default=str).encode()
    writer.write(_HDR.pack(len(data)) + data)
    await writer.drain()


async def _recv(reader: asyncio.StreamReader) -> Dict[str, Any]:
    n = _HDR.unpack(await reader.readexactly(_HDR.size))[0]
    if n > MAX_MSG:
        raise ConnectionError(f"control message of {n} bytes")
    return json.loads(await reader.readexactly(n))


def _result_from(d: Dict[str, Any]) -> TaskResult:
    d = dict(d)
    d.pop("completion_time", None)
    return TaskResult(**{k: v for k, v in d.items() if k in TaskResult.model_fields})


def agent_descriptor(agent) -> Dict[str, Any]:
    cfg = agent.config
    return {"id": agent.id, "role": cfg.role, "role_type": str(getattr(cfg, "role_type", "worker")),
            "goal": getattr(cfg, "goal", ""), "description": getattr(cfg, "description", ""),
            "specializations": list(getattr(cfg, "specializations", None) or []),
            "required_capabilities": list(getattr(cfg, "required_capabilities", None) or []),
            "max_queue_size": int(getattr(cfg, "max_queue_size", 100)),
            "max_task_complexity": int(getattr(cfg, "max_task_complexity", 5))}


async def _agent_metrics(agent) -> Dict[str, Any]:
    try:
        m = await agent.get_metrics()
    except Exception:  # noqa: BLE001
        m = {}
    return {k: v for k, v in m.items() if isinstance(v, (int, float, str, bool)) or v is None}


# =====================================================================================
class RankState:
    def __init__(self, rank: int, writer: Optional[asyncio.StreamWriter]):
        self.rank = rank
        self.writer = writer
        self.alive = writer is not None or rank == 0
        self.last_hb = time.monotonic()
        self.load: Dict[str, float] = {}
        self.agent_metrics: Dict[str, Dict[str, Any]] = {}
        self.pending: Dict[int, asyncio.Future] = {}
        self.inflight = 0  # requests (exec + llm) currently routed to this rank


class PlaneServer:
    """Rank 0 side: accepts the worker ranks, routes requests, detects lost ranks."""

    def __init__(self, world: int, host: str = "127.0.0.1", port: Optional[int] = None,
                 hb_timeout: float = 5.0, local_load: Optional[Callable[[], Dict[str, float]]] = None,
                 secret: Optional[str] = None):
        self.world = world
        self._secret = secret or plane_secret()
        self.rejected = 0  # hellos refused (bad secret, rank out of range or already alive)
        self.agent_rank: Dict[Any, int] = {}  # agent id -> rank (NodeManager keeps it current)
        self.host = host
        self.port = port or plane_port()
        self.hb_timeout = hb_timeout
        self.local_load = local_load
        self.ranks: Dict[int, RankState] = {0: RankState(0, None)}
        self.local_inflight: Optional[Callable[[], float]] = None  # rank 0's own running work
        self.hellos: Dict[int, Dict[str, Any]] = {}
        self._ids = itertools.count(1)
        self._server: Optional[asyncio.AbstractServer] = None
        self._monitor: Optional[asyncio.Task] = None
        self._joined = asyncio.Event()
        self.on_rank_lost: List[Callable[[int], Any]] = []
        self._on_submit: Optional[Callable[[Dict[str, Any]], Any]] = None
        self._submit_backlog: List[tuple] = []  # submits that arrived before a handler was set
        self.lost: List[int] = []

    async def start(self, join_timeout: float = 300.0):
        self._server = await asyncio.start_server(self._handle, self.host, self.port)
        self._monitor = asyncio.ensure_future(self._monitor_loop())
        if self.world > 1:
            await asyncio.wait_for(self._joined.wait(), join_timeout)

    async def stop(self):
        self._stopping = True
        for r, st in list(self.ranks.items()):
            if r != 0 and st.alive and st.writer is not None:
                try:
                    await _send(st.writer, {"op": "shutdown"})
                except Exception:  # noqa: BLE001
                    pass
        if self._monitor:
            self._monitor.cancel()
        if self._server:
            self._server.close()
            try:
                await asyncio.wait_for(self._server.wait_closed(), 5)
            except Exception:  # noqa: BLE001
                pass

    # ---------------------------------------------------------------- connections
    async def _handle(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter):
        rank = None
        st = None
        try:
            hello = await _recv(reader)
            r = hello.get("rank") if hello.get("op") == "hello" else None
            ok = (isinstance(r, int) and 0 < r < self.world
                  and hmac.compare_digest(str(hello.get("secret", "")), self._secret)
                  and not (r in self.ranks and self.ranks[r].alive))
            if not ok:
                self.rejected += 1
                log.warning("control plane: refused a hello (rank %r)", r)
                writer.close()
                return
            rank = r
            st = RankState(rank, writer)
            st.load = hello.get("load", {})
            self.ranks[rank] = st
            self.hellos[rank] = hello
            if len([r for r in self.ranks if r != 0]) >= self.world - 1:
                self._joined.set()
            while True:
                msg = await _recv(reader)
                op = msg.get("op")
                if op == "hb":
                    st.last_hb = time.monotonic()
                    st.load = msg.get("load", {})
                    st.agent_metrics = msg.get("agents", {})
                elif op == "reply":
                    fut = st.pending.pop(msg["id"], None)
                    if fut is not None and not fut.done():
                        if msg.get("ok"):
                            fut.set_result(msg.get("result"))
                        else:
                            fut.set_exception(RuntimeError(msg.get("error", "remote error")))
                elif op == "submit":
                    if self._on_submit is None:
                        self._submit_backlog.append((st, msg))
                    else:
                        asyncio.ensure_future(self._serve_submit(st, msg))
        except (asyncio.IncompleteReadError, ConnectionError, OSError):
            pass
        finally:
            # only the connection that owns the rank's live state can declare it lost
            if rank is not None and self.ranks.get(rank) is st:
                self._declare_lost(rank, "connection closed")

    @property
    def on_submit(self):
        return self._on_submit

    @on_submit.setter
    def on_submit(self, fn):
        """Handler for tasks submitted on other ranks; submits that arrived earlier run now."""
        self._on_submit = fn
        backlog, self._submit_backlog = self._submit_backlog, []
        for st, msg in backlog:
            asyncio.ensure_future(self._serve_submit(st, msg))

    async def _serve_submit(self, st: RankState, msg: Dict[str, Any]):
        try:
            res = await self._on_submit(msg["task"])
            out = {"op": "reply", "id": msg["id"], "ok": True, "result": res}
        except Exception as e:  # noqa: BLE001
            out = {"op": "reply", "id": msg["id"], "ok": False, "error": repr(e)}
        if st.alive and st.writer is not None:
            try:
                await _send(st.writer, out)
            except Exception:  # noqa: BLE001
                pass

    async def _monitor_loop(self):
        while True:
            await asyncio.sleep(max(0.05, self.hb_timeout / 10))
            now = time.monotonic()
            for r, st in list(self.ranks.items()):
                if r != 0 and st.alive and now - st.last_hb > self.hb_timeout:
                    self._declare_lost(r, f"no heartbeat for {now - st.last_hb:.1f}s")

    def _declare_lost(self, rank: int, why: str):
        st = self.ranks.get(rank)
        if st is None or not st.alive:
            return
        st.alive = False
        if getattr(self, "_stopping", False):  # orderly shutdown, not a failure
            log.debug("rank %d left (%s)", rank, why)
        else:
            self.lost.append(rank)
            log.warning("rank %d lost (%s): %d requests in flight failed over", rank, why, len(st.pending))
        for fut in st.pending.values():
            if not fut.done():
                fut.set_exception(AgentLostError(f"rank {rank} lost ({why})"))
        st.pending.clear()
        try:
            if st.writer is not None:
                st.writer.close()
        except Exception:  # noqa: BLE001
            pass
        for cb in self.on_rank_lost:
            try:
                r = cb(rank)
                if asyncio.iscoroutine(r):
                    asyncio.ensure_future(r)
            except Exception as e:  # noqa: BLE001
                log.error("on_rank_lost hook failed: %s", e)

    # ---------------------------------------------------------------- requests
    async def call(self, rank: int, op: str, timeout: Optional[float] = None, **payload) -> Any:
        st = self.ranks.get(rank)
        if st is None or not st.alive or st.writer is None:
            raise AgentLostError(f"rank {rank} is not available")
        rid = next(self._ids)
        fut = asyncio.get_running_loop().create_future()
        st.pending[rid] = fut
        st.inflight += 1
        try:
            await _send(st.writer, {"op": op, "id": rid, **payload})
            return await (asyncio.wait_for(fut, timeout) if timeout else fut)
        except (ConnectionError, OSError) as e:
            self._declare_lost(rank, f"send failed: {e}")
            raise AgentLostError(f"rank {rank} lost") from e
        finally:
            st.inflight -= 1
            st.pending.pop(rid, None)

    def notify(self, rank: int, op: str, **payload):
        st = self.ranks.get(rank)
        if st is not None and st.alive and st.writer is not None:
            asyncio.ensure_future(self._notify(st, {"op": op, **payload}))

    async def _notify(self, st: RankState, msg):
        try:
            await _send(st.writer, msg)
        except Exception:  # noqa: BLE001
            pass

    # ---------------------------------------------------------------- load view
    def alive_ranks(self) -> List[int]:
        return sorted(r for r, st in self.ranks.items() if st.alive)

    def load_table(self) -> List[Dict[str, float]]:
        """Per-rank load (GlobalLoadView fields + in-flight requests), index = rank."""
        out = []
        for r in range(self.world):
            st = self.ranks.get(r)
            row = dict(st.load) if st is not None else {}
            if r == 0 and self.local_load is not None:
                row.update(self.local_load())
            row["alive"] = 1.0 if (st is not None and st.alive) else 0.0
            row["inflight"] = float(st.inflight) if st is not None else 0.0
            if r == 0 and self.local_inflight is not None:
                row["inflight"] += float(self.local_inflight())
            out.append(row)
        return out

    def least_loaded_rank(self, extra: Optional[Dict[int, float]] = None) -> int:
        """Fewest requests in flight + queued, then KV-cache utilisation; ties rotate."""
        table = self.load_table()
        live = self.alive_ranks()
        self._rr = (getattr(self, "_rr", -1) + 1) % max(1, self.world)
        return min(live, key=lambda r: (table[r].get("inflight", 0.0) + (extra or {}).get(r, 0.0)
                                        + table[r].get("queue_size", 0.0),
                                        round(table[r].get("kv_cache_utilization", 0.0), 2),
                                        (r - self._rr) % max(1, self.world)))


# =====================================================================================
class PlaneWorker:
    """Rank r > 0 side: hosts local agents (and the rank's LLM) for the manager on rank 0."""

    def __init__(self, rank: int, agents: Sequence[Any], llm: Any = None, host: str = "127.0.0.1",
                 port: Optional[int] = None, hb_interval: float = 0.5,
                 load_fn: Optional[Callable[[], Dict[str, float]]] = None,
                 agent_factory: Optional[Callable[..., Any]] = None, secret: Optional[str] = None):
        self.rank = rank
        self._secret = secret or plane_secret()
        self.agents: Dict[str, Any] = {a.id: a for a in agents}
        self.llm = llm
        self.host = host
        self.port = port or plane_port()
        self.hb_interval = hb_interval
        self.load_fn = load_fn
        self.agent_factory = agent_factory
        self._reader: Optional[asyncio.StreamReader] = None
        self._writer: Optional[asyncio.StreamWriter] = None
        self._ids = itertools.count(1)
        self._pending: Dict[int, asyncio.Future] = {}
        self._tasks: set = set()
        self.executed: List[str] = []  # task ids run here (tests / accounting)
        self.before_exec: Optional[Callable[[str], Any]] = None  # fault-injection hook

    async def connect(self, timeout: float = 300.0):
        t0 = time.monotonic()
        while True:
            try:
                self._reader, self._writer = await asyncio.open_connection(self.host, self.port)
                break
            except OSError:
                if time.monotonic() - t0 > timeout:
                    raise
                await asyncio.sleep(0.1)
        await _send(self._writer, {"op": "hello", "rank": self.rank, "secret": self._secret, "load": self._load(),
                                   "agents": [agent_descriptor(a) for a in self.agents.values()]})

    def _load(self) -> Dict[str, float]:
        base = {"queue_size": 0.0, "running_tasks": float(sum(len(getattr(a, "active_tasks", ())) for a in
                                                                 self.agents.values())),
                "idle_agents": float(sum(1 for a in self.agents.values() if str(a.status) == "idle"))}
        if self.load_fn is not None:
            base.update(self.load_fn())
        return base

    async def _heartbeat_loop(self):
        while True:
            metrics = {aid: await _agent_metrics(a) for aid, a in list(self.agents.items())}
            await _send(self._writer, {"op": "hb", "load": self._load(), "agents": metrics})
            await asyncio.sleep(self.hb_interval)

    async def serve_forever(self):
        """Handle the manager's requests until it says stop (or the connection drops)."""
        hb = asyncio.ensure_future(self._heartbeat_loop())
        try:
            while True:
                msg = await _recv(self._reader)
                op = msg.get("op")
                # the plane's shutdown; an agent-level "stop" (it names an agent_id) is a request
                if op == "shutdown" or (op == "stop" and "agent_id" not in msg):
                    break
                if op == "reply":
                    fut = self._pending.pop(msg["id"], None)
                    if fut is not None and not fut.done():
                        if msg.get("ok"):
                            fut.set_result(msg.get("result"))
                        else:
                            fut.set_exception(RuntimeError(msg.get("error", "remote error")))
                    continue
                t = asyncio.ensure_future(self._dispatch(msg))
                self._tasks.add(t)
                t.add_done_callback(self._tasks.discard)
        except (asyncio.IncompleteReadError, ConnectionError, OSError):
            pass
        finally:
            hb.cancel()
            for t in list(self._tasks):
                t.cancel()
            try:
                self._writer.close()
            except Exception:  # noqa: BLE001
                pass

    async def submit(self, task: Any) -> TaskResult:
        """Submit a task on this rank: it is forwarded to the node's manager (rank 0)."""
        rid = next(self._ids)
        fut = asyncio.get_running_loop().create_future()
        self._pending[rid] = fut
        await _send(self._writer, {"op": "submit", "id": rid, "task": Task.from_any(task).to_dict()})
        return _result_from(await fut)

    async def _reply(self, rid, ok: bool, result=None, error: str = ""):
        try:
            await _send(self._writer, {"op": "reply", "id": rid, "ok": ok, "result": result, "error": error})
        except Exception:  # noqa: BLE001
            pass

    async def _dispatch(self, msg: Dict[str, Any]):
        op, rid = msg["op"], msg.get("id")
        try:
            if op in ("prefetch", "drop"):  # notifications, no reply
                a = self.agents.get(msg["agent_id"])
                if a is not None:
                    if op == "prefetch" and hasattr(a, "prefetch_opening"):
                        a.prefetch_opening(Task.from_any(msg["task"]))
                    elif op == "drop" and hasattr(a, "drop_opening"):
                        a.drop_opening(msg["task_id"])
                return
            res = await self._handle(op, msg)
            await self._reply(rid, True, res)
        except asyncio.CancelledError:
            raise
        except Exception as e:  # noqa: BLE001
            await self._reply(rid, False, error=repr(e))

    async def _handle(self, op: str, msg: Dict[str, Any]) -> Any:
        if op == "llm":
            r = await self.llm.generate_response(msg["messages"], tools=msg.get("tools"),
                                                 response_format=msg.get("response_format"))
            return r
        if op == "create_agent":
            a = self.agent_factory(**msg.get("kw", {}))
            if asyncio.iscoroutine(a):
                a = await a
            await a.start()
            self.agents[a.id] = a
            return agent_descriptor(a)
        a = self.agents[msg["agent_id"]]
        if op == "exec":
            task = Task.from_any(msg["task"])
            if self.before_exec is not None:
                self.before_exec(task.id)
            self.executed.append(task.id)
            r = await a.execute_task(task)
            return r.model_dump(mode="json")
        if op == "add_task":
            return await a.add_task(Task.from_any(msg["task"]))
        if op == "remove_task":
            t = await a.remove_task(msg["task_id"])
            return t.to_dict() if t is not None else None
        if op == "queue":
            return sorted(a.tasks)
        if op == "suitability":
            return float(await a.evaluate_task_suitability(Task.from_any(msg["task"])))
        if op in ("start", "stop", "reset", "pause_task_acceptance", "resume_task_acceptance"):
            await getattr(a, op)()
            return True
        if op == "remove_agent":
            self.agents.pop(a.id, None)
            await a.stop()
            return True
        raise ValueError(f"unknown op {op}")


# =====================================================================================
class _ProxyConfig:
    def __init__(self, d: Dict[str, Any]):
        self.role = d["role"]
        self.role_type = d.get("role_type", "worker")
        self.goal = d.get("goal", "")
        self.description = d.get("description", "")
        self.specializations = d.get("specializations", [])
        self.required_capabilities = d.get("required_capabilities", [])
        self.max_queue_size = d.get("max_queue_size", 100)
        self.max_task_complexity = d.get("max_task_complexity", 5)
        self.allow_delegation = False
        self.max_concurrent_tasks = 1


class RemoteAgent:
    """An agent living on another rank, seen from the manager (rank 0). Implements the
    agent protocol the orchestrator and the control-plane services use."""

    def __init__(self, plane: PlaneServer, rank: int, desc: Dict[str, Any]):
        self.plane = plane
        self.rank = rank
        self.id = desc["id"]
        self.config = _ProxyConfig(desc)
        self.status = AgentStatus.IDLE
        self._accepting = True
        self.active_tasks: set = set()
        self.tasks: Dict[str, Task] = {}  # this agent's queued tasks (mirrored from its rank)
        self.last_heartbeat = datetime.now()

    def __repr__(self) -> str:
        return f"RemoteAgent({self.config.role!r}, rank={self.rank})"

    @property
    def specializations(self) -> List[str]:
        return list(self.config.specializations)

    @property
    def accepting_tasks(self) -> bool:
        return self._accepting and self.plane.ranks.get(self.rank, RankState(self.rank, None)).alive

    async def execute_task(self, task) -> TaskResult:
        task = Task.from_any(task)
        self.active_tasks.add(task.id)
        self.status = AgentStatus.BUSY
        try:
            d = await self.plane.call(self.rank, "exec", agent_id=self.id, task=task.to_dict())
            return _result_from(d)
        finally:
            self.active_tasks.discard(task.id)
            self.tasks.pop(task.id, None)
            if not self.active_tasks and self.status == AgentStatus.BUSY and self._accepting:
                self.status = AgentStatus.IDLE

    def prefetch_opening(self, task: Task):
        self.plane.notify(self.rank, "prefetch", agent_id=self.id, task=Task.from_any(task).to_dict())

    def drop_opening(self, task_id: str):
        self.plane.notify(self.rank, "drop", agent_id=self.id, task_id=task_id)

    async def add_task(self, task) -> str:
        t = Task.from_any(task)
        await self.plane.call(self.rank, "add_task", agent_id=self.id, task=t.to_dict())
        self.tasks[t.id] = t
        return t.id

    async def remove_task(self, task_id: str) -> Optional[Task]:
        await self.plane.call(self.rank, "remove_task", agent_id=self.id, task_id=task_id)
        return self.tasks.pop(task_id, None)

    async def remote_queue(self) -> List[str]:
        return await self.plane.call(self.rank, "queue", agent_id=self.id)

    async def get_metrics(self) -> Dict[str, Any]:
        st = self.plane.ranks.get(self.rank)
        m = dict(st.agent_metrics.get(self.id, {})) if st is not None else {}
        m.setdefault("queue_size", len(self.tasks))
        m.setdefault("active_tasks", len(self.active_tasks))
        if st is not None:
            m["kv_cache_utilization"] = float(st.load.get("kv_cache_utilization", 0.0))
            m["rank"] = self.rank
        return m

    async def evaluate_task_suitability(self, task) -> float:
        t = task if isinstance(task, dict) else Task.from_any(task).to_dict()
        try:
            return float(await self.plane.call(self.rank, "suitability", timeout=10, agent_id=self.id, task=t))
        except Exception:  # noqa: BLE001
            return 0.0

    async def send_heartbeat(self) -> datetime:
        st = self.plane.ranks.get(self.rank)
        if st is None or not st.alive:
            raise AgentLostError(f"rank {self.rank} lost")
        self.last_heartbeat = datetime.now()
        return self.last_heartbeat

    async def _op(self, op: str):
        try:
            await self.plane.call(self.rank, op, timeout=30, agent_id=self.id)
        except AgentLostError:
            pass

    async def start(self):
        await self._op("start")

    async def stop(self):
        self.status = AgentStatus.STOPPED
        await self._op("stop")

    async def reset(self):
        await self._op("reset")
        self.status = AgentStatus.IDLE

    async def pause_task_acceptance(self):
        self._accepting = False
        await self._op("pause_task_acceptance")

    async def resume_task_acceptance(self):
        self._accepting = True
        await self._op("resume_task_acceptance")

    async def wait_for_tasks(self, poll: float = 0.05, timeout: Optional[float] = None):
        t0 = time.monotonic()
        while self.active_tasks:
            if timeout is not None and time.monotonic() - t0 > timeout:
                raise asyncio.TimeoutError
            await asyncio.sleep(poll)

    async def cleanup_resources(self):
        self.tasks.clear()


# =====================================================================================
class DistributedLLM:
    """The manager's LLM: each call goes to the least-loaded live rank's engine (local call
    on rank 0, RPC elsewhere). Same protocol as engine.local_llm.BaseLLM."""

    provider = "distributed"

    def __init__(self, plane: PlaneServer, local_llm: Any, affinity: bool = True):
        self.plane = plane
        self.local = local_llm
        self.affinity = affinity and os.environ.get("PILOTTAI_LLM_AFFINITY", "1") != "0"
        self.model_name = getattr(local_llm, "model_name", "llama-3-8b")
        self.usage = {"calls": 0, "prompt_tokens": 0, "completion_tokens": 0}
        self.calls_by_rank: Dict[int, int] = {}
        self._local_inflight = 0

    async def generate_response(self, messages: List[Dict[str, str]], tools: Optional[List[Dict]] = None,
                                response_format: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
        aff = self.plane.agent_rank.get(TASK_AGENT.get()) if self.affinity else None
        while True:
            # the rank of the task's own agent (its prompt prefix is cached there), else the
            # least-loaded live rank
            if aff is not None and self.plane.ranks.get(aff) is not None and self.plane.ranks[aff].alive:
                r = aff
            else:
                r = self.plane.least_loaded_rank(extra={0: float(self._local_inflight)})
            # (remote ranks' in-flight count already includes their routed calls)
            self.calls_by_rank[r] = self.calls_by_rank.get(r, 0) + 1
            try:
                if r == 0:
                    self._local_inflight += 1
                    try:
                        out = await self.local.generate_response(messages, tools=tools, response_format=response_format)
                    finally:
                        self._local_inflight -= 1
                else:
                    out = await self.plane.call(r, "llm", messages=messages, tools=tools,
                                                response_format=response_format)
                break
            except AgentLostError:
                aff = None
                continue  # that rank died under the call: send it elsewhere
        u = out.get("usage", {})
        self.usage["calls"] += 1
        self.usage["prompt_tokens"] += int(u.get("prompt_tokens", 0))
        self.usage["completion_tokens"] += int(u.get("completion_tokens", 0))
        return out

    async def apredict(self, prompt: str, response_format: Optional[Dict[str, Any]] = None) -> str:
        r = await self.generate_response([{"role": "user", "content": prompt}], response_format=response_format)
        return r["content"]

    async def apredict_messages(self, messages: List[Dict], functions: List[Dict]) -> Dict[str, Any]:
        return await self.generate_response(messages, tools=functions)


# =====================================================================================
class NodeManager:
    """Rank 0: builds the node-wide agent pool on a Serve and keeps it in sync with the
    plane (proxies of lost ranks leave the pool; DynamicScaling's create_agent lands on
    the least-loaded rank)."""

    def __init__(self, plane: PlaneServer, serve):
        self.plane = plane
        self.serve = serve
        self.proxies: Dict[str, RemoteAgent] = {}
        self.rank_of: Dict[str, int] = {}
        plane.agent_rank = self.rank_of  # DistributedLLM's task -> rank affinity
        plane.on_rank_lost.append(self._rank_lost)
        plane.on_submit = self._remote_submit
        serve.node = self
        serve.agent_rank = lambda a: self.rank_of.get(a.id, 0)
        # rank 0's engine load for routing = tasks running on its local agents
        plane.local_inflight = lambda: float(sum(1 for aid in serve.running_tasks.values()
                                                 if self.rank_of.get(aid, 0) == 0))

    def attach_remote_agents(self):
        for r, hello in sorted(self.plane.hellos.items()):
            for d in hello.get("agents", []):
                self._add_proxy(r, d)

    def _add_proxy(self, rank: int, desc: Dict[str, Any]) -> RemoteAgent:
        p = RemoteAgent(self.plane, rank, desc)
        self.proxies[p.id] = p
        self.rank_of[p.id] = rank
        self.serve._register_agent(p)
        return p

    def register_local(self, agents: Sequence[Any]):
        for a in agents:
            self.rank_of[a.id] = 0

    async def _rank_lost(self, rank: int):
        for aid, p in list(self.proxies.items()):
            if p.rank == rank:
                self.proxies.pop(aid, None)
                p.status = AgentStatus.ERROR
                await self.serve.remove_agent(aid)

    async def _remote_submit(self, task_dict: Dict[str, Any]) -> Dict[str, Any]:
        r = await self.serve.execute_task(Task.from_any(task_dict), timeout=None)
        return r.model_dump(mode="json")

    async def create_agent(self, **kw):
        """DynamicScaling hook: a new worker on the least-loaded live rank."""
        r = self.plane.least_loaded_rank()
        if r == 0 or self.plane.world == 1:
            return None  # the caller falls back to a local agent
        desc = await self.plane.call(r, "create_agent", timeout=60, kw=kw)
        p = RemoteAgent(self.plane, r, desc)
        self.proxies[p.id] = p
        self.rank_of[p.id] = r
        return p

    def executions_by_rank(self) -> Dict[int, int]:
        """Finished tasks (completed or failed) per rank, from the agent each task last ran on
        (Serve records it in task.metadata["_agent_id"]); every rank with agents appears."""
        out: Dict[int, int] = {r: 0 for r in self.rank_of.values()}
        done = set(self.serve.completed_tasks) | set(self.serve.failed_tasks)
        for tid in done:
            t = self.serve.tasks.get(tid)
            aid = t.metadata.get("_agent_id") if t is not None else None
            if aid is not None and aid in self.rank_of:
                r = self.rank_of[aid]
                out[r] = out.get(r, 0) + 1
        return out

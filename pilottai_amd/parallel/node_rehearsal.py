"""Multi-process rehearsal of the node control plane on the CPU (no GPU, no engine).

Each rank is a process with schema-valid model-free LLMs (engine.local_llm.SchemaLLM,
a fixed latency per call) and real BaseAgents; rank 0 runs the single manager Serve over
the node-wide pool (parallel/node_plane.py). Scenarios, each verifiable from rank 0's
report:

  balance  tasks submitted at rank 0 AND forwarded from the last rank (skewed
           submission) end up spread over the ranks within +-1 task per rank
  lb_move  the LoadBalancer moves queued tasks from an agent on rank 1 to one on rank 2
  scale    DynamicScaling's create_agent places a new worker on the least-loaded rank
  kill     rank 2 dies (os._exit) in the middle of the run: every submitted task still
           completes exactly once (its in-flight tasks are re-queued on survivors)
  throughput / throughput_indep
           capacity of the plane: world x per_rank closed-loop clients
           for `duration` seconds, every LLM call taking `latency` s (the measured per-call
           latency of a rank). "throughput": all clients talk to rank 0's one manager Serve over
           the node-wide pool; "throughput_indep": every rank runs its own Serve over its own
           agents. Reports tasks/s and rank 0's event-loop lag (a 10 ms sleep probe).

    python -m pilottai_amd.parallel.node_rehearsal --world 8 --scenario balance
"""
from __future__ import annotations

import argparse
import asyncio
import json
import multiprocessing as mp
import os
import secrets
import socket
import sys
import time
from typing import Any, Dict, List


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _agents(rank: int, n: int, llm):
    from ..core.agent import BaseAgent
    from ..core.config import AgentConfig
    from ..core.policy import ControlPolicy
    from ..tools.tool import Tool, echo_tool

    pol = ControlPolicy("fixed", 1)
    return [BaseAgent(AgentConfig(role=f"worker-r{rank}-{i}", goal="Summarize documents", max_iterations=2),
                      llm=llm, tools=[Tool(name="echo", description="identity tool", function=echo_tool,
                                           max_retries=1)], policy=pol)
            for i in range(n)]


async def _rank0(world: int, port: int, scenario: str, per_rank: int, n_tasks: int, latency: float,
                 forwarded: int = 0) -> Dict[str, Any]:
    from ..core.task import Task
    from ..engine.local_llm import SchemaLLM
    from ..orchestration.load_balancer import LoadBalancer, LoadMetrics
    from ..serve import Serve
    from .node_plane import DistributedLLM, NodeManager, PlaneServer

    llm = SchemaLLM(seed=0, latency_s=latency)
    agents = _agents(0, per_rank, llm)
    plane = PlaneServer(world, port=port, hb_timeout=2.0)
    await plane.start(join_timeout=120)
    serve = Serve(agents=agents, config={"name": "node", "max_concurrent_tasks": 4 * world * per_rank,
                                         "policy": "fixed", "max_queue_size": 100000, "task_timeout": 120,
                                         "agent_wait_timeout": 120})
    node = NodeManager(plane, serve)
    node.register_local(agents)
    node.attach_remote_agents()
    serve._manager_llm = DistributedLLM(plane, llm)
    await serve.start()
    out: Dict[str, Any] = {"scenario": scenario, "world": world, "agents": len(serve.agents)}
    try:
        if scenario in ("balance", "kill"):
            tasks = [Task(description=f"Summarize the document and list its key findings: doc {i}")
                     for i in range(n_tasks)]
            results = await asyncio.gather(*(serve.execute_task(t) for t in tasks))
            t_end = time.time() + 60
            while serve.metrics["processed_tasks"] < n_tasks + forwarded and time.time() < t_end:
                await asyncio.sleep(0.05)  # tasks forwarded from other ranks
            out["submitted"] = len(tasks) + forwarded
            out["processed"] = int(serve.metrics["processed_tasks"])
            out["succeeded"] = sum(1 for r in results if r.success) + sum(
                1 for t, r in serve.completed_tasks.items() if "forwarded" in serve.tasks[t].description)
            out["completed_ids"] = len(serve.completed_tasks)
            out["unique_completed"] = len(set(serve.completed_tasks))
            out["requeued"] = int(serve.metrics.get("requeued_tasks", 0))
            out["lost_ranks"] = list(plane.lost)
            out["local_executed"] = sum(a.task_metrics.get("completed", 0) + a.task_metrics.get("failed", 0)
                                        for a in agents)
            out["llm_calls_by_rank"] = {str(k): v for k, v in serve._manager_llm.calls_by_rank.items()}
            out["agents_after"] = len(serve.agents)
            out["executions_by_rank"] = {str(k): v for k, v in node.executions_by_rank().items()}
        elif scenario == "lb_move":
            p1 = next(p for p in node.proxies.values() if p.rank == 1)
            p2 = next(p for p in node.proxies.values() if p.rank == 2)
            ids = []
            for i in range(3):
                ids.append(await p1.add_task(Task(description=f"queued work item {i}")))
            lb = LoadBalancer(serve, {"balance_batch_size": 2})
            metrics = {p1.id: LoadMetrics(cpu_usage=0.9, memory_usage=0.9, queue_size=3),
                       p2.id: LoadMetrics(cpu_usage=0.05, memory_usage=0.05, queue_size=0)}
            await lb._redistribute_tasks([p1.id], [p2.id], metrics)
            out["moved"] = lb.moves
            out["src_queue"] = await p1.remote_queue()
            out["dst_queue"] = await p2.remote_queue()
            out["queued_ids"] = ids
            # stopping ONE remote agent is an agent request, not the plane's shutdown: its rank
            # keeps serving (scale-down of a remote worker)
            await p1.stop()
            await asyncio.sleep(0.3)
            out["lost_after_agent_stop"] = list(plane.lost)
            out["rank1_alive"] = bool(plane.ranks[1].alive)
            out["rank1_serving"] = isinstance(await p1.remote_queue(), list)
        elif scenario == "throughput":
            out.update(await _closed_loop(serve, world * per_rank, latency))
        elif scenario == "scale":
            before = {r: 0 for r in range(world)}
            for aid, r in node.rank_of.items():
                before[r] += 1
            # make rank 0 look busy so the new agent must land elsewhere
            plane.local_load = lambda: {"queue_size": 100.0}
            a = await serve.create_agent(role="scaled-worker")
            await serve.add_child_agent(a)
            out["new_rank"] = node.rank_of.get(a.id)
            out["registered"] = a.id in serve.agents
            r = await serve.execute_task(Task(description="Summarize the document: scaled"))
            out["scaled_ok"] = r.success
    finally:
        await serve.stop()
        await plane.stop()
    return out


THROUGHPUT_S = 8.0  # measured window of the throughput scenarios (after a 1 s warm-up)


async def _closed_loop(serve, n_clients: int, latency: float) -> Dict[str, Any]:
    """n_clients closed-loop clients on `serve`; tasks/s over the window + event-loop lag."""
    from ..core.task import Task

    loop = asyncio.get_running_loop()
    t_start = time.time() + 1.0
    t_end = t_start + THROUGHPUT_S
    done = [0]
    lags: List[float] = []

    async def client(i):
        k = 0
        while time.time() < t_end:
            r = await serve.execute_task(Task(description=f"Summarize the document and list its findings: {i}/{k}"))
            k += 1
            if r.success and t_start <= time.time() < t_end:
                done[0] += 1

    async def probe():
        while time.time() < t_end:
            t0 = loop.time()
            await asyncio.sleep(0.01)
            if time.time() >= t_start:
                lags.append(loop.time() - t0 - 0.01)

    await asyncio.gather(probe(), *(client(i) for i in range(n_clients)))
    lags.sort()
    pct = lambda q: round(1e3 * lags[min(len(lags) - 1, int(q * len(lags)))], 2) if lags else None  # noqa: E731
    return {"clients": n_clients, "latency_s": latency, "window_s": THROUGHPUT_S,
            "tasks_per_s": round(done[0] / THROUGHPUT_S, 2),
            "loop_lag_ms_p50": pct(0.5), "loop_lag_ms_p99": pct(0.99), "loop_lag_ms_max": pct(1.0)}


async def _independent(rank: int, per_rank: int, latency: float) -> Dict[str, Any]:
    from ..engine.local_llm import SchemaLLM
    from ..serve import Serve

    llm = SchemaLLM(seed=rank, latency_s=latency)
    agents = _agents(rank, per_rank, llm)
    serve = Serve(agents=agents, manager_llm=llm,
                  config={"name": f"indep-{rank}", "max_concurrent_tasks": 4 * per_rank, "policy": "fixed",
                          "max_queue_size": 100000, "task_timeout": 120, "agent_wait_timeout": 120})
    await serve.start()
    try:
        res = await _closed_loop(serve, per_rank, latency)
    finally:
        await serve.stop()
    res["rank"] = rank
    if rank == 0:
        res["scenario"] = "throughput_indep"
    return res


async def _worker(rank: int, world: int, port: int, scenario: str, per_rank: int, latency: float,
                  submit: int) -> Dict[str, Any]:
    from ..core.task import Task
    from ..engine.local_llm import SchemaLLM
    from .node_plane import PlaneWorker

    llm = SchemaLLM(seed=rank, latency_s=latency)
    agents = _agents(rank, per_rank, llm)
    for a in agents:
        await a.start()
    w = PlaneWorker(rank, agents, llm=llm, port=port, hb_interval=0.2,
                    agent_factory=lambda **kw: _agents(rank, 1, llm)[0])
    if scenario == "kill" and rank == 2:
        seen = {"n": 0}

        def die(_tid):
            seen["n"] += 1
            if seen["n"] == 3:  # two tasks done here, the third is in flight: the rank dies
                os._exit(17)
        w.before_exec = die
    await w.connect(timeout=120)
    forwarded: List[bool] = []
    if submit:
        async def fwd():
            rs = await asyncio.gather(*(w.submit(Task(description=f"Summarize the document: forwarded {rank}-{i}"))
                                        for i in range(submit)))
            forwarded.extend(r.success for r in rs)
        ft = asyncio.ensure_future(fwd())
        await w.serve_forever()
        if not ft.done():
            ft.cancel()
    else:
        await w.serve_forever()
    return {"rank": rank, "executed": len(w.executed), "forwarded_ok": sum(forwarded)}


def _entry(rank, world, port, scenario, per_rank, n_tasks, latency, q):
    try:
        if scenario == "throughput_indep":
            res = asyncio.run(_independent(rank, per_rank, latency))
        elif rank == 0:
            fwd = n_tasks // 2 if scenario == "balance" and world > 1 else 0
            res = asyncio.run(_rank0(world, port, scenario, per_rank, n_tasks - fwd, latency, fwd))
        else:
            submit = n_tasks // 2 if (scenario == "balance" and rank == world - 1) else 0
            res = asyncio.run(_worker(rank, world, port, scenario, per_rank, latency, submit))
        q.put(res)
    except Exception as e:  # noqa: BLE001
        q.put({"rank": rank, "error": repr(e)})
        raise


def run(world: int, scenario: str, per_rank: int = 2, n_tasks: int = 0, latency: float = 0.01,
        timeout: float = 240.0) -> Dict[str, Any]:
    """Run the scenario over `world` processes; returns rank 0's report + per-rank stats."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    # the control plane's shared secret reaches every spawned rank through the environment
    os.environ.setdefault("PILOTTAI_PLANE_SECRET", secrets.token_hex(16))
    # balance: one wave — half the pool's worth submitted at rank 0, half forwarded from
    # the last rank, all at once — must land one task per agent
    n_tasks = n_tasks or (world * per_rank * (1 if scenario == "balance" else 5))
    procs = [ctx.Process(target=_entry, args=(r, world, port, scenario, per_rank,
                                               n_tasks if r == 0 and scenario == "balance" else n_tasks,
                                               latency, q), daemon=True)
             for r in range(world)]
    for p in procs:
        p.start()
    reports: List[Dict[str, Any]] = []
    t0 = time.time()
    expect = world - (1 if scenario == "kill" and world > 2 else 0)
    while len(reports) < expect and time.time() - t0 < timeout:
        try:
            reports.append(q.get(timeout=1.0))
        except Exception:  # noqa: BLE001 — queue.Empty
            if all(not p.is_alive() for p in procs) and q.empty():
                break
    for p in procs:
        p.join(timeout=10)
        if p.is_alive():
            p.kill()
    main = next((r for r in reports if "scenario" in r), {})
    main["ranks"] = sorted((r for r in reports if "scenario" not in r), key=lambda r: r.get("rank", 0))
    main["exitcodes"] = [p.exitcode for p in procs]
    if scenario == "throughput_indep":  # rank 0's report holds its own rate: add the others'
        main["rank0_tasks_per_s"] = main.get("tasks_per_s", 0.0)
        main["tasks_per_s"] = round(main.get("tasks_per_s", 0.0) + sum(r.get("tasks_per_s", 0.0)
                                                                        for r in main["ranks"]), 2)
        main["clients"] = world * per_rank
    return main


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--scenario", default="balance",
                    choices=["balance", "lb_move", "scale", "kill", "throughput", "throughput_indep"])
    ap.add_argument("--per-rank", type=int, default=2)
    ap.add_argument("--tasks", type=int, default=0)
    ap.add_argument("--latency", type=float, default=0.01, help="seconds per LLM call")
    a = ap.parse_args()
    print(json.dumps(run(a.world, a.scenario, a.per_rank, a.tasks, latency=a.latency)))
    return 0


if __name__ == "__main__":
    sys.exit(main())

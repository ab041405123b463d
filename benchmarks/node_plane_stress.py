#!/usr/bin/env python3
"""Capacity of the multi-GPU control plane with every rank's agents on schema LLMs (no GPU).

The node plane (parallel/node_plane.py) carries, for every task of the whole node, the
manager's decisions on rank 0 and the dispatch to the rank that hosts the chosen agent, as
length-prefixed JSON over localhost TCP, plus heartbeats and load reports. In the real
8-GPU run each rank's engine answers an agent call in ~80 ms (8-worker per-call latency);
this benchmark replaces the engines with `SchemaLLM` (instant, or a fixed latency) so the
plane, rank 0's event loop and the manager are the only work left -- i.e. it measures how
many tasks/s the plane can route before it, not the GPUs, limits the node.

    python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        --master-port 29561 benchmarks/node_plane_stress.py --latency 0 --tasks-per-client 8

(PILOTTAI_DIST_BACKEND=gloo is set here: CPU ranks only.) Rank 0 prints one JSON line:
tasks/s, task latency p50 / p99, rank-0 event-loop lag p50 / p99, executions per rank.
Reference: the reference runs all agents in one asyncio loop (pilott/pilott.py:272-303).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import secrets
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("PILOTTAI_DIST_BACKEND", "gloo")


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else 0.0


async def run(a, rank: int, world: int):
    from pilottai_amd.core.agent import BaseAgent
    from pilottai_amd.core.config import AgentConfig
    from pilottai_amd.core.policy import ControlPolicy
    from pilottai_amd.core.task import Task
    from pilottai_amd.engine.local_llm import SchemaLLM
    from pilottai_amd.parallel import comm
    from pilottai_amd.parallel.node_plane import DistributedLLM, NodeManager, PlaneServer, PlaneWorker
    from pilottai_amd.serve import Serve
    from pilottai_amd.tools.tool import Tool, echo_tool

    async def coll(fn, *args):
        return await asyncio.to_thread(fn, *args)

    n_local = a.workers // world
    llm = SchemaLLM(seed=rank, latency_s=a.latency)
    policy = ControlPolicy("fixed", a.steps_per_task)
    agents = [BaseAgent(AgentConfig(role=f"analyst-{rank}-{i}", goal="Summarize documents",
                                    max_iterations=a.steps_per_task + 1, task_timeout=900), llm=llm,
                        tools=[Tool(name="echo", description="identity tool", function=echo_tool, max_retries=1)],
                        policy=policy)
              for i in range(n_local)]
    os.environ["PILOTTAI_PLANE_SECRET"] = await coll(
        comm.broadcast_object, secrets.token_hex(16) if rank == 0 else None)
    if rank > 0:
        for ag in agents:
            await ag.start()
        worker = PlaneWorker(rank, agents, llm=llm)
        await worker.connect()
        serving = asyncio.ensure_future(worker.serve_forever())
        await coll(comm.barrier)  # warmup done
        await coll(comm.barrier)  # timed round done
        await serving
        for ag in agents:
            await ag.stop()
        return {"calls": len(llm.calls)}

    plane = PlaneServer(world)
    await plane.start()
    serve = Serve(agents=agents, config={"name": "plane-stress", "policy": "fixed", "steps_per_task": a.steps_per_task,
                                         "max_queue_size": 100000, "task_timeout": 900, "agent_wait_timeout": 900,
                                         "max_concurrent_tasks": a.workers})
    mgr = NodeManager(plane, serve)
    mgr.register_local(agents)
    mgr.attach_remote_agents()
    dllm = DistributedLLM(plane, llm)
    serve._manager_llm = dllm
    await serve.start()
    lat, lags = [], []

    async def client(ci, n, rec):
        for j in range(n):
            t0 = time.perf_counter()
            r = await serve.execute_task(Task(description=f"Summarize document {ci}-{j} and list its findings."))
            if not r.success:
                raise RuntimeError(f"task failed: {r.error}")
            if rec:
                lat.append(time.perf_counter() - t0)

    async def probe(stop):
        loop = asyncio.get_running_loop()
        while not stop.is_set():
            t = loop.time()
            await asyncio.sleep(0.01)
            lags.append(loop.time() - t - 0.01)

    await asyncio.gather(*(client(i, 1, False) for i in range(a.clients)))
    await coll(comm.barrier)
    e0 = dict(mgr.executions_by_rank())
    stop = asyncio.Event()
    pr = asyncio.ensure_future(probe(stop))
    t0 = time.perf_counter()
    await asyncio.gather(*(client(i, a.tasks_per_client, True) for i in range(a.clients)))
    dt = time.perf_counter() - t0
    stop.set()
    await pr
    e1 = mgr.executions_by_rank()
    await coll(comm.barrier)
    await serve.stop()
    await plane.stop()
    n = len(lat)
    return {"metric": "control-plane capacity: agent-tasks/s routed by the node plane (schema LLMs, no GPU)",
            "value": round(n / dt, 1), "unit": "tasks/s", "ranks": world, "workers": a.workers,
            "clients": a.clients, "llm_latency_s": a.latency, "llm_calls_per_task": 7,
            "tasks": n, "seconds": round(dt, 3),
            "task_p50_ms": round(1000 * pct(lat, 0.5), 2), "task_p99_ms": round(1000 * pct(lat, 0.99), 2),
            "rank0_loop_lag_ms": {"p50": round(1000 * pct(lags, 0.5), 2), "p99": round(1000 * pct(lags, 0.99), 2)},
            "executions_by_rank": {str(k): e1.get(k, 0) - e0.get(k, 0) for k in sorted(e1)},
            # manager LLM calls routed over the plane (the task's own agent's rank, else least loaded)
            "manager_calls_by_rank": {str(k): v for k, v in sorted(dllm.calls_by_rank.items())}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=64, help="agents over all ranks")
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--tasks-per-client", type=int, default=8)
    ap.add_argument("--steps-per-task", type=int, default=1)
    ap.add_argument("--latency", type=float, default=0.0, help="seconds per schema-LLM call")
    a = ap.parse_args()
    from pilottai_amd.parallel import comm

    rank, world, _ = comm.init_distributed()
    res = asyncio.run(run(a, rank, world))
    if rank == 0:
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

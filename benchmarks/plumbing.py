#!/usr/bin/env python3
"""BASELINE config 1: orchestration plumbing on the CPU asyncio loop — no GPU, no LLM.

Reproduces the reference measurement of BASELINE.md §3: the real `Serve` queue,
worker loop and orchestrator path (task analysis + result evaluation through an
instant fake manager LLM), echo agents, closed-loop clients that submit a task
and await its result. Reference (8-vCPU Xeon): 5,052 tasks/s p50 0.153 ms at 1
client; 5,125 tasks/s p50 1.325 ms at 8; 5,312 tasks/s p50 10.426 ms at 64.

    python benchmarks/plumbing.py [--clients 1,8,64] [--tasks 20000] [--same-box-reference]

--same-box-reference runs the reference's own Serve (benchmarks/reference_plumbing.py)
alternating with ours, on this machine, so the comparison does not depend on BASELINE.md's
survey-session hardware.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

REF = {1: (5052, 0.153, 0.402), 8: (5125, 1.325, 6.414), 64: (5312, 10.426, 34.909)}

_ANALYSIS = json.dumps({"requires_decomposition": False, "complexity": "low", "dependencies": [],
                        "estimated_resources": {"time": "1m", "agents": 1, "tools": []}, "priority": 1})
_EVAL = json.dumps({"success": True, "quality": {"completeness": 1, "accuracy": 1}, "requires_retry": False})


class InstantLLM:
    """Fake manager LLM: returns valid orchestrator JSON immediately."""

    async def apredict(self, prompt, response_format=None):
        schema = (response_format or {}).get("schema", "")
        return _EVAL if schema.endswith("result_evaluation") else _ANALYSIS

    async def generate_response(self, messages, **kw):
        return {"content": _ANALYSIS}


def make_echo_agent_cls():
    from pilottai_amd.core.agent import BaseAgent
    from pilottai_amd.core.task import TaskResult

    class EchoAgent(BaseAgent):
        async def _execute_task_internal(self, task):
            return TaskResult(success=True, output=task.description, execution_time=0.0)

    return EchoAgent


async def run(clients: int, n_tasks: int):
    from pilottai_amd.core.config import AgentConfig
    from pilottai_amd.core.task import Task
    from pilottai_amd.serve import Serve

    Echo = make_echo_agent_cls()
    agents = [Echo(AgentConfig(role=f"echo-{i}", goal="echo")) for i in range(clients)]
    serve = Serve(agents=agents, manager_llm=InstantLLM(),
                  config={"max_concurrent_tasks": clients, "max_queue_size": 100000})
    await serve.start()
    lat = []
    per = max(1, n_tasks // clients)
    # client interleaving: which client submitted each task (in submission order) and how
    # many tasks were in flight at once -- with truly concurrent clients the submissions of
    # different clients alternate and ~clients tasks are in flight (Little's law: mean
    # latency ~= clients / throughput)
    order = []
    state = {"inflight": 0, "max_inflight": 0}

    async def client(ci):
        for j in range(per):
            t0 = time.perf_counter()
            order.append(ci)
            state["inflight"] += 1
            state["max_inflight"] = max(state["max_inflight"], state["inflight"])
            r = await serve.execute_task(Task(description=f"echo {ci}-{j}"))
            state["inflight"] -= 1
            lat.append(time.perf_counter() - t0)
            if not r.success:
                raise RuntimeError(r.error)

    await asyncio.gather(*(client(i) for i in range(clients)))  # warmup pass
    lat.clear()
    order.clear()
    state["max_inflight"] = 0
    t0 = time.perf_counter()
    await asyncio.gather(*(client(i) for i in range(clients)))
    dt = time.perf_counter() - t0
    await serve.stop()
    lat.sort()
    n = len(lat)
    switches = sum(1 for a_, b_ in zip(order, order[1:]) if a_ != b_)
    mean_ms = 1000 * sum(lat) / n
    return {"clients": clients, "tasks": n, "tasks_per_s": round(n / dt, 1),
            "p50_ms": round(1000 * lat[n // 2], 3), "p99_ms": round(1000 * lat[min(n - 1, int(0.99 * n))], 3),
            "mean_ms": round(mean_ms, 3),
            # Little's law check: clients / throughput (ms) vs the measured mean latency
            "littles_law_ms": round(1000 * clients / (n / dt), 3),
            # fraction of consecutive submissions made by different clients (1 client: 0)
            "interleave_frac": round(switches / max(1, len(order) - 1), 3),
            "max_inflight": state["max_inflight"],
            "reference_tasks_per_s": REF.get(clients, (None,))[0], "reference_p50_ms": REF.get(clients, (0, None))[1]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", default="1,8,64")
    ap.add_argument("--tasks", type=int, default=20000)
    ap.add_argument("--repeat", type=int, default=3, help="runs per client count; the median is reported")
    ap.add_argument("--same-box-reference", action="store_true",
                    help="also run the reference's own Serve on this machine (benchmarks/reference_plumbing.py), "
                         "alternating with ours, and report the ratio of the medians")
    a = ap.parse_args()
    ref_mods = None
    if a.same_box_reference:
        from benchmarks import reference_plumbing as rp

        ref_mods = rp._import_reference()
    rows = []
    for c in a.clients.split(","):
        ours, theirs = [], []
        for _ in range(a.repeat):  # interleaved: both see the same machine load
            ours.append(asyncio.run(run(int(c), a.tasks)))
            if ref_mods is not None:
                theirs.append(asyncio.run(rp.run(int(c), a.tasks, ref_mods)))
        runs = sorted(ours, key=lambda r: r["tasks_per_s"])
        med = dict(runs[len(runs) // 2])
        med["runs_tasks_per_s"] = [r["tasks_per_s"] for r in runs]
        if theirs:
            tr = sorted(theirs, key=lambda r: r["tasks_per_s"])
            rm = tr[len(tr) // 2]
            med.update(same_box_reference_tasks_per_s=rm["tasks_per_s"], same_box_reference_p50_ms=rm["p50_ms"],
                       same_box_reference_runs=[r["tasks_per_s"] for r in tr],
                       vs_same_box_reference=round(med["tasks_per_s"] / rm["tasks_per_s"], 2))
        rows.append(med)
    for r in rows:
        print(json.dumps(r), flush=True)
    best = rows[-1]
    print(json.dumps({"metric": "config 1 plumbing: completed agent-tasks/s (CPU, echo agents, fake LLM)",
                      "value": best["tasks_per_s"], "unit": "tasks/s", "n_gpus": 0,
                      "p50_task_latency_ms": best["p50_ms"], "clients": best["clients"],
                      "vs_reference": round(best["tasks_per_s"] / REF[best["clients"]][0], 2)
                      if best["clients"] in REF else None,
                      "vs_same_box_reference": best.get("vs_same_box_reference")}), flush=True)


if __name__ == "__main__":
    main()

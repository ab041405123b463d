#!/usr/bin/env python3
"""The REFERENCE's config-1 plumbing on THIS machine, so benchmarks/plumbing.py can be read
against a same-box number (BASELINE.md §3 quotes an 8-vCPU Xeon from the survey session).

Procedure of BASELINE.md §3, steps 1-5: the reference package (/root/reference/pilott,
Python source, read-only) is copied to a scratch directory and imported with
`cryptography.fernet.Fernet`, `dotenv.load_dotenv` and `litellm.acompletion` stubbed (not
installed here) and an `asyncio.timeout` polyfill (Python 3.10); `Serve(agents=[EchoAgent x
C], manager_llm=<instant fake>, config={"max_concurrent_tasks": C, "max_queue_size": 100000})`;
`Serve._execute_task_with_timeout` wrapped to resolve one future per task; C closed-loop
clients `await s.add_task(Task(...))` and then that task's future. The orchestrator's INFO
log lines go to a null stream (they are formatted, as in the reference, but not printed).

    python benchmarks/reference_plumbing.py [--clients 1,8,64] [--tasks 4096] [--repeat 3]
"""
from __future__ import annotations

import argparse
import asyncio
import io
import json
import logging
import os
import shutil
import sys
import tempfile
import time
import types

REF = "/root/reference/pilott"
_ANALYSIS = json.dumps({"requires_decomposition": False, "complexity": "low", "dependencies": [],
                        "estimated_resources": {"time": "1m", "agents": 1, "tools": []}, "priority": 1})
_EVAL = json.dumps({"success": True, "quality_score": 9, "matches_requirements": True, "requires_retry": False})


def _stubs():
    crypto = types.ModuleType("cryptography")
    fernet = types.ModuleType("cryptography.fernet")

    class Fernet:  # noqa: D401 -- stub: the plumbing path never encrypts
        def __init__(self, key=b""):
            self.key = key

        @staticmethod
        def generate_key():
            return b"0" * 44

        def encrypt(self, b):
            return b

        def decrypt(self, b):
            return b
    fernet.Fernet = Fernet
    crypto.fernet = fernet
    dotenv = types.ModuleType("dotenv")
    dotenv.load_dotenv = lambda *a, **k: None
    litellm = types.ModuleType("litellm")

    async def acompletion(*a, **k):
        raise RuntimeError("no network")
    litellm.acompletion = acompletion
    litellm.set_verbose = False
    sys.modules.update({"cryptography": crypto, "cryptography.fernet": fernet, "dotenv": dotenv, "litellm": litellm})
    if not hasattr(asyncio, "timeout"):  # Python 3.10: the 3.11 context manager
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from pilottai_amd.utils.timeouts import timeout as _timeout

        asyncio.timeout = _timeout


def _import_reference():
    tmp = tempfile.mkdtemp(prefix="refplumb-")
    shutil.copytree(REF, os.path.join(tmp, "pilott"))
    sys.path.insert(0, tmp)
    _stubs()
    from pilott.core.agent import BaseAgent
    from pilott.core.task import Task, TaskResult
    from pilott.pilott import Serve
    return Serve, BaseAgent, Task, TaskResult


class _FakeLLM:
    async def apredict(self, prompt):
        return _EVAL if prompt.lstrip().startswith("Task:") else _ANALYSIS  # result_evaluation vs task_analysis

    async def generate_response(self, messages, tools=None):
        return {"content": _ANALYSIS}


async def run(clients: int, n_tasks: int, mods):
    Serve, BaseAgent, Task, TaskResult = mods

    class EchoAgent(BaseAgent):
        async def _execute_task_internal(self, task):
            return TaskResult(success=True, output=task.description, execution_time=0.0)

    agents = [EchoAgent(role=f"echo-{i}", goal="echo", llm=_FakeLLM()) for i in range(clients)]
    s = Serve(agents=agents, manager_llm=_FakeLLM(), config={"max_concurrent_tasks": clients,
                                                              "max_queue_size": 100000})
    null = logging.StreamHandler(io.StringIO())
    for lg in [s.logger] + [a.logger for a in agents]:
        for h in list(lg.handlers):
            lg.removeHandler(h)
        lg.addHandler(null)
        lg.propagate = False
    futs = {}
    orig = s._execute_task_with_timeout

    async def wrapped(task):
        try:
            r = await orig(task)
        except Exception as e:  # noqa: BLE001
            r = e
        f = futs.pop(task.id, None)
        if f is not None and not f.done():
            f.set_result(r)
        return r
    s._execute_task_with_timeout = wrapped
    await s.start()
    lat = []
    per = max(1, n_tasks // clients)
    loop = asyncio.get_running_loop()

    async def client(ci):
        for j in range(per):
            t0 = time.perf_counter()
            t = Task(description=f"echo {ci}-{j}")
            futs[t.id] = loop.create_future()
            f = futs[t.id]
            await s.add_task(t)
            r = await f
            if isinstance(r, Exception) or not r.success:
                raise RuntimeError(f"reference task failed: {r}")
            lat.append(time.perf_counter() - t0)

    await asyncio.gather(*(client(i) for i in range(clients)))  # warmup pass
    lat.clear()
    t0 = time.perf_counter()
    await asyncio.gather(*(client(i) for i in range(clients)))
    dt = time.perf_counter() - t0
    await s.stop()
    lat.sort()
    n = len(lat)
    return {"clients": clients, "tasks": n, "tasks_per_s": round(n / dt, 1), "p50_ms": round(1000 * lat[n // 2], 3),
            "p99_ms": round(1000 * lat[min(n - 1, int(0.99 * n))], 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", default="1,8,64")
    ap.add_argument("--tasks", type=int, default=4096)
    ap.add_argument("--repeat", type=int, default=3)
    a = ap.parse_args()
    mods = _import_reference()
    for c in a.clients.split(","):
        runs = sorted((asyncio.run(run(int(c), a.tasks, mods)) for _ in range(a.repeat)),
                      key=lambda r: r["tasks_per_s"])
        med = dict(runs[len(runs) // 2], runs_tasks_per_s=[r["tasks_per_s"] for r in runs], impl="reference")
        print(json.dumps(med), flush=True)


if __name__ == "__main__":
    main()

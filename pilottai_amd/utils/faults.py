"""Deterministic fault injection for tests and benchmarks (the
reference has none beyond AsyncMock patches, tests/test_factory.py:126-139).

    inj = FaultInjector()
    inj.drop_heartbeat(agent, seconds=2)     # liveness probe fails -> FaultTolerance CRITICAL
    await inj.crash_agent(agent)             # agent stops; in-flight work fails over
    inj.stall_engine(engine, seconds=5)      # engine loop holds work without progress -> GPUHealthProbe
    inj.fail_llm(llm, times=2)               # next LLM calls raise -> retries / re-delegation
    inj.delay_collectives(0.05)              # every torch.distributed call sleeps first
    inj.restore()                            # undo everything still active

Every fault is recorded in `inj.log`; `restore()` is idempotent.
"""
from __future__ import annotations

import time
from typing import Any, Callable, List, Tuple


class FaultInjector:
    def __init__(self):
        self.log: List[Tuple[float, str, str]] = []
        self._undo: List[Callable[[], None]] = []

    def _rec(self, kind: str, target: Any):
        self.log.append((time.time(), kind, str(getattr(target, "id", target))))

    # -- agents ------------------------------------------------------------
    def drop_heartbeat(self, agent, seconds: float = float("inf")):
        until = time.monotonic() + seconds
        orig = agent.send_heartbeat

        async def hb():
            if time.monotonic() < until:
                raise RuntimeError("injected: heartbeat dropped")
            return await orig()

        agent.send_heartbeat = hb
        self._undo.append(lambda: setattr(agent, "send_heartbeat", orig))
        self._rec("drop_heartbeat", agent)

    async def crash_agent(self, agent):
        self._rec("crash_agent", agent)
        await agent.stop()

    # -- LLM / engine ------------------------------------------------------
    def fail_llm(self, llm, times: int = 1, exc: type = RuntimeError):
        left = {"n": times}
        for name in ("generate_response", "apredict"):
            orig = getattr(llm, name, None)
            if orig is None:
                continue

            def make(orig=orig, name=name):
                async def f(*a, **kw):
                    if left["n"] > 0:
                        left["n"] -= 1
                        raise exc(f"injected: {name} failure")
                    return await orig(*a, **kw)
                return f

            setattr(llm, name, make())
            self._undo.append(lambda orig=orig, name=name: setattr(llm, name, orig))
        self._rec("fail_llm", llm)

    def stall_engine(self, engine, seconds: float):
        """The engine keeps its queued work but completes no step for `seconds`
        (what a wedged kernel or collective looks like from the host)."""
        until = time.monotonic() + seconds
        orig = engine.step

        def step():
            if time.monotonic() < until:
                time.sleep(0.01)
                return False
            return orig()

        engine.step = step
        self._undo.append(lambda: setattr(engine, "step", orig))
        self._rec("stall_engine", engine)

    # -- collectives -------------------------------------------------------
    def delay_collectives(self, seconds: float):
        import torch.distributed as dist

        names = ("all_reduce", "all_gather", "all_gather_into_tensor", "broadcast", "barrier")
        saved = {n: getattr(dist, n) for n in names}

        def wrap(fn):
            def g(*a, **kw):
                time.sleep(seconds)
                return fn(*a, **kw)
            return g

        for n, fn in saved.items():
            setattr(dist, n, wrap(fn))
        self._undo.append(lambda: [setattr(dist, n, fn) for n, fn in saved.items()])
        self._rec("delay_collectives", seconds)

    def restore(self):
        while self._undo:
            self._undo.pop()()

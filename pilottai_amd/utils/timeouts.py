"""Cheap asyncio deadlines for the orchestration hot path.

`asyncio.wait_for` (Python 3.10) wraps the awaited coroutine in a new Task plus a
timer for every call; a task crosses several of them (queue worker, agent,
client wait), which made them the single largest cost of a plumbing-only task
(benchmarks/plumbing.py). `timeout()` arms one timer that cancels the *current*
task instead — the same mechanism as 3.11's `asyncio.timeout` — and converts
that cancellation into `asyncio.TimeoutError`. `None` means no deadline and no
work at all.
"""
from __future__ import annotations

import asyncio
from typing import Any, Awaitable, Optional


class timeout:  # noqa: N801 — mirrors asyncio.timeout
    __slots__ = ("delay", "_handle", "_task", "expired")

    def __init__(self, delay: Optional[float]):
        self.delay = delay
        self._handle = None
        self._task = None
        self.expired = False

    async def __aenter__(self) -> "timeout":
        if self.delay is not None:
            self._task = asyncio.current_task()
            self._handle = asyncio.get_running_loop().call_later(max(0.0, self.delay), self._fire)
        return self

    def _fire(self):
        self.expired = True
        self._task.cancel()

    async def __aexit__(self, et, e, tb) -> bool:
        if self._handle is not None:
            self._handle.cancel()
        if self.expired and et is asyncio.CancelledError:
            if hasattr(self._task, "uncancel"):  # Python >= 3.11 bookkeeping
                self._task.uncancel()
            raise asyncio.TimeoutError from None
        return False


async def with_timeout(aw: Awaitable[Any], delay: Optional[float]) -> Any:
    """`await aw` with a deadline (drop-in for asyncio.wait_for on coroutines)."""
    if delay is None:
        return await aw
    async with timeout(delay):
        return await aw

"""Per-step semantic-memory lookups from many agents, coalesced into one index pass.

The reference's agents consult memory inside their work, one query at a time
(pilott/memory/enhanced_memory.py:93-116 `semantic_search`, called from
docs/examples/pdf_processing/example_agents.py:328-331). With 64 workers on one
GPU that is 64 separate scans of the index per agent step. Here every agent step
`await`s `MemoryLookupBatcher.search(...)`; ONE flush task at a time answers every
request pending when it starts by ONE `EnhancedMemory.search_batch` call, i.e. one
streaming pass of the HIP cosine top-k kernel over the HBM-resident rows
(csrc/ops/similarity.hip, up to 64 queries per pass), on the same GPU as the
engine; requests that arrive while a pass runs wait for the next pass together.
(A flush per event-loop tick queued behind the index lock instead: at 100M rows,
33 ms per pass, that was 190 passes for 384 lookups.) Writes (`store`) are coalesced
the same way.

`stats` reports lookups, passes and the device time of the passes (HIP events around
the kernel on the index's own stream; beside a busy engine that span also contains any
wait for CUs the engine holds, so it bounds the kernel time from above).

Co-scheduling with the engine (`attach_engine`): a 205-GB index pass is a
streaming read that halves the speed of the engine's memory-bound (decode-sized) steps but
costs a compute-bound 2,048-token prefill step only ~6 % (BENCHMARKS.md, config 4). The engine
announces every step it launches (LLMEngine.add_step_listener); with a gate attached, a pass
whose queries are embedded waits until the engine launches a step of at least `gate_tokens`
tokens -- or for at most `gate_max_wait_s` -- and then starts right behind that launch, so the
scan overlaps compute-bound work. `stats` counts the passes that started beside such a step and
the ones the latency cap released. With a gate attached, pending writes and the queries pending
beside them are embedded in one call (one round trip through the engine, `shared_embeds`).
"""
from __future__ import annotations

import asyncio
import logging
import time
from collections import deque
from typing import Any, Dict, List, Optional, Set, Tuple

from .enhanced_memory import EnhancedMemory, MemoryItem

_log = logging.getLogger("pilottai.memory")


class MemoryLookupBatcher:
    LAT_KEEP = 1 << 16
    def __init__(self, memory: EnhancedMemory, max_batch: int = 256, time_device: bool = True,
                 min_batch: int = 1, max_wait_s: float = 0.0):
        """min_batch / max_wait_s: before a pass, wait (in 1 ms sleeps) until `min_batch`
        queries are pending or the oldest has waited `max_wait_s` — more queries share each
        streaming pass over the index (whose cost does not depend on the query count up to
        64), at a bounded latency cost."""
        self.memory = memory
        self.max_batch = max_batch
        self.min_batch = max(1, int(min_batch))
        self.max_wait_s = float(max_wait_s)
        self.time_device = time_device
        self._pending: List[Tuple[str, Optional[Set[str]], int, int, "asyncio.Future", float]] = []
        self._writes: List[Tuple[str, Dict[str, Any], Set[str], int, "asyncio.Future"]] = []
        self._flush_scheduled = False
        self._active = False  # a flush task is running (it drains everything pending)
        if time_device and getattr(getattr(memory.index, "device", None), "type", "cpu") == "cuda":
            memory.index.pass_events = []  # the index records (start, end) around each pass
        self.stats = {"lookups": 0, "passes": 0, "stores": 0, "store_batches": 0, "host_s": 0.0,
                      "device_s": 0.0, "max_batch_seen": 0, "passes_beside_heavy": 0, "passes_capped": 0,
                      "gate_wait_s": 0.0, "shared_embeds": 0,
                      "embed_s": 0.0, "search_s": 0.0, "queued_s": 0.0,
                      "store_failures": 0, "lookup_failures": 0}
        self._gate_tokens = 0
        self._gate_wait = 0.0
        self._heavy: Optional[asyncio.Event] = None
        self._last_heavy = 0.0
        # per-lookup latency (s) for p50 / p99: the most recent LAT_KEEP, plus the running total
        self._lat: deque = deque(maxlen=self.LAT_KEEP)
        self.lat_count = 0
        self._engine = None
        self._listener = None

    # ----------------------------------------------------------------- engine gate
    def attach_engine(self, engine, gate_tokens: int = 1024, max_wait_s: float = 0.03):
        """Co-schedule index passes with the engine's compute-bound steps (module docstring).
        Call from the event loop that runs the lookups."""
        self.detach_engine()
        loop = asyncio.get_running_loop()
        self._heavy = asyncio.Event()
        self._gate_tokens = int(gate_tokens)
        self._gate_wait = float(max_wait_s)

        def on_launch(T: int):
            if T >= self._gate_tokens and not loop.is_closed():
                try:
                    loop.call_soon_threadsafe(self._mark_heavy)
                except RuntimeError:  # the loop closed between the check and the call
                    pass
        engine.add_step_listener(on_launch)
        self._engine, self._listener = engine, on_launch

    def detach_engine(self):
        """Remove the step listener `attach_engine` registered (no-op when none)."""
        if self._engine is not None and self._listener is not None:
            rm = getattr(self._engine, "remove_step_listener", None)
            if rm is not None:
                rm(self._listener)
        self._engine = self._listener = None
        self._heavy = None

    def _mark_heavy(self):
        self._last_heavy = time.perf_counter()
        self._heavy.set()

    async def _await_heavy(self):
        """Return once a heavy step was just launched (within 2 ms), or at the latency cap
        (counted from here: the queries are embedded, only the scan waits)."""
        t0 = time.perf_counter()
        if t0 - self._last_heavy < 0.002:
            self.stats["passes_beside_heavy"] += 1
            return
        self._heavy.clear()
        left = self._gate_wait
        try:
            if left <= 0:
                raise asyncio.TimeoutError
            await asyncio.wait_for(self._heavy.wait(), left)
            self.stats["passes_beside_heavy"] += 1
        except asyncio.TimeoutError:
            self.stats["passes_capped"] += 1
        self.stats["gate_wait_s"] += time.perf_counter() - t0

    def latency_summary(self, since: int = 0) -> dict:
        """p50 / p99 of the lookups after the first `since` (a `lat_count` taken earlier); only
        the most recent LAT_KEEP lookups are kept."""
        n = min(len(self._lat), max(0, self.lat_count - since))
        lat = sorted(list(self._lat)[len(self._lat) - n:]) if n else []
        if not lat:
            return {}
        pick = lambda q: round(1000 * lat[min(len(lat) - 1, int(q * len(lat)))], 2)  # noqa: E731
        return {"lookup_p50_ms": pick(0.5), "lookup_p99_ms": pick(0.99), "lookups": len(lat)}

    # ----------------------------------------------------------------- API
    async def search(self, query: str, limit: int = 5, tags: Optional[Set[str]] = None,
                     min_priority: int = 0) -> List[MemoryItem]:
        fut = asyncio.get_running_loop().create_future()
        self._pending.append((query, tags, int(min_priority), int(limit), fut, time.perf_counter()))
        self._schedule()
        return await fut

    async def store(self, text: str, metadata: Optional[Dict[str, Any]] = None, tags: Optional[Set[str]] = None,
                    priority: int = 0) -> int:
        fut = asyncio.get_running_loop().create_future()
        self._writes.append((text, dict(metadata or {}), set(tags or ()), int(priority), fut))
        self._schedule()
        return await fut

    def lookup_device_seconds(self) -> float:
        """Device time of every finished lookup pass so far (synchronises the events)."""
        evs = getattr(self.memory.index, "pass_events", None) or []
        while evs:
            a, b = evs.pop(0)
            b.synchronize()
            self.stats["device_s"] += a.elapsed_time(b) / 1e3
        return self.stats["device_s"]

    # ----------------------------------------------------------------- batching
    def _schedule(self):
        if not self._flush_scheduled:
            self._flush_scheduled = True
            asyncio.get_running_loop().call_soon(self._start_flush)

    def _start_flush(self):
        self._flush_scheduled = False
        if not self._active:
            asyncio.ensure_future(self._flush())

    async def _flush(self):
        self._active = True
        try:
            while self._writes or self._pending:
                await self._flush_once()
        finally:
            self._active = False

    async def _flush_once(self):
        writes, self._writes = self._writes, []
        pre = None  # (batch, query vectors) embedded together with the writes
        if writes:
            taken = []
            try:
                wvecs = None
                if self._heavy is not None and self._pending and self.min_batch <= 1:
                    # engine embedder: the writes and the pending queries share ONE embedding
                    # round trip through the engine (they were two in sequence)
                    taken, self._pending = self._pending[: self.max_batch], self._pending[self.max_batch:]
                    te = time.perf_counter()
                    allv = await self.memory.embed_queries([w[0] for w in writes] + [b[0] for b in taken])
                    self.stats["embed_s"] += time.perf_counter() - te
                    wvecs, pre = allv[: len(writes)], (taken, allv[len(writes):])
                    self.stats["shared_embeds"] += 1
                rows = await self.memory.store_semantic_batch([w[0] for w in writes], [w[1] for w in writes],
                                                              [w[2] for w in writes], [w[3] for w in writes],
                                                              vecs=wvecs)
                for w, r in zip(writes, rows):
                    if not w[4].done():
                        w[4].set_result(r)
                self.stats["stores"] += len(writes)  # only writes the store accepted
            except Exception as e:  # noqa: BLE001
                self.stats["store_failures"] += len(writes)
                _log.error("memory write of %d item(s) failed: %r", len(writes), e)
                for w in writes:
                    if not w[4].done():
                        w[4].set_exception(e)
                if taken and pre is None:  # the shared embedding failed: the queries go again alone
                    self._pending = taken + self._pending
            self.stats["store_batches"] += 1
        if pre is None and self._pending and self.min_batch > 1 and self.max_wait_s > 0:
            while len(self._pending) < self.min_batch and not self._writes and \
                    time.perf_counter() - self._pending[0][5] < self.max_wait_s:
                await asyncio.sleep(0.001)
            self.stats["coalesce_waits"] = self.stats.get("coalesce_waits", 0) + 1
        if pre is not None or self._pending:
            if pre is not None:
                batch, vecs = pre
            else:
                batch, self._pending = self._pending[: self.max_batch], self._pending[self.max_batch:]
                vecs = None
            limit = max(b[3] for b in batch)
            t0 = time.perf_counter()
            try:
                qs = [b[0] for b in batch]
                if self._heavy is not None:  # embed now, scan beside the next compute-bound step
                    if vecs is None:
                        te = time.perf_counter()
                        vecs = await self.memory.embed_queries(qs)
                        self.stats["embed_s"] += time.perf_counter() - te
                    await self._await_heavy()
                ts = time.perf_counter()
                hits = await self.memory.search_batch(qs, tags=[b[1] for b in batch],
                                                      min_priority=[b[2] for b in batch], limit=limit, vecs=vecs)
                self.stats["search_s"] += time.perf_counter() - ts
                now = time.perf_counter()
                for b, h in zip(batch, hits):
                    self._lat.append(now - b[5])
                    self.lat_count += 1
                    self.stats["queued_s"] += t0 - b[5]
                    if not b[4].done():
                        b[4].set_result(h[: b[3]])
            except Exception as e:  # noqa: BLE001
                self.stats["lookup_failures"] += len(batch)
                for b in batch:
                    if not b[4].done():
                        b[4].set_exception(e)
            self.stats["host_s"] += time.perf_counter() - t0
            self.stats["lookups"] += len(batch)
            self.stats["passes"] += 1
            self.stats["max_batch_seen"] = max(self.stats["max_batch_seen"], len(batch))

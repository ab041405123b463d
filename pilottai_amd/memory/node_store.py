"""One node-wide semantic store over the agent-DP ranks.

The reference has ONE EnhancedMemory that every agent searches and writes back to
(pilott/memory/enhanced_memory.py:60-116; the PDF example's agents share lookups and
write-backs through it, docs/examples/pdf_processing/example_agents.py:151,328-331). With one
process per GPU that store must be node-wide, not one private copy per rank:

* rows are SHARDED: rank r holds the rows whose global id g satisfies g % world == r, at local
  row g // world of its HBM-resident SemanticIndex (100M x 1024 bf16 over 8 GPUs = 12.5M rows,
  25.6 GB per GPU); a write goes to the writer's own shard (its owner), so a vector never
  leaves the GPU that embedded it;
* the small host-side items (text, metadata, tags, priority, expiry) are REPLICATED on every
  rank, so a hit on any shard resolves locally;
* queries are answered in lockstep ROUNDS that every rank's store thread joins: exchange the
  round's counts, replicate the round's writes (then every owner inserts them), all-gather the
  query vectors (RCCL over xGMI on GPUs), scan the local shard once for every rank's queries
  (one streaming pass of the HIP cosine top-k kernel, filters in-kernel), all-gather the
  (global row, score) candidates, and merge each rank's own queries' top-k.
  A write made on rank A in one round is visible to a search from rank B in the same round.

Tags are exchanged as strings (each shard maps them to its own filter bits), expiry is
wall-clock. With world == 1 the store degenerates to a local index (no collectives).
Host metadata travels on a gloo group, the vectors and candidates on the device group
(RCCL; gloo on CPU).
"""
from __future__ import annotations

import asyncio
import threading
import time
from datetime import datetime, timedelta
from typing import Any, Callable, Dict, List, Optional, Sequence, Set, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .embedding import HashingEmbedder
from .enhanced_memory import MemoryItem
from .semantic_index import SemanticIndex

K_MAX = 64  # candidates per shard per query (the kernel's top-k bound)


class NodeSemanticStore:
    def __init__(self, index: SemanticIndex, embedder=None, group=None, cpu_group=None, max_queries: int = 64,
                 fallback_text: Optional[Callable[[int], str]] = None, idle_s: float = 0.002):
        """index: this rank's shard. group: the process group of the agent-DP ranks (device
        collectives: RCCL on GPUs); cpu_group: a gloo group over the same ranks (host metadata;
        defaults to `group` when that is gloo). max_queries: queries per rank per round."""
        self.index = index
        self.embedder = embedder or HashingEmbedder(index.dim)
        self.group = group
        self.cpu_group = cpu_group if cpu_group is not None else group
        on = dist.is_available() and dist.is_initialized()
        self.rank = dist.get_rank(group) if on else 0
        self.world = dist.get_world_size(group) if on else 1
        self.max_queries = int(max_queries)
        self.fallback_text = fallback_text
        self.idle_s = idle_s
        self.items: Dict[int, MemoryItem] = {}  # global row -> item (replicated)
        self._lock = threading.Lock()
        # (vector, min_priority, tags, k, future, loop or None, raw rows wanted)
        self._queries: List[Tuple[np.ndarray, int, Set[str], int, Any, Any, bool]] = []
        self._writes: List[Tuple[np.ndarray, MemoryItem, Any, Any]] = []
        self._stop = False
        self._thread: Optional[threading.Thread] = None
        self._err: Optional[BaseException] = None
        self.stats = {"rounds": 0, "idle_rounds": 0, "lookups": 0, "writes": 0, "round_s": 0.0,
                      "scan_s": 0.0, "max_queries_round": 0}
        self._dev_coll = self._pick_device()

    # ------------------------------------------------------------------ setup
    def _pick_device(self) -> torch.device:
        if self.world > 1 and dist.get_backend(self.group) == "nccl":
            return self.index.device
        return torch.device("cpu")

    @property
    def global_rows(self) -> int:
        return self.index.count  # this shard's rows (the node total: sum over ranks)

    def start(self):
        """Start this rank's round thread (every rank of the group must start one)."""
        if self._thread is None:
            self._thread = threading.Thread(target=self._run, name="pilottai-node-memory", daemon=True)
            self._thread.start()

    def stop(self, timeout: float = 120.0):
        """Leave once every rank has stopped and no rank has pending work."""
        self._stop = True
        if self._thread is not None:
            self._thread.join(timeout)
            self._thread = None

    # ------------------------------------------------------------------ API (asyncio)
    async def embed_queries(self, queries: Sequence[str]) -> np.ndarray:
        return await asyncio.get_running_loop().run_in_executor(None, self._embed, list(queries))

    async def search_batch(self, queries: Sequence[str], tags: Optional[Sequence[Optional[Set[str]]]] = None,
                           min_priority: Optional[Sequence[int]] = None, limit: int = 5,
                           mode: str = "semantic", vecs=None) -> List[List[MemoryItem]]:
        if mode != "semantic":
            raise ValueError("the node-wide store answers semantic searches only")
        Q = len(queries)
        if Q == 0:
            return []
        tags = list(tags) if tags is not None else [None] * Q
        minp = list(min_priority) if min_priority is not None else [0] * Q
        loop = asyncio.get_running_loop()
        if vecs is None:
            vecs = await loop.run_in_executor(None, self._embed, list(queries))
        else:
            vecs = vecs.float().cpu().numpy() if isinstance(vecs, torch.Tensor) else np.asarray(vecs, np.float32)
        futs = []
        with self._lock:
            self._check()
            for i in range(Q):
                f = loop.create_future()
                self._queries.append((vecs[i], int(minp[i]), set(tags[i] or ()), max(1, min(int(limit), K_MAX)),
                                      f, loop, False))
                futs.append(f)
        return list(await asyncio.gather(*futs))

    async def semantic_search(self, query: str, tags: Optional[Set[str]] = None, min_priority: int = 0,
                              limit: int = 5) -> List[MemoryItem]:
        if not query:
            raise ValueError("Query cannot be empty")
        return (await self.search_batch([query], [tags], [min_priority], limit))[0]

    async def store_semantic_batch(self, texts: Sequence[str], metadatas=None, tags=None, priorities=None,
                                   ttl: Optional[float] = None) -> List[int]:
        if any(not t for t in texts):
            raise ValueError("Text cannot be empty")
        items = [MemoryItem(text=t, metadata=(metadatas[i] if metadatas else {}),
                            tags=set(tags[i]) if tags else set(), priority=(priorities[i] if priorities else 0),
                            expires_at=datetime.now() + timedelta(seconds=ttl) if ttl is not None else None)
                 for i, t in enumerate(texts)]
        if not items:
            return []
        loop = asyncio.get_running_loop()
        vecs = await loop.run_in_executor(None, self._embed, [it.text for it in items])
        futs = []
        with self._lock:
            self._check()
            for v, it in zip(vecs, items):
                f = loop.create_future()
                self._writes.append((v, it, f, loop))
                futs.append(f)
        return list(await asyncio.gather(*futs))

    async def store_semantic(self, text: str, metadata: Optional[Dict[str, Any]] = None,
                             tags: Optional[Set[str]] = None, priority: int = 0, ttl: Optional[float] = None) -> int:
        return (await self.store_semantic_batch([text], [metadata or {}], [set(tags or ())], [priority], ttl))[0]

    def __len__(self) -> int:
        return len(self.items)

    def _check(self):
        if self._err is not None:
            raise RuntimeError(f"node memory store failed: {self._err!r}")
        if self._thread is None:
            raise RuntimeError("node memory store not started (call start() on every rank)")

    def _embed(self, texts: List[str]) -> np.ndarray:
        v = self.embedder(texts)
        v = v.float().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v, dtype=np.float32)
        return v.reshape(len(texts), self.index.dim)

    # ------------------------------------------------------------------ rounds (store thread)
    def _run(self):
        import contextlib

        ctx = contextlib.nullcontext()
        if self.index.device.type == "cuda":
            torch.cuda.set_device(self.index.device)
            # the round's copies and RCCL collectives are ordered behind this stream only, not
            # behind the engine's work on the default stream (a round must not wait for a step)
            ctx = torch.cuda.stream(torch.cuda.Stream(device=self.index.device, priority=-1))
        with ctx:
            self._loop()

    def _loop(self):
        try:
            idle = 0
            while True:
                busy, done = self._round()
                if done:
                    break
                if busy:
                    idle = 0
                else:
                    idle += 1
                    self.stats["idle_rounds"] += 1
                    time.sleep(min(self.idle_s * idle, 0.005))
        except BaseException as e:  # noqa: BLE001 -- fail every waiter loudly
            self._err = e
            with self._lock:
                pend = [(q[4], q[5]) for q in self._queries] + [(w[2], w[3]) for w in self._writes]
                self._queries, self._writes = [], []
            for f, loop in pend:
                _deliver(f, loop, RuntimeError(f"node memory store failed: {e!r}"), exc=True)

    def _gather_obj(self, obj) -> list:
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        dist.all_gather_object(out, obj, group=self.cpu_group)
        return out

    def _gather_tensor(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *t.shape] on the collective device."""
        if self.world == 1:
            return t.unsqueeze(0)
        t = t.to(self._dev_coll).contiguous()
        if self._dev_coll.type == "cpu":
            parts = [torch.empty_like(t) for _ in range(self.world)]
            dist.all_gather(parts, t, group=self.group)
            return torch.stack(parts)
        out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t, group=self.group)
        return out

    def _round(self) -> Tuple[bool, bool]:
        """One lockstep round; returns (any work anywhere, every rank stopped and idle)."""
        with self._lock:
            qs, self._queries = self._queries[:self.max_queries], self._queries[self.max_queries:]
            ws, self._writes = self._writes, []
        hdr = self._gather_obj((len(qs), len(ws), bool(self._stop)))
        nq = [h[0] for h in hdr]
        nw = [h[1] for h in hdr]
        if sum(nq) == 0 and sum(nw) == 0:
            return False, all(h[2] for h in hdr)
        t0 = time.perf_counter()
        self.stats["rounds"] += 1
        # ---- writes: the owner (the writer's rank) inserts the vectors into its shard; every
        # rank learns (global row, item) in rank order
        recs = []
        if ws:
            rows = self.index.add(np.stack([w[0] for w in ws]), [w[1].priority for w in ws],
                                  [w[1].tags for w in ws],
                                  [w[1].expires_at.timestamp() if w[1].expires_at else None for w in ws])
            recs = [(r * self.world + self.rank, w[1].model_dump(mode="json")) for r, w in zip(rows, ws)]
        if sum(nw):
            for lst in self._gather_obj(recs):
                for g, d in lst:
                    self.items[int(g)] = MemoryItem(**d)
            for (g, _), w in zip(recs, ws):
                _deliver(w[2], w[3], int(g))
            self.stats["writes"] += len(ws)
        if sum(nq) == 0:
            self.stats["round_s"] += time.perf_counter() - t0
            return True, False
        # ---- queries: every rank's vectors, filters and k
        QM = max(nq)
        dim = self.index.dim
        qv = torch.zeros(QM, dim, dtype=torch.float32)
        for i, q in enumerate(qs):
            qv[i] = torch.from_numpy(np.ascontiguousarray(q[0], dtype=np.float32))
        allv = self._gather_tensor(qv)  # [W, QM, dim]
        meta = self._gather_obj([(q[1], sorted(q[2]), q[3]) for q in qs])
        kmax = max(m[2] for lst in meta for m in lst)
        flat_v, flat_p, flat_t, owners = [], [], [], []
        for r in range(self.world):
            for i, (mp, tg, _k) in enumerate(meta[r]):
                flat_v.append(allv[r, i])
                flat_p.append(mp)
                flat_t.append(tuple(tg))
                owners.append((r, i))
        ts = time.perf_counter()
        hits = self.index.search(torch.stack(flat_v).cpu().numpy(), kmax, flat_p, flat_t) if self.index.count else \
            [[] for _ in flat_v]
        self.stats["scan_s"] += time.perf_counter() - ts
        cand = torch.full((self.world, QM, kmax, 2), -1.0, dtype=torch.float64)
        for (r, i), lst in zip(owners, hits):
            for j, (row, sc) in enumerate(lst[:kmax]):
                cand[r, i, j, 0] = row * self.world + self.rank
                cand[r, i, j, 1] = sc
        allc = self._gather_tensor(cand).cpu()  # [W shards, W ranks, QM, kmax, 2]
        for i, q in enumerate(qs):
            c = allc[:, self.rank, i].reshape(-1, 2)
            c = c[c[:, 0] >= 0]
            order = torch.argsort(c[:, 1], descending=True)[: q[3]]
            rows = [(int(c[j, 0]), float(c[j, 1])) for j in order.tolist()]
            _deliver(q[4], q[5], rows if q[6] else self._items_for(rows))
        self.stats["lookups"] += len(qs)
        self.stats["max_queries_round"] = max(self.stats["max_queries_round"], sum(nq))
        self.stats["round_s"] += time.perf_counter() - t0
        return True, False

    def _items_for(self, rows: List[Tuple[int, float]]) -> List[MemoryItem]:
        """Replicated items of merged hits, best first, then ordered like EnhancedMemory
        (-priority, timestamp); bulk-loaded rows without an item use fallback_text."""
        res = []
        for g, _ in rows:
            it = self.items.get(g)
            if it is not None:
                if not it.is_expired():
                    res.append(it)
            elif self.fallback_text is not None:
                res.append(MemoryItem(text=self.fallback_text(g)))
        res.sort(key=lambda x: (-x.priority, x.timestamp))
        return res

    # ------------------------------------------------------------------ raw candidates (tests, tools)
    def search_rows_blocking(self, vecs: np.ndarray, k: int, min_priority: Sequence[int],
                             tags: Sequence[Sequence[str]], timeout: float = 120.0) -> List[List[Tuple[int, float]]]:
        """From any thread: enqueue raw query vectors for the next round and wait for their
        merged [(global row, score), ...] lists (the store thread must be running)."""
        import concurrent.futures as cf

        futs = [cf.Future() for _ in range(len(vecs))]
        with self._lock:
            self._check()
            for i, v in enumerate(vecs):
                self._queries.append((np.asarray(v, np.float32), int(min_priority[i]), set(tags[i] or ()),
                                      max(1, min(int(k), K_MAX)), futs[i], None, True))
        return [f.result(timeout) for f in futs]

    def store_rows_blocking(self, vecs: np.ndarray, items: Sequence[MemoryItem], timeout: float = 120.0) -> List[int]:
        """From any thread: write raw vectors with their items (owner: this rank); returns the
        global rows once the round that replicated them has run."""
        import concurrent.futures as cf

        futs = [cf.Future() for _ in range(len(vecs))]
        with self._lock:
            self._check()
            for v, it, f in zip(vecs, items, futs):
                self._writes.append((np.asarray(v, np.float32), it, f, None))
        return [f.result(timeout) for f in futs]


def _deliver(fut, loop, val, exc: bool = False):
    """Resolve an asyncio future from the store thread (loop given) or a concurrent one."""
    if loop is None:
        if not fut.done():
            fut.set_exception(val) if exc else fut.set_result(val)
    else:
        loop.call_soon_threadsafe(_set_exc if exc else _set_res, fut, val)


def _set_res(fut, val):
    if not fut.done():
        fut.set_result(val)


def _set_exc(fut, e):
    if not fut.done():
        fut.set_exception(e)

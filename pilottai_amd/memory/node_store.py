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
Host metadata travels through the node's shared-memory all-gather (parallel/host_gather.py;
gloo only when the ranks span hosts), the vectors and candidates on the device group (RCCL over
xGMI; on CPU the shared-memory plane too).
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
        # hits / remote_hits: returned rows, and those held by another rank's shard
        self.stats = {"rounds": 0, "idle_rounds": 0, "lookups": 0, "writes": 0, "round_s": 0.0,
                      "scan_s": 0.0, "max_queries_round": 0, "hits": 0, "remote_hits": 0}
        self._dev_coll = self._pick_device()
        # host payloads (counts, filters, tags, items; on CPU also vectors and candidates) go
        # through a shared-memory all-gather between the node's ranks (parallel/host_gather.py)
        from pilottai_amd.parallel.host_gather import HostGather

        self._host = HostGather(self.cpu_group) if self.world > 1 else None

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
            vecs = _as_rows(vecs, Q, self.index.dim)
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
                                   ttl: Optional[float] = None, vecs=None) -> List[int]:
        """`vecs`: the texts' embeddings when the caller already has them (embed_queries), the
        same contract as EnhancedMemory.store_semantic_batch (memory/store_protocol.py)."""
        if any(not t for t in texts):
            raise ValueError("Text cannot be empty")
        items = [MemoryItem(text=t, metadata=(metadatas[i] if metadatas else {}),
                            tags=set(tags[i]) if tags else set(), priority=(priorities[i] if priorities else 0),
                            expires_at=datetime.now() + timedelta(seconds=ttl) if ttl is not None else None)
                 for i, t in enumerate(texts)]
        if not items:
            return []
        loop = asyncio.get_running_loop()
        if vecs is None:
            vecs = await loop.run_in_executor(None, self._embed, [it.text for it in items])
        else:
            vecs = _as_rows(vecs, len(items), self.index.dim)
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
        return self._host.gather_obj(obj)

    def _gather_host(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *t.shape] of a host tensor through the host plane."""
        if self.world == 1:
            return t.unsqueeze(0)
        return torch.from_numpy(self._host.gather_array(t.numpy()))

    def _gather_tensor(self, t: torch.Tensor, device: Optional[torch.device] = None, group=None) -> torch.Tensor:
        """[world, *t.shape] on `device` (default: the collective device of `self.group`)."""
        if self.world == 1:
            return t.unsqueeze(0)
        dev = self._dev_coll if device is None else device
        grp = self.group if group is None else group
        t = t.to(dev).contiguous()
        if dev.type == "cpu" and self._host is not None and self._host.transport == "shm":
            return self._gather_host(t)
        if dev.type == "cpu":
            parts = [torch.empty_like(t) for _ in range(self.world)]
            dist.all_gather(parts, t, group=grp)
            return torch.stack(parts)
        out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t, group=grp)
        return out

    def _exchange(self, t: torch.Tensor) -> torch.Tensor:
        """All-to-all of [world, ...] (row q goes to rank q): RCCL on the device group, the
        shared-memory plane on CPU."""
        if self.world == 1:
            return t.clone()
        t = t.contiguous()
        if t.device.type == "cpu" and self._host is not None and self._host.transport == "shm":
            return torch.from_numpy(self._host.all_to_all_array(t.numpy()))
        out = torch.empty_like(t)
        dist.all_to_all_single(out, t, group=self.group)
        return out

    def _round(self) -> Tuple[bool, bool]:
        """One lockstep round; returns (any work anywhere, every rank stopped and idle).

        Collectives per round: an idle round is ONE 4-int all-gather on the
        host plane (no pickling); a busy round adds the query vectors (device group,
        device-resident), a [QM, 3] int meta tensor, the candidates as (global row, score)
        tensors packed on the device, and object gathers only for what has no fixed shape:
        the written items (rounds with writes) and query tag strings (rounds with tags). The
        host payloads travel through the node's shared-memory plane (HostGather), microseconds
        per all-gather instead of a gloo loopback-TCP round trip."""
        with self._lock:
            qs, self._queries = self._queries[:self.max_queries], self._queries[self.max_queries:]
            ws, self._writes = self._writes, []
        any_tags = any(q[2] for q in qs)
        hdr = torch.tensor([len(qs), len(ws), int(bool(self._stop)), int(any_tags)], dtype=torch.int64)
        hdr = self._gather_host(hdr)
        nq = hdr[:, 0].tolist()
        nw = hdr[:, 1].tolist()
        if sum(nq) == 0 and sum(nw) == 0:
            return False, bool(hdr[:, 2].all())
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
        # ---- queries: every rank's vectors (one host->device copy, then device-resident),
        # filters and k
        QM = max(nq)
        W = self.world
        dim = self.index.dim
        qv = torch.zeros(QM, dim, dtype=torch.float32)
        if qs:
            qv[:len(qs)] = torch.from_numpy(np.stack([q[0] for q in qs]).astype(np.float32, copy=False))
        allv = self._gather_tensor(qv.to(self._dev_coll))  # [W, QM, dim]
        meta = torch.zeros(QM, 2, dtype=torch.int64)
        if qs:
            meta[:len(qs)] = torch.from_numpy(np.array([(q[1], q[3]) for q in qs], dtype=np.int64))
        allm = self._gather_host(meta)  # [W, QM, 2]
        kmax = int(allm[:, :, 1].max())
        alltags = self._gather_obj([sorted(q[2]) for q in qs]) if bool(hdr[:, 3].any()) else [[]] * W
        valid = torch.arange(QM).unsqueeze(0) < torch.tensor(nq).unsqueeze(1)  # [W, QM]
        vflat = valid.flatten()
        flat_v = allv.reshape(W * QM, dim)[vflat.to(allv.device)]
        flat_p = allm[:, :, 0].flatten()[vflat]
        flat_t = [tuple(alltags[r][i]) if alltags[r] else () for r in range(W) for i in range(nq[r])]
        ts = time.perf_counter()
        n_flat = int(vflat.sum())
        cand_s = torch.full((W * QM, kmax), float("-inf"), dtype=torch.float32, device=self._dev_coll)
        cand_r = torch.full((W * QM, kmax), -1, dtype=torch.int64, device=self._dev_coll)
        if self.index.count:
            qmasks, exact = self.index.query_masks(flat_t)
            pos = vflat.nonzero().flatten().to(self._dev_coll)
            if all(exact):  # the common case: the kernel's tensors go straight into the gather
                s_, r_ = self.index.search_tensors(flat_v, kmax, flat_p, qmasks)
                if s_.is_cuda:  # the pass ran on the index's stream: order this round's stream behind it
                    torch.cuda.current_stream(s_.device).wait_stream(self.index._stream)
                s_, r_ = s_.to(self._dev_coll), r_.to(self._dev_coll).long()
            else:  # overflow tags re-checked on the host (SemanticIndex.search)
                hits = self.index.search(flat_v, kmax, flat_p.tolist(), flat_t)
                s_ = torch.full((n_flat, kmax), float("-inf"), dtype=torch.float32)
                r_ = torch.full((n_flat, kmax), -1, dtype=torch.int64)
                for i, lst in enumerate(hits):
                    if lst:
                        a = np.asarray(lst, dtype=np.float64)
                        r_[i, :len(lst)] = torch.from_numpy(a[:, 0].astype(np.int64))
                        s_[i, :len(lst)] = torch.from_numpy(a[:, 1].astype(np.float32))
                s_, r_ = s_.to(self._dev_coll), r_.to(self._dev_coll)
            hit = r_ >= 0
            cand_r[pos] = torch.where(hit, r_ * W + self.rank, r_)
            cand_s[pos] = torch.where(hit, s_.float(), torch.full_like(s_, float("-inf"), dtype=torch.float32))
        self.stats["scan_s"] += time.perf_counter() - ts
        # all-to-all: shard q's candidates for THIS rank's queries, [W shards, QM, kmax] -- each
        # rank receives only its own queries' rows (an all-gather would move W times the bytes)
        alls = self._exchange(cand_s.view(W, QM, kmax))
        allr = self._exchange(cand_r.view(W, QM, kmax))
        # merge this rank's queries: [QM, W * kmax] sorted by score on the collective device
        ms = alls.permute(1, 0, 2).reshape(QM, W * kmax)
        mr = allr.permute(1, 0, 2).reshape(QM, W * kmax)
        top_s, order = torch.topk(ms[:len(qs)], min(kmax, W * kmax), dim=1, sorted=True)
        # misses score -inf, so each row's hits lead it: one host copy, then plain slicing
        ms = top_s.cpu().numpy()
        mr = torch.gather(mr[:len(qs)], 1, order).cpu().numpy()
        nhit = (mr >= 0).sum(axis=1)
        for i, q in enumerate(qs):
            got = mr[i, :min(int(nhit[i]), q[3])]
            self.stats["hits"] += len(got)
            self.stats["remote_hits"] += int((got % W != self.rank).sum())
        for i, q in enumerate(qs):
            m = min(int(nhit[i]), q[3])
            rows = list(zip(mr[i, :m].tolist(), ms[i, :m].tolist()))
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


def _as_rows(vecs, n: int, dim: int) -> np.ndarray:
    """Caller-provided embeddings (array or tensor, any device) as [n, dim] fp32 host rows."""
    if isinstance(vecs, torch.Tensor):
        vecs = vecs.detach().float().cpu().numpy()
    v = np.asarray(vecs, dtype=np.float32).reshape(n, dim)
    return v


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

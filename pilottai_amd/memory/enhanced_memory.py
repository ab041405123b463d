"""EnhancedMemory — semantic / task / interaction / pattern stores
(reference: pilott/memory/enhanced_memory.py:9-292).

`store_semantic` embeds the text (memory/embedding.py) into an HBM-resident
SemanticIndex; `semantic_search` ranks by cosine similarity with the
reference's filters (min_priority, tag intersection, TTL expiry) evaluated inside
the HIP top-k kernel, then orders the `limit` hits by (-priority, timestamp) like
the reference. `mode="substring"` keeps the reference's exact case-insensitive
substring semantics. An empty store returns [] (the reference raised, App. A
#26); eviction never corrupts the indices (ring-buffer row ids).

`search_batch` answers many queries in ONE kernel pass — the engine-side batching
agents use when each of 64 workers consults memory on every step.
"""
from __future__ import annotations

import asyncio
from collections import deque
from datetime import datetime, timedelta
from typing import Any, Callable, Deque, Dict, List, Optional, Sequence, Set

from pydantic import BaseModel, ConfigDict, Field

from .embedding import HashingEmbedder
from .semantic_index import SemanticIndex


class MemoryItem(BaseModel):
    model_config = ConfigDict(arbitrary_types_allowed=True)
    text: str
    metadata: Dict[str, Any] = Field(default_factory=dict)
    timestamp: datetime = Field(default_factory=datetime.now)
    tags: Set[str] = Field(default_factory=set)
    priority: int = Field(default=0, ge=0)
    expires_at: Optional[datetime] = None
    version: int = 1

    def is_expired(self) -> bool:
        return self.expires_at is not None and datetime.now() > self.expires_at


class EnhancedMemory:
    def __init__(self, max_size: int = 10000, cleanup_interval: float = 3600, embedder=None,
                 index: Optional[SemanticIndex] = None, dim: int = 1024, device=None,
                 fallback_text: Optional[Callable[[int], str]] = None, storage: str = "bf16"):
        """storage: the index's row format when it is created here ("bf16", or "q16": 16-bit
        fixed point with the two-stage exact scan, memory/semantic_index.py)."""
        self.max_size = max_size
        self.cleanup_interval = cleanup_interval
        self.embedder = embedder or HashingEmbedder(dim)
        self.index = index or SemanticIndex(dim=getattr(self.embedder, "dim", dim),
                                            capacity=min(max_size, 1 << 16) if max_size else 1 << 16,
                                            device=device, growable=True, max_capacity=max_size,
                                            storage=storage)
        self._items: Dict[int, MemoryItem] = {}
        self._task_history: Dict[str, Deque[Dict[str, Any]]] = {}
        self._agent_interactions: Dict[str, Dict[str, Any]] = {}
        self._pattern_store: Dict[str, Dict[str, Any]] = {}
        self.max_task_history = 1000
        self.last_cleanup = datetime.now()
        self._semantic_lock = asyncio.Lock()
        self._task_lock = asyncio.Lock()
        self._interaction_lock = asyncio.Lock()
        self._pattern_lock = asyncio.Lock()
        self._cleanup_task: Optional[asyncio.Task] = None
        # rows bulk-loaded on the device (SemanticIndex.add_device) have no host-side
        # MemoryItem; with fallback_text their hits are returned as MemoryItem(text=...)
        self.fallback_text = fallback_text

    async def start(self):
        if self._cleanup_task is None:
            self._cleanup_task = asyncio.create_task(self._periodic_cleanup())

    async def stop(self):
        if self._cleanup_task:
            self._cleanup_task.cancel()
            try:
                await self._cleanup_task
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
            self._cleanup_task = None

    # ---------------------------------------------------------------- semantic
    async def store_semantic(self, text: str, metadata: Optional[Dict[str, Any]] = None,
                             tags: Optional[Set[str]] = None, priority: int = 0, ttl: Optional[float] = None) -> int:
        if not text:
            raise ValueError("Text cannot be empty")
        items = [MemoryItem(text=text, metadata=metadata or {}, tags=set(tags or ()), priority=priority,
                            expires_at=datetime.now() + timedelta(seconds=ttl) if ttl is not None else None)]
        async with self._semantic_lock:
            if getattr(self.index.device, "type", "cpu") == "cuda":
                return (await asyncio.get_running_loop().run_in_executor(None, self._store_items, items))[0]
            return self._store_items(items)[0]

    async def store_semantic_batch(self, texts: Sequence[str], metadatas=None, tags=None, priorities=None,
                                   ttl: Optional[float] = None, vecs=None) -> List[int]:
        """`vecs`: the texts' embeddings when the caller already has them (embed_queries)."""
        n = len(texts)
        items = [MemoryItem(text=t, metadata=(metadatas[i] if metadatas else {}),
                            tags=set(tags[i]) if tags else set(), priority=(priorities[i] if priorities else 0),
                            expires_at=datetime.now() + timedelta(seconds=ttl) if ttl is not None else None)
                 for i, t in enumerate(texts)]
        if any(not t for t in texts):
            raise ValueError("Text cannot be empty")
        async with self._semantic_lock:
            if not n:
                return []
            if getattr(self.index.device, "type", "cpu") == "cuda":
                # the embedder may be the serving engine itself (EngineEmbedder), and the row
                # writes are host->device copies: both in a worker thread, so the event loop
                # keeps serving the agents meanwhile
                return await asyncio.get_running_loop().run_in_executor(None, self._store_items, items, vecs)
            return self._store_items(items, vecs)

    def _store_items(self, items: List[MemoryItem], vecs=None) -> List[int]:
        if vecs is None:
            vecs = self.embedder([it.text for it in items])
        rows = self.index.add(vecs, [it.priority for it in items], [it.tags for it in items],
                              [it.expires_at.timestamp() if it.expires_at else None for it in items])
        for r, it in zip(rows, items):
            self._items[r] = it  # overwriting a ring slot evicts the old item
        return rows

    async def semantic_search(self, query: str, tags: Optional[Set[str]] = None, min_priority: int = 0,
                              limit: int = 5, mode: str = "semantic") -> List[MemoryItem]:
        if not query:
            raise ValueError("Query cannot be empty")
        res = await self.search_batch([query], tags=[tags], min_priority=[min_priority], limit=limit, mode=mode)
        return res[0]

    async def embed_queries(self, queries: Sequence[str]):
        """The query embeddings (a worker thread on the GPU: the embedder may be the serving
        engine); pass them to search_batch(vecs=...) to run the index pass later."""
        if getattr(self.index.device, "type", "cpu") == "cuda":
            return await asyncio.get_running_loop().run_in_executor(None, self.embedder, list(queries))
        return self.embedder(list(queries))

    async def search_batch(self, queries: Sequence[str], tags: Optional[Sequence[Optional[Set[str]]]] = None,
                           min_priority: Optional[Sequence[int]] = None, limit: int = 5,
                           mode: str = "semantic", vecs=None) -> List[List[MemoryItem]]:
        """`vecs`: the queries' embeddings from embed_queries (skips embedding here)."""
        Q = len(queries)
        tags = list(tags) if tags is not None else [None] * Q
        minp = list(min_priority) if min_priority is not None else [0] * Q
        async with self._semantic_lock:
            if mode == "substring":
                return [self._substring(q, t, p, limit) for q, t, p in zip(queries, tags, minp)]

            def run():
                v = self.embedder(list(queries)) if vecs is None else vecs
                return self.index.search(v, limit, minp, [t or () for t in tags])

            if getattr(self.index.device, "type", "cpu") == "cuda":
                # embed + one kernel pass + wait in a worker thread: the event loop (all
                # the agents) keeps running while the pass is on the GPU
                hits = await asyncio.get_running_loop().run_in_executor(None, run)
            else:
                hits = run()
        out = []
        for lst in hits:
            items = [self._items[r] for r, _ in lst if r in self._items and not self._items[r].is_expired()]
            if self.fallback_text is not None:
                items += [MemoryItem(text=self.fallback_text(r)) for r, _ in lst if r not in self._items]
            out.append(sorted(items, key=lambda x: (-x.priority, x.timestamp)))
        return out

    def _substring(self, query: str, tags, min_priority: int, limit: int) -> List[MemoryItem]:
        ql = query.lower()
        tags = set(tags or ())
        matches = []
        for r in sorted(self._items):
            it = self._items[r]
            if it.priority < min_priority or it.is_expired() or not tags <= it.tags:
                continue
            if ql in it.text.lower():
                matches.append(it)
                if len(matches) >= limit:
                    break
        return sorted(matches, key=lambda x: (-x.priority, x.timestamp))

    # ---------------------------------------------------------------- tasks / interactions
    async def store_task(self, task_id: str, task_data: Dict[str, Any]) -> None:
        if not task_id or not task_data:
            raise ValueError("Task ID and data required")
        async with self._task_lock:
            h = self._task_history.setdefault(task_id, deque(maxlen=self.max_task_history))
            h.append({"data": dict(task_data), "timestamp": datetime.now(), "version": len(h) + 1})

    async def store_interaction(self, agent_id: str, interaction_type: str, data: Dict[str, Any]) -> None:
        if not agent_id or not interaction_type or not data:
            raise ValueError("Agent ID, interaction type, and data required")
        async with self._interaction_lock:
            d = self._agent_interactions.setdefault(agent_id, {})
            ts = datetime.now()
            key = ts.isoformat()
            while key in d:  # same-microsecond interactions must not overwrite each other
                ts = ts + timedelta(microseconds=1)
                key = ts.isoformat()
            d[key] = {"type": interaction_type, "data": dict(data), "timestamp": ts, "version": len(d) + 1}

    async def get_interactions(self, agent_id: str, interaction_type: Optional[str] = None) -> List[Dict[str, Any]]:
        async with self._interaction_lock:
            vals = list(self._agent_interactions.get(agent_id, {}).values())
        return [v for v in vals if interaction_type is None or v["type"] == interaction_type]

    async def store_pattern(self, name: str, data: Any, ttl: Optional[float] = None) -> None:
        if not name:
            raise ValueError("Pattern name required")
        async with self._pattern_lock:
            self._pattern_store[name] = {"data": data, "timestamp": datetime.now(),
                                         "expires_at": datetime.now() + timedelta(seconds=ttl) if ttl else None}

    async def get_pattern(self, name: str) -> Optional[Any]:
        if not name:
            raise ValueError("Pattern name required")
        async with self._pattern_lock:
            p = self._pattern_store.get(name)
            if p is None:
                return None
            if p["expires_at"] and datetime.now() > p["expires_at"]:
                del self._pattern_store[name]
                return None
            return p["data"]

    async def get_recent_tasks(self, limit: int = 10, task_type: Optional[str] = None) -> List[Dict[str, Any]]:
        if limit < 1:
            raise ValueError("Limit must be positive")
        async with self._task_lock:
            allt = [e for h in self._task_history.values() for e in h
                    if task_type is None or e["data"].get("type") == task_type]
        return sorted(allt, key=lambda x: x["timestamp"], reverse=True)[:limit]

    # ---------------------------------------------------------------- maintenance
    async def _periodic_cleanup(self):
        while True:
            await asyncio.sleep(self.cleanup_interval)
            try:
                await self.cleanup()
            except Exception:  # noqa: BLE001
                pass

    async def cleanup(self):
        async with self._semantic_lock, self._pattern_lock:
            dead = [r for r, it in self._items.items() if it.is_expired()]
            if dead:
                self.index.delete(dead)
                for r in dead:
                    del self._items[r]
            now = datetime.now()
            for name in [n for n, p in self._pattern_store.items() if p["expires_at"] and now > p["expires_at"]]:
                del self._pattern_store[name]
        self.last_cleanup = datetime.now()

    def clear(self) -> None:
        if self._items:
            self.index.delete(list(self._items))
        self._items.clear()
        self._task_history.clear()
        self._agent_interactions.clear()
        self._pattern_store.clear()

    def __len__(self) -> int:
        return len(self._items)

    # ---------------------------------------------------------------- checkpoint (App. D MemoryItem format)
    def to_dict(self) -> Dict[str, Any]:
        # each semantic item records its index row: with the index saved beside the JSON
        # (SemanticIndex.save, utils/checkpoint.py) the restore re-attaches it without re-embedding
        return {"semantic": [dict(self._items[r].model_dump(mode="json"), row=r) for r in sorted(self._items)],
                "tasks": {k: [dict(e, timestamp=e["timestamp"].isoformat()) for e in v]
                          for k, v in self._task_history.items()},
                "patterns": {k: {"data": v["data"], "timestamp": v["timestamp"].isoformat(),
                                 "expires_at": v["expires_at"].isoformat() if v["expires_at"] else None}
                             for k, v in self._pattern_store.items()}}

    async def load_dict(self, d: Dict[str, Any], index_restored: bool = False):
        """Restore from to_dict() form. `index_restored`: self.index was loaded from the same
        checkpoint (SemanticIndex.load), so an item that recorded its row is re-attached to that
        row as is; only items without a stored row are embedded again."""
        items, rows = [], []
        for x in d.get("semantic", []):
            x = dict(x)
            r = x.pop("row", None)
            items.append(MemoryItem(**x))
            rows.append(r if index_restored and r is not None and 0 <= int(r) < self.index.count else None)
        if items:
            async with self._semantic_lock:
                for r, it in zip(rows, items):
                    if r is not None:
                        self._items[int(r)] = it
                fresh = [it for r, it in zip(rows, items) if r is None]
                if fresh:
                    self._store_items(fresh)
        for k, v in d.get("tasks", {}).items():
            h = self._task_history.setdefault(k, deque(maxlen=self.max_task_history))
            for e in v:
                h.append(dict(e, timestamp=datetime.fromisoformat(e["timestamp"])))
        for k, v in d.get("patterns", {}).items():
            self._pattern_store[k] = {"data": v["data"], "timestamp": datetime.fromisoformat(v["timestamp"]),
                                      "expires_at": datetime.fromisoformat(v["expires_at"]) if v["expires_at"] else None}

"""Orchestrator memory (reference: pilott/core/memory.py:9-134).

Bounded history of MemoryEntry {timestamp, data, tags, priority} with a tag index,
time-range search, context and pattern maps. Entries carry a monotonically
increasing sequence number and the tag index stores sequence numbers, so the
index never points at the wrong entry after the bounded deque evicts old ones
(the reference's positional index went stale, App. A #25), and
`retrieve_by_timerange` really uses binary search over the time-ordered history.
"""
from __future__ import annotations

import asyncio
import bisect
from collections import deque
from datetime import datetime
from typing import Any, Deque, Dict, List, Optional

from pydantic import BaseModel, Field


class MemoryEntry(BaseModel):
    timestamp: datetime
    data: Dict[str, Any]
    tags: List[str] = Field(default_factory=list)
    priority: int = 1


class Memory:
    MAX_HISTORY_SIZE = 1000
    MAX_CONTEXT_SIZE = 100
    MAX_PATTERNS_SIZE = 50

    def __init__(self, max_history: int = MAX_HISTORY_SIZE):
        self.MAX_HISTORY_SIZE = max_history
        self.history: Deque[MemoryEntry] = deque()
        self._seqs: Deque[int] = deque()
        self._next_seq = 0
        self.context: Dict[str, Any] = {}
        self.patterns: Dict[str, Any] = {}
        self.tag_index: Dict[str, Deque[int]] = {}
        self.memory_lock = asyncio.Lock()

    # -- internals -------------------------------------------------------------
    def _entry(self, seq: int) -> Optional[MemoryEntry]:
        if not self._seqs:
            return None
        i = seq - self._seqs[0]
        if 0 <= i < len(self.history):
            return self.history[i]
        return None

    def _evict(self):
        old = self.history.popleft()
        seq = self._seqs.popleft()
        for t in old.tags:
            idx = self.tag_index.get(t)
            while idx and idx[0] <= seq:
                idx.popleft()
            if idx is not None and not idx:
                del self.tag_index[t]

    # -- API --------------------------------------------------------------------
    async def store(self, data: Dict[str, Any], tags: Optional[List[str]] = None, priority: int = 1):
        async with self.memory_lock:
            self.store_nowait(data, tags, priority)

    def store_nowait(self, data: Dict[str, Any], tags: Optional[List[str]] = None, priority: int = 1,
                     timestamp: Optional[datetime] = None):
        entry = MemoryEntry(timestamp=timestamp or datetime.now(), data=data, tags=list(tags or []),
                            priority=priority)
        if self.history and entry.timestamp < self.history[-1].timestamp:
            entry.timestamp = self.history[-1].timestamp  # keep the history time-ordered
        self.history.append(entry)
        seq = self._next_seq
        self._next_seq += 1
        self._seqs.append(seq)
        for t in entry.tags:
            self.tag_index.setdefault(t, deque()).append(seq)
        while len(self.history) > self.MAX_HISTORY_SIZE:
            self._evict()

    def retrieve(self, query: Dict[str, Any], tags: Optional[List[str]] = None, limit: int = 10,
                 min_priority: int = 0) -> List[MemoryEntry]:
        """Most recent entries matching `query` (and any of `tags`), newest first."""
        if tags:
            seqs = sorted({s for t in tags for s in self.tag_index.get(t, ())}, reverse=True)
            cands = (self._entry(s) for s in seqs)
        else:
            cands = reversed(self.history)
        out: List[MemoryEntry] = []
        for e in cands:
            if e is None:
                continue
            if e.priority >= min_priority and self.matches_query(e.data, query):
                out.append(e)
                if len(out) >= limit:
                    break
        return out

    def retrieve_by_timerange(self, start_time: datetime,
                              end_time: Optional[datetime] = None) -> List[MemoryEntry]:
        end_time = end_time or datetime.now()
        ts = [e.timestamp for e in self.history]
        lo = bisect.bisect_left(ts, start_time)
        hi = bisect.bisect_right(ts, end_time)
        return [self.history[i] for i in range(lo, hi)]

    def update_context(self, key: str, value: Any):
        self.context[key] = value
        if len(self.context) > self.MAX_CONTEXT_SIZE:
            def ts(k):
                v = self.context[k]
                return v.get("timestamp", datetime.min) if isinstance(v, dict) else datetime.min
            del self.context[min(self.context, key=ts)]

    def store_pattern(self, name: str, data: Any):
        if name not in self.patterns and len(self.patterns) >= self.MAX_PATTERNS_SIZE:
            oldest = min(self.patterns, key=lambda k: self.patterns[k]["timestamp"])
            del self.patterns[oldest]
        self.patterns[name] = {"data": data, "timestamp": datetime.now()}

    @staticmethod
    def matches_query(data: Dict[str, Any], query: Dict[str, Any]) -> bool:
        return all(k in data and data[k] == v for k, v in query.items())

    def cleanup(self, older_than: Optional[datetime] = None):
        if older_than is not None:
            while self.history and self.history[0].timestamp <= older_than:
                self._evict()

    def __len__(self) -> int:
        return len(self.history)

    # -- checkpoint (SURVEY App. D MemoryEntry format) ---------------------------
    def to_dict(self) -> Dict[str, Any]:
        return {"history": [e.model_dump(mode="json") for e in self.history],
                "context": self.context, "patterns": {k: {"data": v["data"], "timestamp": v["timestamp"].isoformat()}
                                                      for k, v in self.patterns.items()}}

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "Memory":
        m = cls()
        for e in d.get("history", []):
            ent = MemoryEntry(**e)
            m.store_nowait(ent.data, ent.tags, ent.priority, timestamp=ent.timestamp)
        m.context = dict(d.get("context", {}))
        for k, v in d.get("patterns", {}).items():
            m.patterns[k] = {"data": v["data"], "timestamp": datetime.fromisoformat(v["timestamp"])}
        return m

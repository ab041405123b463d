"""Multi-source knowledge queries with an LRU+TTL cache
(reference: pilott/knowledge/knowledge_manager.py:9-266).

query_knowledge(query, source_types) queries each named source under a
per-source lock with retries (max_retries, retry_delay) and a per-source
timeout, all within a 30 s budget; non-empty results are cached (OrderedDict LRU,
>= 100 entries, TTL >= 60 s) keyed by JSON(query, sorted sources). cleanup()
expires entries and re-tests failing sources.
"""
from __future__ import annotations

import asyncio
import json
import logging
from collections import OrderedDict
from datetime import datetime
from typing import Any, Dict, List, Optional

from pydantic import BaseModel, Field

from pilottai_amd.tools.knowledge import KnowledgeSource


class CacheEntry(BaseModel):
    value: Any = None
    timestamp: datetime = Field(default_factory=datetime.now)
    ttl: float = 3600
    access_count: int = 0
    last_access: datetime = Field(default_factory=datetime.now)


class KnowledgeManager:
    QUERY_TIMEOUT = 30.0

    def __init__(self, cache_size: int = 1000, cache_ttl: float = 3600):
        self.sources: Dict[str, KnowledgeSource] = {}
        self.cache: "OrderedDict[str, CacheEntry]" = OrderedDict()
        self.last_updated: Dict[str, datetime] = {}
        self.source_locks: Dict[str, asyncio.Lock] = {}
        self.cache_lock = asyncio.Lock()
        self.MAX_CACHE_SIZE = max(100, cache_size)
        self.DEFAULT_CACHE_TTL = max(60, cache_ttl)
        self.hits = 0
        self.misses = 0
        self._cleanup_task: Optional[asyncio.Task] = None
        self.logger = logging.getLogger("pilottai_amd.knowledge")

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

    async def add_source(self, source: KnowledgeSource) -> bool:
        if source.name in self.sources:
            self.logger.error("source %s already exists", source.name)
            return False
        self.sources[source.name] = source
        self.source_locks[source.name] = asyncio.Lock()
        self.last_updated[source.name] = datetime.now()
        source.is_connected = await self._test_connection(source)
        return source.is_connected

    async def remove_source(self, name: str) -> bool:
        src = self.sources.pop(name, None)
        self.source_locks.pop(name, None)
        if src is None:
            return False
        await src.disconnect()
        await self.invalidate_cache(source_name=name)
        return True

    async def query_knowledge(self, query: str, source_types: List[str], ttl: Optional[float] = None,
                              force_refresh: bool = False) -> List[Any]:
        if not query:
            raise ValueError("Query cannot be empty")
        if not source_types:
            raise ValueError("Source types cannot be empty")
        key = self._generate_cache_key(query, source_types)
        if not force_refresh:
            cached = await self._get_from_cache(key)
            if cached is not None:
                self.hits += 1
                return cached
        self.misses += 1
        results: List[Any] = []

        async def run():
            for name in source_types:
                src = self.sources.get(name)
                if src is None:
                    continue
                try:
                    async with self.source_locks[name]:
                        r = await self._query_source_with_retry(src, query)
                    if r is not None:
                        results.append(r)
                except Exception as e:  # noqa: BLE001
                    self.logger.error("query of %s failed: %s", name, e)
                    src.error_count += 1

        try:
            await asyncio.wait_for(run(), self.QUERY_TIMEOUT)
        except asyncio.TimeoutError:
            self.logger.error("knowledge query timed out")
            return results
        if results:
            await self._add_to_cache(key, results, ttl)
        return results

    async def _query_source_with_retry(self, src: KnowledgeSource, query: str) -> Optional[Any]:
        for attempt in range(max(1, src.max_retries)):
            try:
                if not src.is_connected and not await self._test_connection(src):
                    raise ConnectionError(f"Source {src.name} is not connected")
                return await asyncio.wait_for(src.query(query), src.timeout)
            except Exception as e:  # noqa: BLE001
                src.error_count += 1
                self.logger.warning("source %s attempt %d failed: %s", src.name, attempt + 1, e)
                if attempt < src.max_retries - 1:
                    await asyncio.sleep(src.retry_delay)
        return None

    async def _test_connection(self, src: KnowledgeSource) -> bool:
        try:
            return bool(await asyncio.wait_for(src.connect(), src.timeout))
        except Exception as e:  # noqa: BLE001
            self.logger.error("connection test for %s failed: %s", src.name, e)
            return False

    async def _get_from_cache(self, key: str) -> Optional[Any]:
        async with self.cache_lock:
            e = self.cache.get(key)
            if e is None:
                return None
            if not self._is_cache_entry_valid(e):
                del self.cache[key]
                return None
            self.cache.move_to_end(key)
            e.access_count += 1
            e.last_access = datetime.now()
            return e.value

    async def _add_to_cache(self, key: str, value: Any, ttl: Optional[float] = None):
        async with self.cache_lock:
            while len(self.cache) >= self.MAX_CACHE_SIZE:
                self.cache.popitem(last=False)
            self.cache[key] = CacheEntry(value=value, timestamp=datetime.now(), ttl=ttl or self.DEFAULT_CACHE_TTL)
            self.cache.move_to_end(key)

    @staticmethod
    def _is_cache_entry_valid(e: CacheEntry) -> bool:
        return (datetime.now() - e.timestamp).total_seconds() < e.ttl

    @staticmethod
    def _generate_cache_key(query: str, source_types: List[str]) -> str:
        return json.dumps({"query": query, "sources": sorted(source_types)}, sort_keys=True)

    async def invalidate_cache(self, source_name: Optional[str] = None, pattern: Optional[str] = None):
        async with self.cache_lock:
            if source_name:
                dead = [k for k in self.cache if source_name in json.loads(k)["sources"]]
            elif pattern:
                dead = [k for k in self.cache if pattern in k]
            else:
                self.cache.clear()
                return
            for k in dead:
                del self.cache[k]

    async def _periodic_cleanup(self):
        while True:
            await asyncio.sleep(3600)
            try:
                await self.cleanup()
            except Exception as e:  # noqa: BLE001
                self.logger.error("cleanup error: %s", e)

    async def cleanup(self):
        async with self.cache_lock:
            for k in [k for k, v in self.cache.items() if not self._is_cache_entry_valid(v)]:
                del self.cache[k]
        for src in self.sources.values():
            if src.error_count > src.max_retries:
                src.is_connected = False
                if await self._test_connection(src):
                    src.error_count = 0
                    src.is_connected = True

    def get_source_stats(self) -> Dict[str, Dict[str, Any]]:
        return {n: {"access_count": s.access_count, "error_count": s.error_count,
                    "last_access": s.last_access.isoformat(), "is_connected": s.is_connected}
                for n, s in self.sources.items()}

    def get_cache_stats(self) -> Dict[str, Any]:
        total = self.hits + self.misses
        return {"size": len(self.cache), "max_size": self.MAX_CACHE_SIZE, "hits": self.hits, "misses": self.misses,
                "hit_ratio": self.hits / total if total else 0.0, "default_ttl": self.DEFAULT_CACHE_TTL}

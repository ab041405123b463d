"""Knowledge sources (reference: pilott/tools/knowledge.py:5-62 and the duplicate in
pilott/knowledge/knowledge_manager.py:16-26, merged here — SURVEY §2.3, App. A #28).

One `KnowledgeSource` type carries both the connection lifecycle
(connect/query/disconnect) and the retry/timeout fields the KnowledgeManager
needs. Built-in kinds:
  "memory"   — in-process list of documents; query = case-insensitive match
  "file"     — a text file or a directory of *.txt/*.md/*.json files
  "semantic" — an EnhancedMemory (HBM semantic index); query = top-k search
  "callable" — `connection["fn"](query)` (sync or async)
  "database" / "api" — accepted for API compatibility; they delegate to
                       `connection["fn"]` when provided, else return no results.
"""
from __future__ import annotations

import asyncio
import inspect
import json
from datetime import datetime
from pathlib import Path
from typing import Any, Dict, List, Optional

from pydantic import BaseModel, ConfigDict, Field, PrivateAttr


class KnowledgeSource(BaseModel):
    model_config = ConfigDict(arbitrary_types_allowed=True)

    name: str
    type: str = "memory"
    connection: Dict[str, Any] = Field(default_factory=dict)
    last_access: datetime = Field(default_factory=datetime.now)
    access_count: int = 0
    error_count: int = 0
    is_connected: bool = False
    max_retries: int = 3
    retry_delay: float = 1.0
    timeout: float = 30.0
    limit: int = 5
    _docs: List[str] = PrivateAttr(default_factory=list)

    async def connect(self) -> bool:
        kind = self.type
        try:
            if kind == "memory":
                self._docs = [str(d) for d in self.connection.get("documents", [])]
            elif kind == "file":
                p = Path(self.connection.get("path", ""))
                files = [p] if p.is_file() else sorted(
                    f for ext in ("*.txt", "*.md", "*.json") for f in p.glob(ext)) if p.exists() else []
                if not files:
                    return False
                self._docs = [f.read_text(errors="replace") for f in files]
            elif kind == "semantic":
                if self.connection.get("memory") is None:
                    return False
            elif kind in ("callable", "database", "api"):
                if kind == "callable" and not callable(self.connection.get("fn")):
                    return False
            else:
                return False
            self.is_connected = True
            return True
        except Exception:  # noqa: BLE001
            self.is_connected = False
            return False

    async def query(self, query: str) -> Any:
        if not self.is_connected and not await self.connect():
            raise ConnectionError(f"Source {self.name} is not connected")
        self.access_count += 1
        self.last_access = datetime.now()
        kind = self.type
        if kind in ("memory", "file"):
            q = query.lower()
            hits = [d for d in self._docs if q in d.lower()]
            return hits[: self.limit]
        if kind == "semantic":
            mem = self.connection["memory"]
            items = await mem.semantic_search(query, limit=self.limit)
            return [{"text": it.text, "metadata": it.metadata, "priority": it.priority} for it in items]
        fn = self.connection.get("fn")
        if fn is None:
            return {}
        r = fn(query)
        return await r if inspect.isawaitable(r) else r

    async def disconnect(self) -> bool:
        self.is_connected = False
        self._docs = []
        return True

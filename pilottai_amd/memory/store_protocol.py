"""The one semantic-store contract that every memory backend implements.

Agents reach semantic memory only through `MemoryLookupBatcher` (memory/batcher.py), which
calls the store's coroutine API below. Two stores implement it:

* `EnhancedMemory` (memory/enhanced_memory.py) -- one GPU's HBM-resident index;
* `NodeSemanticStore` (memory/node_store.py) -- rows sharded over the agent-DP ranks.

The reference has one store (pilott/memory/enhanced_memory.py:60-116, `store_semantic` /
`semantic_search`); here the two backends drifted once (round 5: the batcher passed `vecs=`
to a store that did not take it, and every node-mode write failed). `SemanticStore` is the
Protocol both classes are checked against (tests/test_node_memory.py compares the parameter
lists), so a keyword the batcher relies on cannot be missing from one of them again.
"""
from __future__ import annotations

import inspect
from typing import Any, List, Optional, Protocol, Sequence, Set, runtime_checkable


@runtime_checkable
class SemanticStore(Protocol):
    async def embed_queries(self, queries: Sequence[str]) -> Any:
        """Embeddings of `queries` ([n, dim]; a device tensor or an array), to pass as `vecs=`."""

    async def search_batch(self, queries: Sequence[str], tags: Optional[Sequence[Optional[Set[str]]]] = None,
                           min_priority: Optional[Sequence[int]] = None, limit: int = 5,
                           mode: str = "semantic", vecs=None) -> List[list]:
        """Top-`limit` MemoryItems per query; `vecs` skips embedding."""

    async def store_semantic_batch(self, texts: Sequence[str], metadatas=None, tags=None, priorities=None,
                                   ttl: Optional[float] = None, vecs=None) -> List[int]:
        """Append items; returns their (global) row ids; `vecs` skips embedding."""

    async def semantic_search(self, query: str, tags: Optional[Set[str]] = None, min_priority: int = 0,
                              limit: int = 5) -> list:
        ...

    async def store_semantic(self, text: str, metadata=None, tags: Optional[Set[str]] = None, priority: int = 0,
                             ttl: Optional[float] = None) -> int:
        ...


PROTOCOL_METHODS = ("embed_queries", "search_batch", "store_semantic_batch", "semantic_search", "store_semantic")


def signature_mismatches(cls) -> List[str]:
    """Methods of `cls` whose parameters are missing any of the protocol's (by name) or are
    not coroutines; [] when `cls` satisfies the contract."""
    bad = []
    for name in PROTOCOL_METHODS:
        impl = getattr(cls, name, None)
        if impl is None or not inspect.iscoroutinefunction(impl):
            bad.append(f"{name}: missing or not async")
            continue
        want = list(inspect.signature(getattr(SemanticStore, name)).parameters)
        have = inspect.signature(impl).parameters
        missing = [p for p in want if p not in have and not any(
            v.kind == inspect.Parameter.VAR_KEYWORD for v in have.values())]
        if missing:
            bad.append(f"{name}: missing parameters {missing}")
    return bad

"""Agent-level data parallelism over the GPUs of a node.

One process per GPU, each with its own engine and `Serve`; worker agents are
sharded over the ranks (`shard_workers`). `GlobalLoadView` gives every rank the
same picture of the whole node with one small all-gather (RCCL over xGMI on
GPUs, gloo on CPU): per-rank queued / running tasks, idle agents, KV-cache
utilisation and engine throughput — what a front-end or DynamicScaling uses to
pick the least-loaded replica for new work.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from .comm import _coll_device

LOAD_FIELDS = ("queue_size", "running_tasks", "idle_agents", "kv_cache_utilization", "engine_tokens_per_s")


def shard_workers(n_workers: int, world: int, rank: int) -> range:
    """Contiguous shard of worker indices for `rank` (sizes differ by at most one)."""
    base, extra = divmod(n_workers, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def local_load(serve) -> List[float]:
    m = serve.get_metrics()
    eng = m.get("engine") or {}
    kv = 1.0 - eng.get("free_kv_blocks", 1) / max(1, eng.get("total_kv_blocks", 1)) if eng else 0.0
    busy = max(1e-9, float(eng.get("busy_s", 0.0)))
    return [float(m.get("queue_size", 0)), float(m.get("running_tasks", 0)), float(m.get("idle_agents", 0)),
            float(kv), float(eng.get("tokens", 0.0)) / busy if eng else 0.0]


class GlobalLoadView:
    def __init__(self, group: Optional["dist.ProcessGroup"] = None):
        self.group = group
        self.table: List[Dict[str, float]] = []

    def update(self, load: List[float]) -> List[Dict[str, float]]:
        """Collective: every rank contributes its load vector, all get the table."""
        t = torch.tensor(load, dtype=torch.float64, device=_coll_device())
        if dist.is_initialized():
            world = dist.get_world_size(self.group)
            out = torch.empty(world, len(load), dtype=torch.float64, device=t.device)
            if t.device.type == "cpu":
                parts = [torch.empty_like(t) for _ in range(world)]
                dist.all_gather(parts, t, group=self.group)
                out = torch.stack(parts)
            else:
                dist.all_gather_into_tensor(out, t, group=self.group)
        else:
            out = t.unsqueeze(0)
        self.table = [dict(zip(LOAD_FIELDS, row)) for row in out.cpu().tolist()]
        return self.table

    def least_loaded_rank(self) -> int:
        """Fewest queued + running tasks; ties broken by KV-cache utilisation."""
        if not self.table:
            return 0
        return min(range(len(self.table)),
                   key=lambda r: (self.table[r]["queue_size"] + self.table[r]["running_tasks"],
                                  self.table[r]["kv_cache_utilization"], r))

    def totals(self) -> Dict[str, float]:
        return {k: sum(row[k] for row in self.table) for k in LOAD_FIELDS}

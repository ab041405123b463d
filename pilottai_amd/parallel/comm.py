"""Process groups and collectives (RCCL over xGMI on MI355X, gloo on CPU).

One process per GPU. `torch.distributed` with backend "nccl" is RCCL on ROCm.
Groups used by the framework:

* world   — agent-DP control plane: load counters (all-reduce), shared-context
            broadcast, sharded semantic-index candidate all-gather, barriers.
* TP      — tensor-parallel group of one model replica (70B: TP=8 on one node);
            row-parallel outputs are all-reduced, sampling winners all-gathered.

xGMI is point-to-point (7 links per GPU): decode-size TP all-reduces are latency
bound, so bf16 messages up to 8 MiB go through the custom one-shot/two-shot P2P
kernel (parallel/custom_ar.py, csrc/ops/custom_ar.hip) and larger ones through
RCCL. Both are captured inside the engine's hipGraphs.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist


@dataclass
class TPGroup:
    group: Optional["dist.ProcessGroup"] = None
    rank: int = 0
    size: int = 1
    root: int = 0                                   # global rank of TP rank 0 (the step driver)
    cpu_group: Optional["dist.ProcessGroup"] = None  # gloo group for host-side step headers
    custom: Optional[object] = None                 # CustomAllReduce over P2P IPC buffers (GPU TP)

    @staticmethod
    def single() -> "TPGroup":
        return TPGroup(None, 0, 1)

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        if self.size > 1:
            if self.custom is not None and self.custom.eligible(t):
                return self.custom.all_reduce(t)
            dist.all_reduce(t, group=self.group)
        return t

    def all_reduce_add(self, t: torch.Tensor, resid: torch.Tensor, ss: Optional[torch.Tensor] = None,
                       ss_zero: Optional[torch.Tensor] = None) -> torch.Tensor:
        """resid += all_reduce(t) (in place); ss[:rows] <- row sums of squares of the new resid
        (ss must hold zeros on entry), ss_zero[:rows] <- 0. One fused launch on the custom
        all-reduce (csrc/ops/custom_ar.hip, RES epilogue); otherwise RCCL / gloo + add + stats."""
        rows = resid.shape[0]
        if self.size > 1 and self.custom is not None and self.custom.fusable(t, resid):
            return self.custom.all_reduce_add(t, resid, ss, ss_zero)
        self.all_reduce(t)
        resid.add_(t)
        if ss is not None:
            from pilottai_amd import ops

            ops.row_sumsq(resid, out=ss)
        if ss_zero is not None:
            ss_zero[:rows].zero_()
        return resid

    def all_reduce_max(self, t: torch.Tensor) -> torch.Tensor:
        """In-place elementwise max over the group: fp32 device tensors on the custom P2P
        buffers (capturable, no RCCL in a step graph), anything else through the process group."""
        if self.size > 1:
            if self.custom is not None and self.custom.collective_eligible(t, "max"):
                return self.custom.all_reduce_f32(t, "max")
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return t

    def all_reduce_sum(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over the group (fp32 histograms etc.): the custom P2P buffers when
        eligible (rank-order sums, bit-identical on every rank), else the process group."""
        if self.size > 1:
            if self.custom is not None and self.custom.collective_eligible(t, "sum"):
                return self.custom.all_reduce_f32(t, "sum")
            dist.all_reduce(t, group=self.group)
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenate `t` from every rank along a new leading dim: [size, *t.shape]."""
        if self.size == 1:
            return t.unsqueeze(0)
        if self.custom is not None and self.custom.collective_eligible(t, "gather"):
            return self.custom.all_gather(t)
        if t.device.type == "cpu" or dist.get_backend(self.group) == "gloo":  # gloo: list form
            parts = [torch.empty_like(t) for _ in range(self.size)]
            dist.all_gather(parts, t.contiguous(), group=self.group)
            return torch.stack(parts)
        out = torch.empty((self.size,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        return out

    def broadcast(self, t: torch.Tensor, cpu: bool = False) -> torch.Tensor:
        """Broadcast from the driver (TP rank 0)."""
        if self.size > 1:
            dist.broadcast(t, src=self.root, group=self.cpu_group if cpu else self.group)
        return t


def env_rank_world():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def init_distributed(backend: Optional[str] = None, timeout_s: int = 600, single: bool = False) -> tuple:
    """Initialise the default process group from torchrun-style env vars.

    Returns (rank, world_size, local_rank). backend defaults to "nccl" (RCCL)
    when a GPU is visible, else "gloo". Safe to call twice. A world of one rank
    creates no group unless `single` (a one-process group, e.g. to exercise RCCL).
    """
    rank, world, local = env_rank_world()
    if world <= 1 and not single:
        return 0, 1, 0
    if not dist.is_initialized():
        if backend is None:
            # PILOTTAI_DIST_BACKEND=gloo lets several ranks share one GPU (a 1-GPU
            # rehearsal of the multi-rank bench); RCCL refuses duplicate devices
            backend = os.environ.get("PILOTTAI_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return rank, world, local


def new_tp_groups(tp_size: int, custom_ar: Optional[bool] = None) -> TPGroup:
    """Split the world into contiguous TP groups of `tp_size`; return this rank's group.

    custom_ar: None = use the P2P all-reduce whenever the backend is RCCL; True = also
    under gloo when a GPU is visible (the 1-GPU test that shares GPU 0 between ranks).
    """
    if not dist.is_initialized() or tp_size <= 1:
        return TPGroup.single()
    world = dist.get_world_size()
    rank = dist.get_rank()
    assert world % tp_size == 0, "world size must be a multiple of the TP size"
    mine = None
    gloo_needed = dist.get_backend() != "gloo"
    for start in range(0, world, tp_size):
        ranks = list(range(start, start + tp_size))
        g = dist.new_group(ranks)
        cg = dist.new_group(ranks, backend="gloo") if gloo_needed else g
        if rank in ranks:
            mine = TPGroup(g, rank - start, tp_size, root=start, cpu_group=cg)
    want = custom_ar if custom_ar is not None else dist.get_backend() == "nccl"
    if want and torch.cuda.is_available():
        from pilottai_amd.parallel.custom_ar import CustomAllReduce

        dev = torch.device("cuda", torch.cuda.current_device())
        mine.custom = CustomAllReduce.create(mine.cpu_group, mine.rank, mine.size, dev)
    return mine


def barrier(group=None):
    if dist.is_initialized():
        if dist.get_backend(group) == "nccl":
            dist.barrier(group=group, device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier(group=group)


def all_reduce_max(x: float, device=None) -> float:
    if not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device or _coll_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_sum(values: List[float], device=None) -> List[float]:
    if not dist.is_initialized():
        return list(values)
    t = torch.tensor(values, dtype=torch.float64, device=device or _coll_device())
    dist.all_reduce(t)
    return t.tolist()


def broadcast_object(obj, src: int = 0, group=None):
    """src: a global rank (a member of `group`)."""
    if not dist.is_initialized():
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=src, group=group)
    return lst[0]


def new_dp_group(tp_size: int):
    """The group of TP drivers (global ranks 0, T, 2T, ...): the agent-DP replicas when every
    replica is a TP group of `tp_size` ranks (contiguous, as new_tp_groups). Every rank must
    call this (torch.distributed.new_group is collective); None without a process group."""
    if not dist.is_initialized():
        return None
    return dist.new_group(list(range(0, dist.get_world_size(), max(1, tp_size))))


def broadcast_tokens(ids: Optional[List[int]], src: int = 0) -> List[int]:
    """Shared-context broadcast: token ids from `src` to every rank,
    as two tensor broadcasts (length, ids) — RCCL over xGMI on GPUs, gloo on CPU."""
    if not dist.is_initialized():
        return list(ids or [])
    dev = _coll_device()
    n = torch.tensor([len(ids) if dist.get_rank() == src else 0], dtype=torch.int64, device=dev)
    dist.broadcast(n, src=src)
    buf = torch.tensor(ids, dtype=torch.int32, device=dev) if dist.get_rank() == src else \
        torch.empty(int(n.item()), dtype=torch.int32, device=dev)
    if int(n.item()) > 0:
        dist.broadcast(buf, src=src)
    return buf.cpu().tolist()


def _coll_device():
    if dist.is_initialized() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")

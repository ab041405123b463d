"""Custom P2P all-reduce for tensor-parallel messages.

The reference has no distributed backend at all (everything is in-process
Python and one asyncio.Queue; the LLM is an HTTPS call, `pilott/engine/llm.py`). On an
MI355X node the TP=8 70B replica (BASELINE config 2/5) all-reduces the row-parallel
o_proj / down_proj outputs twice per layer: 160 bf16 messages of 16 KiB x tokens per
decode step. RCCL's ring sends such a message through W-1 hops on one xGMI link per
direction; the kernel in csrc/ops/custom_ar.hip instead reads every peer's buffer over
all 7 links at once (one-shot for small messages, reduce-scatter + gather "two-shot"
above `two_shot_bytes`). Messages larger than the IPC buffer go to RCCL.

Setup is collective over the TP group: every rank allocates an uncached IPC buffer
(flags + two data parities), the 64-byte handles are exchanged with
`all_gather_object`, and every rank maps its peers' buffers. All ranks then agree
(MIN all-reduce) on whether every mapping succeeded, so either the whole group uses
the custom path or the whole group stays on RCCL — never a mix, which would deadlock.

The launch has no per-call arguments beyond the tensor (epochs live on the device),
so it is captured into the engine's hipGraphs like any other kernel.
"""
from __future__ import annotations

import contextlib
import logging
import os
from typing import List, Optional

import torch
import torch.distributed as dist

log = logging.getLogger(__name__)

# per data parity: a 2,048-token step of the 70B model (2,048 x 8,192 x bf16), so every TP
# all-reduce of a step graph -- the embedding, o and down projections -- stays on the custom
# path (no RCCL call inside a captured graph)
DEFAULT_CAP_BYTES = 32 << 20
DEFAULT_TWO_SHOT_BYTES = 512 << 10   # above this the 2(W-1)/W traffic of two-shot wins


def _native():
    from pilottai_amd.ops.kernels import require_native

    return require_native()


class CustomAllReduce:
    """In-place bf16 all-reduce over peer-mapped IPC buffers for one TP group."""

    def __init__(self, bases: List[int], rank: int, device: torch.device, cap_bytes: int,
                 own_ptr: int, opened: List[int], two_shot_bytes: int = DEFAULT_TWO_SHOT_BYTES):
        self.C = _native()
        self.bases = bases
        self.world = len(bases)
        self.rank = rank
        self.device = device
        self.cap_bytes = cap_bytes
        self.two_shot_bytes = two_shot_bytes
        self._own = own_ptr
        self._opened = opened
        self.epochs = torch.zeros(self.C.car_group(), dtype=torch.int32, device=device)
        self.err = torch.zeros(1, dtype=torch.int32, device=device)
        self.calls = 0

    # -- construction ---------------------------------------------------------------
    @staticmethod
    def buffer_bytes(cap_bytes: int) -> int:
        return int(_native().car_flag_bytes()) + 2 * cap_bytes

    @classmethod
    def create(cls, group, rank: int, world: int, device: torch.device,
               cap_bytes: int = DEFAULT_CAP_BYTES) -> Optional["CustomAllReduce"]:
        """Collective over `group`; returns None on every rank unless all ranks succeed."""
        if world < 2 or world > 8 or os.environ.get("PILOTTAI_CUSTOM_AR", "1") == "0":
            return None
        C = _native()
        own, handle, err = 0, b"", ""

        def on_device():
            return torch.cuda.device(device) if device.type == "cuda" else contextlib.nullcontext()

        try:
            with on_device():
                own, handle = C.car_alloc(cls.buffer_bytes(cap_bytes))
        except Exception as e:  # noqa: BLE001 - reported collectively below
            err = str(e)
        handles: List = [None] * world
        dist.all_gather_object(handles, handle, group=group)
        opened: List[int] = []
        bases: List[int] = []
        ok = 1 if own else 0
        if ok:
            try:
                with on_device():
                    for i, h in enumerate(handles):
                        if i == rank:
                            bases.append(own)
                        elif not h:
                            raise RuntimeError(f"rank {i} has no IPC buffer")
                        else:
                            p = C.car_open(h)
                            opened.append(p)
                            bases.append(p)
            except Exception as e:  # noqa: BLE001
                err, ok = str(e), 0
        flag = torch.tensor([ok], dtype=torch.int32,
                            device=device if dist.get_backend(group) == "nccl" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        if int(flag.item()) == 0:
            for p in opened:
                C.car_close(p)
            if own:
                C.car_free(own)
            log.warning("custom all-reduce disabled for this TP group (%s); using RCCL", err or "a peer failed")
            return None
        return cls(bases, rank, device, cap_bytes, own, opened)

    # -- use ------------------------------------------------------------------------
    def eligible(self, t: torch.Tensor) -> bool:
        n = t.numel()
        return (t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous() and n % 8 == 0
                and n * 2 <= self.cap_bytes and t.data_ptr() % 16 == 0)

    def all_reduce(self, t: torch.Tensor, two_shot: Optional[bool] = None) -> torch.Tensor:
        """Sum `t` over the group in place (every rank gets bit-identical results)."""
        if two_shot is None:
            two_shot = self.world > 2 and t.numel() * 2 > self.two_shot_bytes
        self.C.car_all_reduce(self.bases, self.rank, [t], [t], self.cap_bytes, self.epochs, self.err,
                              bool(two_shot))
        self.calls += 1
        return t

    def all_reduce_add(self, t: torch.Tensor, resid: torch.Tensor, ss: Optional[torch.Tensor] = None,
                       ss_zero: Optional[torch.Tensor] = None, two_shot: Optional[bool] = None) -> torch.Tensor:
        """resid += sum over the group of `t` in ONE launch (the row-parallel o / down epilogue
        under TP): ss[row] += sum of squares of the written bf16 rows (the next RMSNorm's row
        statistics), ss_zero[:rows] <- 0. Replaces all-reduce -> resid.add_ -> row_sumsq."""
        if two_shot is None:
            two_shot = self.world > 2 and t.numel() * 2 > self.two_shot_bytes
        self.C.car_all_reduce(self.bases, self.rank, [t.reshape(-1)], [resid.reshape(-1)], self.cap_bytes,
                              self.epochs, self.err, bool(two_shot), resids=[resid.reshape(-1)],
                              ss=[ss] if ss is not None else [], ss_zero=[ss_zero] if ss_zero is not None else [],
                              row_len=int(resid.shape[-1]))
        self.calls += 1
        return resid

    # -- small collectives of the TP step graph (custom_ar.hip co_kernel) ---------------
    _OPS = {"sum": 0, "max": 1, "gather": 2}

    def collective_eligible(self, t: torch.Tensor, op: str) -> bool:
        n = t.numel()
        ok_dtype = t.dtype == torch.float32 if op in ("sum", "max") else t.element_size() == 4
        return (t.is_cuda and ok_dtype and t.is_contiguous() and n % 4 == 0 and n > 0
                and n * 4 <= self.cap_bytes and t.data_ptr() % 16 == 0)

    def all_reduce_f32(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """In-place fp32 SUM (rank order: bit-identical on every rank) or MAX over the group."""
        self.C.car_collective(self.bases, self.rank, [t], [t], self.cap_bytes, self.epochs, self.err,
                              self._OPS[op])
        self.calls += 1
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *t.shape]: every rank's `t` (any 4-byte dtype)."""
        out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        self.C.car_collective(self.bases, self.rank, [t], [out], self.cap_bytes, self.epochs, self.err, 2)
        self.calls += 1
        return out

    def fusable(self, t: torch.Tensor, resid: torch.Tensor) -> bool:
        return (self.eligible(t) and resid.is_contiguous() and resid.numel() == t.numel()
                and resid.dtype == torch.bfloat16 and resid.data_ptr() % 16 == 0
                and resid.shape[-1] % 2048 == 0)

    def healthy(self) -> bool:
        """False once any barrier timed out (a peer died or stalled); syncs the stream."""
        return int(self.err.item()) == 0

    def close(self):
        C = self.C
        for p in self._opened:
            C.car_close(p)
        self._opened = []
        if self._own:
            C.car_free(self._own)
            self._own = 0


def local_group_collective(C, tensors: List[torch.Tensor], cap_bytes: int, op: str, state: dict,
                           outs: Optional[List[torch.Tensor]] = None) -> List[torch.Tensor]:
    """Single-process form of the small collectives (tests): W 'ranks' in one launch. op "sum" /
    "max" reduce in place; "gather" returns one [W, n] tensor per rank."""
    W = len(tensors)
    key = (W, cap_bytes)
    if key not in state:
        bufs = [C.car_alloc(CustomAllReduce.buffer_bytes(cap_bytes))[0] for _ in range(W)]
        epochs = torch.zeros(W * C.car_group(), dtype=torch.int32, device=tensors[0].device)
        err = torch.zeros(1, dtype=torch.int32, device=tensors[0].device)
        state[key] = (bufs, epochs, err)
    bufs, epochs, err = state[key]
    if op == "gather":
        outs = outs or [torch.empty((W,) + tuple(t.shape), dtype=t.dtype, device=t.device) for t in tensors]
        C.car_collective(bufs, 0, tensors, outs, cap_bytes, epochs, err, 2)
        return outs
    C.car_collective(bufs, 0, tensors, tensors, cap_bytes, epochs, err, CustomAllReduce._OPS[op])
    return tensors


def local_group_all_reduce(C, tensors: List[torch.Tensor], cap_bytes: int, two_shot: bool,
                           state: dict, resids: Optional[List[torch.Tensor]] = None,
                           ss: Optional[List[torch.Tensor]] = None, ss_zero: Optional[List[torch.Tensor]] = None,
                           row_len: int = 0) -> None:
    """Single-process form used by tests: W 'ranks' share one launch on one GPU.

    `state` caches the W buffers and epoch counters between calls (keyed by W and cap).
    """
    W = len(tensors)
    key = (W, cap_bytes)
    if key not in state:
        bufs = [C.car_alloc(CustomAllReduce.buffer_bytes(cap_bytes))[0] for _ in range(W)]
        epochs = torch.zeros(W * C.car_group(), dtype=torch.int32, device=tensors[0].device)
        err = torch.zeros(1, dtype=torch.int32, device=tensors[0].device)
        state[key] = (bufs, epochs, err)
    bufs, epochs, err = state[key]
    if resids is None:
        C.car_all_reduce(bufs, 0, tensors, tensors, cap_bytes, epochs, err, two_shot)
    else:  # fused residual epilogue: resids[r] += sum, row statistics into ss[r]
        C.car_all_reduce(bufs, 0, tensors, resids, cap_bytes, epochs, err, two_shot, resids=resids,
                         ss=ss or [], ss_zero=ss_zero or [], row_len=row_len)

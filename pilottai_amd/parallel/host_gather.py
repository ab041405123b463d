"""Host-payload all-gather among the ranks of ONE node through shared memory.

The node-wide semantic store (memory/node_store.py) runs a lockstep round every few
milliseconds whose host part -- counts, filters, tag strings, written items -- is a few hundred
bytes per rank. Over gloo (loopback TCP) one such all-gather costs 7-11 ms at 8 ranks in our
measurement (tools/node_store_rounds.py, results/node_store_rounds_r6.jsonl), which made the
host control plane, not the scan, the round's cost. All agent-DP ranks of this framework live
on one MI355X node, so the host hop goes through a POSIX shared-memory segment instead
(csrc/runtime/shm_ring.cpp `ShmGather`: a release-published slot per rank, two banks), the
same idea as the TP step header ring ("shared-memory rings rather than sockets").

Payloads larger than a slot go in several rounds (each rank's total length leads its first
chunk). Ranks on different hosts (never the case for the bench, possible for a user's group)
fall back to gloo object collectives.
"""
from __future__ import annotations

import os
import pickle
import socket
import struct
import uuid
from typing import Any, List

import numpy as np
import torch.distributed as dist

_HDR = struct.Struct("<q")


def _boot_id() -> str:
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            return f.read().strip()
    except OSError:
        return ""


class HostGather:
    def __init__(self, group=None, slot_bytes: int = 1 << 20, timeout_s: float = 600.0, force_gloo: bool = False):
        """group: a gloo-capable process group (used once to agree on the segment, and as the
        fallback transport)."""
        on = dist.is_available() and dist.is_initialized()
        self.group = group
        self.rank = dist.get_rank(group) if on else 0
        self.world = dist.get_world_size(group) if on else 1
        self.timeout_s = float(timeout_s)
        self._shm = None
        self.transport = "local"
        if self.world == 1:
            return
        where = [None] * self.world
        dist.all_gather_object(where, (socket.gethostname(), _boot_id()), group=group)
        if force_gloo or len(set(where)) != 1 or os.environ.get("PILOTTAI_HOST_GATHER") == "gloo":
            self.transport = "gloo"
            return
        from pilottai_amd import _runtime

        box = [f"/pilottai-hg-{os.getpid()}-{uuid.uuid4().hex[:12]}" if self.rank == 0 else None]
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                   group=group)
        if self.rank == 0:
            self._shm = _runtime.ShmGather(box[0], self.world, 0, slot_bytes, True)
        dist.barrier(group=group)
        if self.rank != 0:
            self._shm = _runtime.ShmGather(box[0], self.world, self.rank, slot_bytes, False, 120.0)
        dist.barrier(group=group)
        if self.rank == 0:
            self._shm.unlink()  # every rank has it mapped: no name left behind if a rank crashes
        self.slot = int(self._shm.slot_bytes)
        self.transport = "shm"

    @property
    def waited_s(self) -> float:
        """Seconds this rank spent waiting for peers inside shared-memory all-gathers."""
        return float(self._shm.waited_s) if self._shm is not None else 0.0

    # ------------------------------------------------------------------ payloads
    def gather_bytes(self, payload: bytes) -> List[bytes]:
        if self.world == 1:
            return [payload]
        if self._shm is None:
            out = [None] * self.world
            dist.all_gather_object(out, payload, group=self.group)
            return out
        data = _HDR.pack(len(payload)) + payload
        parts = [[] for _ in range(self.world)]
        totals = None
        off = 0
        while True:
            got = self._shm.all_gather(data[off:off + self.slot], self.timeout_s)
            if got is None:
                raise RuntimeError(f"host all-gather timed out after {self.timeout_s} s (a rank died or left)")
            off += self.slot
            if totals is None:
                totals = [_HDR.unpack_from(g)[0] + _HDR.size for g in got]
            for q, g in enumerate(got):
                parts[q].append(g)
            if off >= max(totals):
                break
        return [b"".join(p)[_HDR.size:totals[q]] for q, p in enumerate(parts)]

    def gather_obj(self, obj: Any) -> list:
        """Objects of this framework's own ranks (never data read from a file)."""
        if self.world == 1:
            return [obj]
        if self._shm is None:
            out = [None] * self.world
            dist.all_gather_object(out, obj, group=self.group)
            return out
        return [pickle.loads(b) for b in self.gather_bytes(pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL))]

    def gather_array(self, a: np.ndarray) -> np.ndarray:
        """[world, *a.shape] (every rank passes the same shape and dtype)."""
        a = np.ascontiguousarray(a)
        if self.world == 1:
            return a[None]
        if self._shm is None:
            import torch

            t = torch.from_numpy(a)
            parts = [torch.empty_like(t) for _ in range(self.world)]
            dist.all_gather(parts, t, group=self.group)
            return np.stack([p.numpy() for p in parts])
        got = self.gather_bytes(a.tobytes())
        return np.stack([np.frombuffer(g, dtype=a.dtype).reshape(a.shape) for g in got])

    def all_to_all_array(self, a: np.ndarray) -> np.ndarray:
        """a: [world, ...], a[q] destined for rank q. Returns [world, ...] whose row q is rank
        q's a[self.rank] (each rank reads only its own chunk of every peer's slot)."""
        a = np.ascontiguousarray(a)
        if a.shape[0] != self.world:
            raise ValueError(f"all_to_all_array: leading dim {a.shape[0]} != world {self.world}")
        if self.world == 1:
            return a.copy()
        chunk = a[0].nbytes
        if self._shm is None or a.nbytes > self.slot:
            return self.gather_array(a)[:, self.rank]
        got = self._shm.all_gather(a.tobytes(), self.timeout_s, self.rank * chunk, chunk)
        if got is None:
            raise RuntimeError(f"host all-to-all timed out after {self.timeout_s} s (a rank died or left)")
        return np.stack([np.frombuffer(g, dtype=a.dtype).reshape(a.shape[1:]) for g in got])

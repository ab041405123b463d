"""HBM-resident embedding index with fused filter + cosine top-k.

Rows are L2-normalised bf16 vectors in one preallocated device matrix
[capacity, D] (100M x 1024 bf16 = 204.8 GB fits one 288 GB MI355X next to an 8B
model), with per-row filter metadata kept beside them on the device:
priority (int32), tag bitmask (int64), expiry (float32 seconds on the index's
clock, 0 = never). Search runs `ops.cosine_topk` (csrc/ops/similarity.hip):
one streaming MFMA pass over the rows for a batch of queries, filters applied
in-kernel, per-slice top-k merged on device.

The index is a ring buffer once full, which is the reference's bounded-deque
eviction (pilott/memory/enhanced_memory.py:27) without its stale-index bug
(App. A #26): row ids are stable until the row is overwritten.

Tags map to bits 0..62 through a registry; further distinct tags share bit 63
and are re-checked exactly on the host for the (few) returned candidates.
`ShardedSemanticIndex` splits rows across ranks and merges per-rank top-k with
one all-gather (RCCL over xGMI).
"""
from __future__ import annotations

import threading
import time
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from pilottai_amd import ops

OVERFLOW_BIT = 63


class TagRegistry:
    def __init__(self):
        self.bits: Dict[str, int] = {}

    def bit(self, tag: str, create: bool = True) -> int:
        b = self.bits.get(tag)
        if b is None:
            if not create:
                return -1
            b = len(self.bits) if len(self.bits) < OVERFLOW_BIT else OVERFLOW_BIT
            if b < OVERFLOW_BIT:
                self.bits[tag] = b
        return b

    def mask(self, tags: Iterable[str], create: bool = True) -> Tuple[int, bool]:
        """(bitmask, exact) — exact is False when an overflow tag is involved."""
        m, exact = 0, True
        for t in tags or ():
            b = self.bit(t, create)
            if b < 0:
                return -1, True  # unknown tag: nothing can match
            if b == OVERFLOW_BIT:
                exact = False
            m |= 1 << b
        if m >= 1 << 63:
            m -= 1 << 64  # two's complement for int64 storage
        return m, exact


STORAGES = ("bf16", "q16")


class SemanticIndex:
    def __init__(self, dim: int = 1024, capacity: int = 1 << 16, device=None, growable: bool = True,
                 max_capacity: Optional[int] = None, storage: str = "bf16"):
        """storage: "bf16" -- rows as bf16 tiles, one-pass bf16 MFMA scan (csrc/ops/similarity.hip);
        "q16" -- rows as 16-bit fixed point in two int8 planes, the two-stage exact scan that
        streams only the high plane (csrc/ops/similarity_q16.hip: 1 byte per dimension per pass
        instead of 2, same bytes resident)."""
        if storage not in STORAGES:
            raise ValueError(f"storage must be one of {STORAGES}, not {storage!r}")
        self.storage = storage
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
                else torch.device("cpu")
        self.device = torch.device(device)
        self.dim = dim
        self.growable = growable
        self.max_capacity = max_capacity or capacity if not growable else (max_capacity or 1 << 31)
        self._alloc(capacity)
        self.size = 0          # rows ever written (ring position = size % capacity)
        self.tags = TagRegistry()
        self.row_tags_py: Dict[int, frozenset] = {}
        self.epoch = time.time()
        self._lock = threading.Lock()
        self._ws: Optional[torch.Tensor] = None
        self._stream = None
        self.pass_events: Optional[list] = None  # set to [] to time every search pass (HIP events)
        self.stats = {"q16_fallbacks": 0}  # q16: batches re-run on the exact scan (drop check)

    def _alloc(self, cap: int):
        d = self.device
        self.capacity = cap
        # Rows are stored fragment-major in tiles of 16 (csrc/ops/similarity.hip):
        # packed[t, s, 16*g + c, :] = row (16t + c), dims 32s + 8g .. +8 — the A
        # operand of one v_mfma_f32_16x16x32_bf16, so every wave load of the scan is
        # 1 KiB contiguous. Row-major access goes through read_rows()/write_rows().
        if self.dim % (64 if self.storage == "q16" else 32):
            raise ValueError(f"index dim {self.dim} must be a multiple of {64 if self.storage == 'q16' else 32}")
        tiles = (cap + 15) // 16
        if self.storage == "q16":
            # hi / lo planes, fragment-major for v_mfma_i32_16x16x64_i8 (ops.q16_pack), and per row
            # (scale, stage-1 error bound factor)
            self.packed = None
            self.hi = torch.zeros(tiles, self.dim // 64, 64, 16, dtype=torch.int8, device=d)
            self.lo = torch.zeros(tiles, self.dim // 64, 64, 16, dtype=torch.int8, device=d)
            self.rmeta = torch.zeros(cap, 2, dtype=torch.float32, device=d)
        else:
            self.packed = torch.zeros(tiles, self.dim // 32, 64, 8, dtype=torch.bfloat16, device=d)
        self.priority = torch.full((cap,), -(1 << 30), dtype=torch.int32, device=d)
        self.tagbits = torch.zeros(cap, dtype=torch.int64, device=d)
        self.expiry = torch.zeros(cap, dtype=torch.float32, device=d)

    def _grow(self, need: int):
        new = self.capacity
        while new < need:
            new *= 2
        new = min(new, self.max_capacity)
        if new <= self.capacity:
            return
        old_planes = self._planes()
        old = (self.priority, self.tagbits, self.expiry, self.capacity)
        old_rmeta = getattr(self, "rmeta", None)
        self._alloc(new)
        n = old[3]
        for (_, dst), (_, src) in zip(self._planes(), old_planes):
            dst[:src.shape[0]] = src
        self.priority[:n] = old[0]
        self.tagbits[:n] = old[1]
        self.expiry[:n] = old[2]
        if old_rmeta is not None:
            self.rmeta[:n] = old_rmeta
        if self.device.type == "cuda":
            # the copies above may be queued on the index's side stream (add() runs _grow under
            # _stream_ctx) while the old blocks were allocated on another stream: keep them out
            # of the caching allocator until the copies reading them are done
            cur = torch.cuda.current_stream(self.device)
            for t in [p for _, p in old_planes] + list(old[:3]) + ([old_rmeta] if old_rmeta is not None else []):
                t.record_stream(cur)

    def _planes(self):
        """(name, tile tensor) of the row storage: what a checkpoint writes and _grow copies."""
        if self.storage == "q16":
            return [("hi", self.hi), ("lo", self.lo)]
        return [("packed", self.packed)]

    @property
    def count(self) -> int:
        return min(self.size, self.capacity)

    # -- row-major views of the packed storage ------------------------------------
    def _p5(self) -> torch.Tensor:
        return self.packed.view(self.packed.shape[0], self.dim // 32, 4, 16, 8)

    def write_rows(self, rows: torch.Tensor, vals: torch.Tensor):
        """Scatter row-major `vals` [n, dim] into rows `rows` (long tensor)."""
        rows = rows.to(self.device)
        if self.storage == "q16":
            hi, lo, sc, bd = ops.q16_quantize(vals.to(self.device))
            DS = self.dim // 64
            for plane, part in ((self.hi, hi), (self.lo, lo)):
                plane.view(plane.shape[0], DS, 4, 16, 16)[rows // 16, :, :, rows % 16, :] = part.view(-1, DS, 4, 16)
            self.rmeta[rows] = torch.stack([sc, bd], 1)
            return
        v = vals.to(self.device, torch.bfloat16).reshape(-1, self.dim // 32, 4, 8)
        self._p5()[rows // 16, :, :, rows % 16, :] = v

    def write_range(self, r0: int, vals: torch.Tensor):
        """Rows r0 .. r0 + len(vals): whole tiles move as one permuted copy."""
        m = int(vals.shape[0])
        if m == 0:
            return
        if self.storage == "q16" and r0 % 16 == 0 and m % 16 == 0:
            hi, lo, sc, bd = ops.q16_quantize(vals.to(self.device))
            self.hi[r0 // 16:(r0 + m) // 16].copy_(ops.q16_pack(hi))
            self.lo[r0 // 16:(r0 + m) // 16].copy_(ops.q16_pack(lo))
            self.rmeta[r0:r0 + m].copy_(torch.stack([sc, bd], 1))
        elif self.storage == "q16":
            self.write_rows(torch.arange(r0, r0 + m, device=self.device), vals)
        elif r0 % 16 == 0 and m % 16 == 0:
            v = vals.to(self.device, torch.bfloat16).reshape(m // 16, 16, self.dim // 32, 4, 8)
            self.packed[r0 // 16:(r0 + m) // 16].view(m // 16, self.dim // 32, 4, 16, 8).copy_(
                v.permute(0, 2, 3, 1, 4))
        else:
            self.write_rows(torch.arange(r0, r0 + m, device=self.device), vals)

    def read_rows(self, r0: int, r1: int) -> torch.Tensor:
        """Row-major copy of rows [r0, r1) as [r1 - r0, dim] bf16 (q16: the dequantised fp32 rows)."""
        t0, t1 = r0 // 16, (r1 + 15) // 16
        if self.storage == "q16":
            v = 256 * ops.q16_unpack(self.hi[t0:t1]).float() + ops.q16_unpack(self.lo[t0:t1]).float()
            return v[r0 - 16 * t0:r1 - 16 * t0] * self.rmeta[r0:r1, :1]
        blk = self._p5()[t0:t1].permute(0, 3, 1, 2, 4).reshape((t1 - t0) * 16, self.dim)
        return blk[r0 - 16 * t0:r1 - 16 * t0]

    def row(self, r: int) -> torch.Tensor:
        return self.read_rows(r, r + 1)[0]

    def now(self) -> float:
        return time.time() - self.epoch

    def add(self, vectors, priorities: Sequence[int], tags: Sequence[Iterable[str]],
            expires_at: Sequence[Optional[float]]) -> List[int]:
        """Append rows; returns their row ids. `expires_at` is wall-clock time.time() or None."""
        v = torch.as_tensor(np.asarray(vectors, dtype=np.float32))
        n = v.shape[0]
        # on the index's stream: the host copies below wait for earlier passes only, never
        # for engine steps queued on the device's default stream
        with self._lock, self._stream_ctx():
            if self.growable and self.size + n > self.capacity and self.capacity < self.max_capacity:
                self._grow(self.size + n)
            rows = [(self.size + i) % self.capacity for i in range(n)]
            self.size += n
            idx = torch.tensor(rows, dtype=torch.long, device=self.device)
            v = torch.nn.functional.normalize(v, dim=1)
            self.write_rows(idx, v.to(self.device, torch.bfloat16))
            self.priority.index_copy_(0, idx, torch.tensor(list(priorities), dtype=torch.int32, device=self.device))
            masks = []
            for r, ts in zip(rows, tags):
                ts = frozenset(ts or ())
                m, exact = self.tags.mask(ts)
                if exact:
                    self.row_tags_py.pop(r, None)  # recoverable from the bitmask
                else:
                    self.row_tags_py[r] = ts       # only rows using the shared overflow bit
                masks.append(m)
            self.tagbits.index_copy_(0, idx, torch.tensor(masks, dtype=torch.int64, device=self.device))
            exp = [0.0 if e is None else max(1e-3, float(e) - self.epoch) for e in expires_at]
            self.expiry.index_copy_(0, idx, torch.tensor(exp, dtype=torch.float32, device=self.device))
        return rows

    def add_device(self, vectors: torch.Tensor, priorities: torch.Tensor, tag_masks: torch.Tensor,
                   expiry: Optional[torch.Tensor] = None, normalized: bool = False) -> Tuple[int, int]:
        """Bulk append from device tensors (no host round trip) — how a 100M-row
        store is filled. `tag_masks` are bit masks over tags already registered in
        `self.tags` (bits 0..62); `expiry` is on the index clock (0 = never).
        Returns (first_row, n); rows wrap around the ring."""
        n = int(vectors.shape[0])
        if n == 0:
            return self.size % self.capacity, 0
        with self._lock:
            if self.growable and self.size + n > self.capacity and self.capacity < self.max_capacity:
                self._grow(self.size + n)
            start = self.size % self.capacity
            self.size += n
            v = vectors.to(self.device)
            if not normalized:
                v = torch.nn.functional.normalize(v.float(), dim=1)
            done = 0
            while done < n:
                r0 = (start + done) % self.capacity
                m = min(n - done, self.capacity - r0)
                sl = slice(r0, r0 + m)
                self.write_range(r0, v[done:done + m])
                self.priority[sl].copy_(priorities[done:done + m])
                self.tagbits[sl].copy_(tag_masks[done:done + m])
                if expiry is None:
                    self.expiry[sl].zero_()
                else:
                    self.expiry[sl].copy_(expiry[done:done + m])
                for r in [k for k in self.row_tags_py if r0 <= k < r0 + m]:
                    self.row_tags_py.pop(r)
                done += m
        return start, n

    def _row_tags(self, row: int) -> frozenset:
        ts = self.row_tags_py.get(row)
        if ts is not None:
            return ts
        with self._stream_ctx():
            bits = int(self.tagbits[row].item())
        return frozenset(t for t, b in self.tags.bits.items() if (bits >> b) & 1)

    def delete(self, rows: Sequence[int]):
        with self._lock, self._stream_ctx():
            idx = torch.tensor(list(rows), dtype=torch.long, device=self.device)
            self.priority.index_fill_(0, idx, -(1 << 30))
            for r in rows:
                self.row_tags_py.pop(r, None)

    def query_masks(self, tags: Sequence[Iterable[str]]) -> Tuple[List[int], List[bool]]:
        """Per query (tag bitmask, exact); an unknown tag gives the -1 sentinel (all bits set),
        which no real row mask can contain."""
        tags = list(tags)
        if not any(tags):  # no tag filter anywhere (the common lookup): nothing to map
            return [0] * len(tags), [True] * len(tags)
        qmasks, exact = [], []
        for ts in tags:
            m, ex = self.tags.mask(frozenset(ts or ()), create=False)
            qmasks.append(m)
            exact.append(ex)
        return qmasks, exact

    def search_tensors(self, q: torch.Tensor, k: int, min_priority, qmasks,
                       now: Optional[float] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """The raw kernel pass: `q` [Q, dim] (any device, any float dtype), `min_priority` and
        `qmasks` lists or int tensors. Returns device tensors (scores [Q, k] fp32, rows [Q, k]
        int32, -1 past the hits), best first, on the index's stream (which the caller must
        order against: synchronize it or read the result inside `_stream_ctx`). Tag filters
        on the shared overflow bit are NOT re-checked here (see `search`)."""
        k = max(1, min(int(k), 64))
        caller = torch.cuda.current_stream(self.device) if q.is_cuda and self.device.type == "cuda" else None
        with self._lock, self._stream_ctx():
            if caller is not None:  # `q` was produced on the caller's stream
                torch.cuda.current_stream(self.device).wait_stream(caller)
            qd = torch.nn.functional.normalize(q.to(self.device, torch.float32), dim=1)
            if self.storage != "q16":  # q16 quantises the fp32 query itself (16-bit fixed point)
                qd = qd.to(torch.bfloat16)
            minp = torch.as_tensor(min_priority, dtype=torch.int32).to(self.device)
            qt = torch.as_tensor(qmasks, dtype=torch.int64).to(self.device)
            ev = None
            if self.pass_events is not None and self.device.type == "cuda":
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            t_now = self.now() if now is None else now - self.epoch
            if self.storage == "q16":
                s, r = ops.q16_topk(qd, self.hi, self.lo, self.rmeta, self.count, k, self.priority,
                                    self.tagbits, self.expiry, minp, qt, t_now, workspace=self._ws, stats=self.stats)
            else:
                s, r = ops.cosine_topk(qd, self.packed, self.count, k, self.priority, self.tagbits, self.expiry, minp,
                                       qt, t_now, workspace=self._ws)
            if ev is not None:
                ev[1].record()
                self.pass_events.append(ev)
        return s, r

    def search(self, queries, k: int, min_priority: Sequence[int], tags: Sequence[Iterable[str]],
               now: Optional[float] = None) -> List[List[Tuple[int, float]]]:
        """Batched filtered top-k: returns per query [(row, score), ...] best first."""
        q = queries if isinstance(queries, torch.Tensor) else torch.as_tensor(np.asarray(queries, dtype=np.float32))
        Q = q.shape[0]
        if Q == 0:
            return []
        k = max(1, min(int(k), 64))
        tag_sets = [frozenset(t or ()) for t in tags]
        qmasks, exact = self.query_masks(tag_sets)
        if self.count == 0:
            return [[] for _ in range(Q)]
        kk = k if all(exact) else min(64, 4 * k)
        s, r = self.search_tensors(q, kk, list(min_priority), qmasks, now)
        with self._stream_ctx():
            s, r = s.cpu().numpy(), r.cpu().numpy()
        out = []
        for i in range(Q):
            res = []
            for row, sc in zip(r[i], s[i]):
                if row < 0:
                    break
                if not exact[i] and not tag_sets[i] <= self._row_tags(int(row)):
                    continue
                res.append((int(row), float(sc)))
                if len(res) >= k:
                    break
            out.append(res)
        return out

    def _stream_ctx(self):
        """Searches run on the index's own HIP stream (non-blocking w.r.t. the engine's):
        co-resident with a serving engine, a lookup pass overlaps the engine's step
        instead of queueing behind its graph, and waiting for the result syncs only
        this stream. Also pins the calling thread to the index's device."""
        import contextlib

        if self.device.type != "cuda":
            return contextlib.nullcontext()
        if self._stream is None:
            # high priority: a lookup pass is on an agent step's critical path, and at
            # normal priority its workgroups wait behind the engine's (10M rows: 36 ms
            # per pass beside a 64-worker engine vs ~4 ms alone)
            self._stream = torch.cuda.Stream(device=self.device, priority=-1)
        st = contextlib.ExitStack()
        st.enter_context(torch.cuda.device(self.device))
        st.enter_context(torch.cuda.stream(self._stream))
        return st

    def memory_bytes(self) -> int:
        rows = sum(p.numel() * p.element_size() for _, p in self._planes())
        return rows + self.capacity * (4 + 8 + 4 + (8 if self.storage == "q16" else 0))

    # -- checkpoint / resume (the embedding matrix as per-GPU binary shards
    # next to the JSON metadata; reference item form pilott/memory/enhanced_memory.py:9-21) --
    CKPT_VERSION = 1

    def save(self, path, chunk_bytes: int = 256 << 20) -> Dict[str, float]:
        """Write the index to directory `path`: packed.npy (the fragment-major bf16 tiles as
        uint16, exactly the device layout), priority.npy / tagbits.npy / expiry.npy (per-row
        filter metadata) and meta.json (dims, ring position, clock epoch, tag registry, the
        overflow-tag rows). Rows leave the device in `chunk_bytes` pieces through one pinned
        staging buffer straight into the .npy files (np.lib.format.open_memmap): no
        whole-index host copy, so a 200 GB store needs only the staging buffer of host RAM.
        Files go to a temp directory renamed into place. Returns timings (s) and bytes."""
        import json
        import os
        import shutil
        import tempfile
        from pathlib import Path

        t0 = time.perf_counter()
        path = Path(path)
        path.parent.mkdir(parents=True, exist_ok=True)
        tmp = Path(tempfile.mkdtemp(prefix=".idx-", dir=str(path.parent)))
        with self._lock:
            n = self.count
            tiles = (n + 15) // 16
            tile_bytes = 0
            for name, plane in self._planes():  # bf16: packed.npy (uint16); q16: hi.npy / lo.npy (int8)
                raw = plane.view(torch.int16) if plane.dtype == torch.bfloat16 else plane
                npdt = np.uint16 if plane.dtype == torch.bfloat16 else np.int8
                pb = int(np.prod(plane.shape[1:])) * plane.element_size()
                tile_bytes += pb
                per = max(1, chunk_bytes // pb)
                out = np.lib.format.open_memmap(tmp / f"{name}.npy", mode="w+", dtype=npdt,
                                                shape=(tiles,) + tuple(plane.shape[1:]))
                stage = None
                for t in range(0, tiles, per):
                    m = min(per, tiles - t)
                    src = raw[t:t + m]
                    if self.device.type == "cuda":
                        if stage is None:
                            stage = torch.empty((per,) + tuple(src.shape[1:]), dtype=raw.dtype, pin_memory=True)
                        stage[:m].copy_(src)  # synchronous D2H into pinned memory
                        out[t:t + m] = stage[:m].numpy().view(npdt)
                    else:
                        out[t:t + m] = src.numpy().view(npdt)
                out.flush()
                del out
            rowarrs = [("priority", self.priority, np.int32), ("tagbits", self.tagbits, np.int64),
                       ("expiry", self.expiry, np.float32)]
            if self.storage == "q16":
                rowarrs.append(("rmeta", self.rmeta, np.float32))
            for name, ten, npdt in rowarrs:
                arr = np.lib.format.open_memmap(tmp / f"{name}.npy", mode="w+", dtype=npdt,
                                                shape=(n,) + tuple(ten.shape[1:]))
                rows = max(1, chunk_bytes // 8)
                for r in range(0, n, rows):
                    arr[r:r + rows] = ten[r:min(n, r + rows)].cpu().numpy()
                arr.flush()
                del arr
            meta = {"version": self.CKPT_VERSION, "storage": self.storage, "dim": self.dim, "count": n, "size": self.size,
                    "capacity": self.capacity, "epoch": self.epoch, "tags": self.tags.bits,
                    "row_tags": {str(k): sorted(v) for k, v in self.row_tags_py.items()}}
        (tmp / "meta.json").write_text(json.dumps(meta))
        if path.exists():
            shutil.rmtree(path)
        os.replace(tmp, path)
        secs = time.perf_counter() - t0
        nbytes = tiles * tile_bytes + n * 16
        return {"rows": n, "bytes": nbytes, "seconds": secs, "GBps": nbytes / max(secs, 1e-9) / 1e9}

    @classmethod
    def load(cls, path, device=None, capacity: Optional[int] = None, growable: bool = True,
             max_capacity: Optional[int] = None, chunk_bytes: int = 256 << 20) -> "SemanticIndex":
        """Restore an index written by save(): the packed tiles go from the memory-mapped .npy to
        the device in `chunk_bytes` pieces through a pinned staging buffer (no whole-index host
        copy, no re-embedding); row ids, ring position, clock epoch and tags are preserved, so
        MemoryItems that recorded their row (EnhancedMemory.to_dict) re-attach directly.
        Only .npy (allow_pickle=False) and JSON are read."""
        import json
        from pathlib import Path

        path = Path(path)
        meta = json.loads((path / "meta.json").read_text())
        if meta.get("version") != cls.CKPT_VERSION:
            raise ValueError(f"unsupported index checkpoint version {meta.get('version')}")
        n, dim = int(meta["count"]), int(meta["dim"])
        cap = max(int(capacity or meta["capacity"]), n, 1)
        if int(meta["size"]) > int(meta["capacity"]) and cap != int(meta["capacity"]):
            # a wrapped ring: its write position is size % capacity and every row is live; under
            # another capacity that position moves and count would take in never-written rows
            raise ValueError(f"index checkpoint is a wrapped ring of capacity {meta['capacity']}: "
                             f"it can only be restored at that capacity, not {cap}")
        idx = cls(dim=dim, capacity=cap, device=device, growable=growable,
                  max_capacity=max_capacity or max(cap, int(meta["capacity"])), storage=meta.get("storage", "bf16"))
        for name, plane in idx._planes():
            arr = np.load(path / f"{name}.npy", mmap_mode="r", allow_pickle=False)
            tiles = arr.shape[0]
            if tiles != (n + 15) // 16 or arr.shape[1:] != tuple(plane.shape[1:]):
                raise ValueError(f"index checkpoint {name}.npy does not match meta.json")
            raw = plane.view(torch.int16) if plane.dtype == torch.bfloat16 else plane
            npdt = np.int16 if plane.dtype == torch.bfloat16 else np.int8
            per = max(1, chunk_bytes // (int(np.prod(plane.shape[1:])) * plane.element_size()))
            stage = None
            for t in range(0, tiles, per):
                m = min(per, tiles - t)
                host = torch.from_numpy(np.array(arr[t:t + m]).view(npdt))
                if idx.device.type == "cuda":
                    if stage is None:
                        stage = torch.empty((per,) + tuple(host.shape[1:]), dtype=raw.dtype, pin_memory=True)
                    stage[:m].copy_(host)
                    raw[t:t + m].copy_(stage[:m], non_blocking=False)
                else:
                    raw[t:t + m].copy_(host)
        rowarrs = [("priority", idx.priority), ("tagbits", idx.tagbits), ("expiry", idx.expiry)]
        if idx.storage == "q16":
            rowarrs.append(("rmeta", idx.rmeta))
        for name, ten in rowarrs:
            arr = np.load(path / f"{name}.npy", mmap_mode="r", allow_pickle=False)
            if arr.shape != (n,) + tuple(ten.shape[1:]):
                raise ValueError(f"index checkpoint {name}.npy has {arr.shape}, expected ({n},)")
            rows = max(1, chunk_bytes // 8)
            for r in range(0, n, rows):
                ten[r:min(n, r + rows)].copy_(torch.from_numpy(np.array(arr[r:r + rows])))
        idx.size = int(meta["size"])
        idx.epoch = float(meta["epoch"])
        idx.tags.bits = {str(k): int(v) for k, v in meta["tags"].items()}
        idx.row_tags_py = {int(k): frozenset(v) for k, v in meta["row_tags"].items()}
        if idx.device.type == "cuda":
            torch.cuda.synchronize(idx.device)
        return idx


class ShardedSemanticIndex:
    """Row-sharded index over the ranks of a process group (one shard per GPU).

    Inserts go to the local shard (global row = local_row * world + rank); a
    search runs the local top-k and merges all ranks' candidates with one
    all-gather. All ranks must call `search` collectively with the same queries.
    """

    def __init__(self, local: SemanticIndex, group=None):
        import torch.distributed as dist

        self.local = local
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1

    def save(self, path, **kw) -> Dict[str, float]:
        """Each rank writes its own shard (path/shard_<rank>): per-GPU binary shards."""
        from pathlib import Path

        return self.local.save(Path(path) / f"shard_{self.rank}", **kw)

    @classmethod
    def load(cls, path, group=None, device=None, **kw) -> "ShardedSemanticIndex":
        import torch.distributed as dist
        from pathlib import Path

        rank = dist.get_rank(group) if dist.is_initialized() else 0
        return cls(SemanticIndex.load(Path(path) / f"shard_{rank}", device=device, **kw), group)

    def add_local(self, *a, **kw) -> List[int]:
        return [r * self.world + self.rank for r in self.local.add(*a, **kw)]

    def search(self, queries, k: int, min_priority, tags, now=None) -> List[List[Tuple[int, float]]]:
        import torch.distributed as dist

        res = self.local.search(queries, k, min_priority, tags, now)
        if self.world == 1:
            return res
        Q = len(res)
        t = torch.full((Q, k, 2), -1.0, dtype=torch.float64)
        for i, lst in enumerate(res):
            for j, (row, sc) in enumerate(lst[:k]):
                t[i, j, 0] = row * self.world + self.rank
                t[i, j, 1] = sc
        dev = self.local.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
        t = t.to(dev)
        # output concatenated along dim 0 (the form both gloo and RCCL accept)
        flat = torch.empty((self.world * Q,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
        dist.all_gather_into_tensor(flat, t, group=self.group)
        allt = flat.view((self.world,) + tuple(t.shape)).cpu()
        out = []
        for i in range(Q):
            cand = allt[:, i].reshape(-1, 2)
            cand = cand[cand[:, 0] >= 0]
            order = torch.argsort(cand[:, 1], descending=True)[:k]
            out.append([(int(cand[j, 0]), float(cand[j, 1])) for j in order])
        return out

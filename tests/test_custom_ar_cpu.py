"""Custom all-reduce setup protocol and TP routing on CPU (gloo, world_size 2).

The kernel itself is covered by tests/test_custom_ar_gpu.py. Here the native
allocator is replaced by a fake so the collective setup can run without a GPU:
* setup is all-or-nothing — one rank failing to allocate or to map a peer makes
  EVERY rank fall back to RCCL (a mix would deadlock), and the ranks that did
  allocate release their buffers;
* on success each rank keeps its own pointer and maps every peer's handle;
* TPGroup.all_reduce sends eligible tensors to the custom path, others to dist.
"""
import json
import os
import socket

import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _FakeNative:
    def __init__(self, rank, fail_alloc=False, fail_open=False):
        self.rank, self.fail_alloc, self.fail_open = rank, fail_alloc, fail_open
        self.freed, self.closed, self.opened = [], [], []

    def car_group(self):
        return 128

    def car_flag_bytes(self):
        return 65536

    def car_alloc(self, nbytes):
        if self.fail_alloc:
            raise RuntimeError("car_alloc: uncached IPC allocation failed")
        return 1000 + self.rank, bytes([self.rank]) * 64

    def car_open(self, handle):
        if self.fail_open:
            raise RuntimeError("car_open: hipIpcOpenMemHandle failed")
        p = 5000 + handle[0]
        self.opened.append(p)
        return p

    def car_close(self, p):
        self.closed.append(p)
        return 0

    def car_free(self, p):
        self.freed.append(p)
        return 0


def _worker(rank, world, port, out, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from pilottai_amd.parallel import custom_ar
    from pilottai_amd.parallel.comm import init_distributed

    init_distributed("gloo")
    fake = _FakeNative(rank, fail_alloc=(mode == "alloc" and rank == 1), fail_open=(mode == "open" and rank == 0))
    custom_ar._native = lambda: fake
    car = custom_ar.CustomAllReduce.create(dist.group.WORLD, rank, world, torch.device("cpu"), cap_bytes=1 << 20)
    res = {"created": car is not None, "freed": fake.freed, "closed": fake.closed, "opened": fake.opened}
    if car is not None:
        res["bases"] = car.bases
    dist.destroy_process_group()
    with open(f"{out}.{rank}", "w") as f:
        json.dump(res, f)


def _run(tmp_path, mode):
    out = str(tmp_path / "car")
    mp.start_processes(_worker, args=(2, _port(), out, mode), nprocs=2, join=True, start_method="spawn")
    return [json.load(open(f"{out}.{r}")) for r in range(2)]


def test_custom_ar_setup_maps_every_peer(tmp_path):
    r0, r1 = _run(tmp_path, "ok")
    assert r0["created"] and r1["created"]
    assert r0["bases"] == [1000, 5001] and r1["bases"] == [5000, 1001]


def test_custom_ar_setup_is_all_or_nothing_on_alloc_failure(tmp_path):
    r0, r1 = _run(tmp_path, "alloc")
    assert not r0["created"] and not r1["created"]
    assert r0["freed"] == [1000]  # rank 0 allocated, then released its buffer


def test_custom_ar_setup_is_all_or_nothing_on_open_failure(tmp_path):
    r0, r1 = _run(tmp_path, "open")
    assert not r0["created"] and not r1["created"]
    assert r0["freed"] == [1000] and r1["freed"] == [1001]
    assert r1["closed"] == r1["opened"] == [5000]  # the mapping rank 1 did make is unmapped


def test_tp_group_routes_eligible_tensors_to_custom(monkeypatch):
    import torch.distributed as dist

    from pilottai_amd.parallel.comm import TPGroup

    calls = []

    class _Custom:
        def eligible(self, t):
            return t.numel() <= 8

        def all_reduce(self, t):
            calls.append(("custom", t.numel()))
            return t

    monkeypatch.setattr(dist, "all_reduce", lambda t, group=None: calls.append(("dist", t.numel())))
    tp = TPGroup(group=None, rank=0, size=2, custom=_Custom())
    tp.all_reduce(torch.zeros(8))
    tp.all_reduce(torch.zeros(16))
    assert calls == [("custom", 8), ("dist", 16)]
    assert TPGroup.single().all_reduce(torch.ones(4)).sum() == 4  # size 1: no collective at all

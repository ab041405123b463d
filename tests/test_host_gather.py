"""Shared-memory host all-gather (parallel/host_gather.py over csrc/runtime/shm_ring.cpp
`ShmGather`): payloads of different sizes per rank, payloads spanning several slots, the
two-bank reuse over many rounds, the all-to-all read, and the gloo fallback giving the same."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, world, port, force_gloo, q):
    import torch.distributed as dist

    from pilottai_amd.parallel.host_gather import HostGather

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hg = HostGather(None, slot_bytes=256, force_gloo=force_gloo)
        out = {"transport": hg.transport}
        # 50 rounds of varied sizes: 0 bytes .. several slots
        res = []
        for i in range(50):
            n = (rank * 97 + i * 131) % 900
            res.append([len(b) == (r * 97 + i * 131) % 900 and b == bytes([(r + i) % 256]) * len(b)
                        for r, b in enumerate(hg.gather_bytes(bytes([(rank + i) % 256]) * n))])
        out["bytes_ok"] = all(all(x) for x in res)
        out["objs"] = hg.gather_obj({"rank": rank, "text": "x" * (rank * 300)})
        a = np.arange(world * 5, dtype=np.int64).reshape(world, 5) + 1000 * rank
        out["a2a"] = hg.all_to_all_array(a).tolist()
        out["arr"] = hg.gather_array(np.full((3, 2), rank, np.float32)).tolist()
        q.put((rank, out))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,force_gloo", [(2, False), (3, False), (3, True)])
def test_host_gather(world, force_gloo):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_entry, args=(r, world, port, force_gloo, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for r in range(world):
        o = got[r]
        assert o["transport"] == ("gloo" if force_gloo else "shm")
        assert o["bytes_ok"]
        assert o["objs"] == [{"rank": s, "text": "x" * (s * 300)} for s in range(world)]
        assert o["a2a"] == [[1000 * s + r * 5 + j for j in range(5)] for s in range(world)]
        assert o["arr"] == [[[float(s)] * 2] * 3 for s in range(world)]

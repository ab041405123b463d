"""Agent-DP global load view over 2 and 4 gloo ranks (§4.4 world-size parametrisation)."""
import json
import os
import socket

import pytest
import torch.multiprocessing as mp

from pilottai_amd.parallel.agent_dp import shard_workers


def test_shard_workers_covers_all():
    for n, w in ((64, 8), (64, 3), (5, 8)):
        shards = [list(shard_workers(n, w, r)) for r in range(w)]
        assert sum(shards, []) == list(range(n))
        assert max(map(len, shards)) - min(map(len, shards)) <= 1


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch

    from pilottai_amd.parallel.agent_dp import GlobalLoadView
    from pilottai_amd.parallel.comm import init_distributed

    init_distributed("gloo")
    view = GlobalLoadView()
    view.update([5.0 - 4 * rank, 2.0, 1.0, 0.1 * rank, 1000.0])
    with open(f"{out}.{rank}", "w") as f:
        json.dump({"table": view.table, "least": view.least_loaded_rank(), "totals": view.totals()}, f)
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_global_load_view_ranks(tmp_path, world):
    out = str(tmp_path / "load")
    mp.start_processes(_worker, args=(world, _port(), out), nprocs=world, join=True, start_method="spawn")
    res = [json.load(open(f"{out}.{r}")) for r in range(world)]
    assert all(r == res[0] for r in res)  # every rank holds the same global view
    # queue sizes 5 - 4r: the last rank has the smallest (most negative) load
    assert res[0]["least"] == world - 1 and len(res[0]["table"]) == world
    assert res[0]["totals"]["queue_size"] == sum(5.0 - 4 * r for r in range(world))

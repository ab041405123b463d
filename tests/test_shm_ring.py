"""Shared-memory header ring (csrc/runtime/shm_ring.cpp): the TP driver -> follower step
header of the engine, multi-process on the CPU."""
import multiprocessing as mp
import os
import time

import pytest

from pilottai_amd import _runtime as R


def _consumer(name, idx, n, q, slow):
    r = R.ShmRing(name, 9, 4, 2, False, 30.0)
    got = []
    for _ in range(n):
        rec = r.get(idx, 30.0)
        got.append(rec)
        if slow:
            time.sleep(0.001)  # the producer must block on this consumer, never overwrite
    q.put((idx, got))


@pytest.mark.parametrize("slow", [False, True])
def test_ring_delivers_every_record_in_order_to_every_consumer(slow):
    name = f"pa_ring_test_{os.getpid()}_{int(slow)}"
    ctx = mp.get_context("spawn")
    prod = R.ShmRing(name, 9, 4, 2, True)
    q = ctx.Queue()
    n = 200
    ps = [ctx.Process(target=_consumer, args=(name, i, n, q, slow and i == 1)) for i in range(2)]
    for p in ps:
        p.start()
    for k in range(n):
        assert prod.put([k, 2 * k, 0, 0, 0, 0, 0, 0, -k], 30.0)
    res = dict(q.get(timeout=60) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    want = [[k, 2 * k, 0, 0, 0, 0, 0, 0, -k] for k in range(n)]
    assert res[0] == want and res[1] == want
    assert prod.published() == n


def test_ring_timeouts_and_geometry_checks():
    name = f"pa_ring_test_t_{os.getpid()}"
    prod = R.ShmRing(name, 3, 2, 1, True)
    cons = R.ShmRing(name, 3, 2, 1, False, 5.0)
    assert cons.get(0, 0.01) is None  # nothing published yet
    assert prod.put([1, 2, 3], 1.0) and prod.put([4, 5, 6], 1.0)
    assert not prod.put([7, 8, 9], 0.05)  # ring full: the consumer has read nothing
    assert cons.get(0, 1.0) == [1, 2, 3]
    assert prod.put([7, 8, 9], 1.0)
    assert cons.get(0, 1.0) == [4, 5, 6] and cons.get(0, 1.0) == [7, 8, 9]
    with pytest.raises(Exception):
        R.ShmRing(name, 4, 2, 1, False, 1.0)  # geometry mismatch
    with pytest.raises(Exception):
        prod.put([1, 2], 1.0)  # record length

"""Two-stage exact top-k over the 16-bit fixed-point index (csrc/ops/similarity_q16.hip) on
the GPU against the CPU reference (ops.reference.q16_topk: exact int64 dot products, the same
float64 -> float32 step): identical rows and bit-identical scores, on random and planted sets,
with the priority / tag / expiry filters, one and many slices, and the exact-scan fallback."""
import pytest
import torch

from pilottai_amd import ops
from pilottai_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _index(N, D, gpu, seed=0, planted=None):
    g = torch.Generator(device=gpu).manual_seed(seed)
    x = torch.randn(N, D, device=gpu, generator=g)
    if planted is not None:
        for row, q in planted:
            x[row] = q + 0.05 * torch.randn(D, device=gpu, generator=g)
    x = torch.nn.functional.normalize(x, dim=1)
    pad = (-N) % 16
    hi, lo, sc, bd = ops.q16_quantize(torch.cat([x, torch.zeros(pad, D, device=gpu)]) if pad else x)
    rmeta = torch.stack([sc, bd], 1).contiguous()
    return ops.q16_pack(hi).contiguous(), ops.q16_pack(lo).contiguous(), rmeta


def _filters(N, Q, gpu, on):
    prio = (torch.arange(N, device=gpu) % 4).to(torch.int32)
    tags = torch.where(torch.arange(N, device=gpu) % 2 == 0, 1, 2).to(torch.int64)
    exp = torch.zeros(N, device=gpu)
    if on:
        exp[torch.arange(N, device=gpu) % 10 == 5] = 1.0  # expired at now = 2
    minp = torch.tensor([(i % 3) if on else 0 for i in range(Q)], dtype=torch.int32, device=gpu)
    qtags = torch.tensor([(1 if i % 4 == 1 else 2 if i % 4 == 3 else 0) if on else 0 for i in range(Q)],
                         dtype=torch.int64, device=gpu)
    return prio, tags, exp, minp, qtags


def _check(gpu, N, D, Q, K, filters, exact=False, seed=0, planted=False):
    g = torch.Generator(device=gpu).manual_seed(seed + 1)
    q = torch.nn.functional.normalize(torch.randn(Q, D, device=gpu, generator=g), dim=1)
    pl = [(int((i * 7919 + 13) % N), q[i]) for i in range(Q)] if planted else None
    hi, lo, rmeta = _index(N, D, gpu, seed, pl)
    prio, tags, exp, minp, qtags = _filters(N, Q, gpu, filters)
    stats = {}
    s, r = ops.q16_topk(q, hi, lo, rmeta, N, K, prio, tags, exp, minp, qtags, 2.0, exact=exact, stats=stats)
    torch.cuda.synchronize()
    qv, qm = ops.q16_queries(q)
    rs, rr = ref.q16_topk(qv.cpu(), qm.cpu(), hi.cpu(), lo.cpu(), rmeta.cpu(), N, K, prio.cpu(), tags.cpu(),
                          exp.cpu(), minp.cpu(), qtags.cpu(), 2.0)
    assert torch.equal(r.cpu(), rr), (r.cpu()[:2], rr[:2])
    assert torch.equal(s.cpu(), rs)
    if planted and not filters:
        assert all(int(r[i, 0]) == pl[i][0] for i in range(Q))
    return stats


@pytest.mark.parametrize("N,D,Q,K,filters", [
    (500, 1024, 1, 1, False), (3000, 1024, 13, 5, True), (50_000, 1024, 64, 64, True),
    (300_000, 1024, 64, 5, False), (300_000, 256, 7, 20, True), (70_001, 512, 33, 3, True)])
def test_q16_two_stage_matches_exact_reference(gpu, N, D, Q, K, filters):
    st = _check(gpu, N, D, Q, K, filters)
    assert st.get("q16_fallbacks", 0) == 0  # random unit vectors: the drop check never fires


@pytest.mark.parametrize("N,Q,K", [(20_000, 16, 5), (200_000, 64, 10)])
def test_q16_exact_scan_matches_reference(gpu, N, Q, K):
    _check(gpu, N, 1024, Q, K, True, exact=True, seed=5)


def test_q16_planted_neighbours_found(gpu):
    _check(gpu, 400_000, 1024, 32, 5, False, seed=7, planted=True)


def test_q16_fallback_on_ties(gpu):
    """Every row the same vector: every slice's list is full of equal upper bounds, the drop
    check fires, and the exact scan answers (same scores as the reference; rows are ties)."""
    N, D, Q, K = 40_000, 1024, 4, 5
    base = torch.nn.functional.normalize(torch.randn(1, D, device=gpu), dim=1).expand(N, D).contiguous()
    hi, lo, sc, bd = ops.q16_quantize(base)
    hi, lo, rmeta = ops.q16_pack(hi), ops.q16_pack(lo), torch.stack([sc, bd], 1).contiguous()
    prio, tags, exp, minp, qtags = _filters(N, Q, gpu, False)
    q = torch.nn.functional.normalize(base[:Q] + 0.01 * torch.randn(Q, D, device=gpu), dim=1)
    stats = {}
    s, r = ops.q16_topk(q, hi, lo, rmeta, N, K, prio, tags, exp, minp, qtags, 2.0, stats=stats)
    qv, qm = ops.q16_queries(q)
    rs, _ = ref.q16_topk(qv.cpu(), qm.cpu(), hi.cpu(), lo.cpu(), rmeta.cpu(), N, K, prio.cpu(), tags.cpu(),
                         exp.cpu(), minp.cpu(), qtags.cpu(), 2.0)
    assert stats.get("q16_fallbacks", 0) == 1
    assert torch.equal(s.cpu(), rs) and bool((r >= 0).all())


def test_q16_semantic_index_on_gpu(gpu):
    """The index front end (storage="q16") on the GPU equals the same index on the CPU."""
    import numpy as np

    from pilottai_amd.memory.semantic_index import SemanticIndex

    g = np.random.default_rng(3)
    v = g.standard_normal((5000, 1024)).astype(np.float32)
    prio = [i % 3 for i in range(5000)]
    tags = [{"a"} if i % 2 else {"b"} for i in range(5000)]
    q = g.standard_normal((9, 1024)).astype(np.float32)
    res = []
    for dev in (gpu, "cpu"):
        idx = SemanticIndex(dim=1024, capacity=1024, device=dev, storage="q16")
        idx.add(v, prio, tags, [None] * 5000)
        res.append(idx.search(q, 7, [0, 1, 2] * 3, [(), ("a",), ("b",)] * 3))
    assert [[r for r, _ in x] for x in res[0]] == [[r for r, _ in x] for x in res[1]]
    # same rows, scores equal up to the last bit of the final fp32 scaling (order of the two scale
    # multiplies differs between the GPU epilogue and the CPU reference)
    for a, b in zip(res[0], res[1]):
        for (_, sa), (_, sb) in zip(a, b):
            assert abs(sa - sb) <= 1e-6 * max(1.0, abs(sb))

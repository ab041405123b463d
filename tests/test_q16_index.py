"""16-bit fixed-point semantic index (memory/semantic_index.py storage="q16",
csrc/ops/similarity_q16.hip) on CPU: the quantisation is exact in its own
terms, the stage-1 error bound holds, and the index's search equals an independent float64
top-k of the dequantised vectors, filters included; checkpoints round-trip."""
import numpy as np
import pytest
import torch

from pilottai_amd import ops
from pilottai_amd.memory.semantic_index import SemanticIndex


def test_q16_quantisation_is_exact_and_bounded():
    g = torch.Generator().manual_seed(0)
    x = torch.nn.functional.normalize(torch.randn(300, 1024, generator=g), dim=1)
    x[3] = 0.0  # an all-zero row stays representable
    hi, lo, sc, bd = ops.q16_quantize(x)
    assert hi.dtype == torch.int8 and int(hi.abs().max()) <= 127 and int(lo.min()) >= -128
    v = 256 * hi.long() + lo.long()
    assert int(v.abs().max()) <= ops.kernels.Q16_MAX
    deq = v.double() * sc.double()[:, None]
    assert float((deq - x.double()).abs().max()) <= float(sc.max()) / 2 + 1e-12  # half a step per coordinate
    # stage-1 bound: |v_q . lo| * s_r * s_q <= c_q * b_r for every (row, query)
    q = torch.nn.functional.normalize(torch.randn(16, 1024, generator=g), dim=1)
    qv, qm = ops.q16_queries(q)
    vq = 256 * qv[:, 0].long() + qv[:, 1].long()
    err = (vq.double() @ lo.double().T).abs() * sc.double()[None, :] * qm[:, 0].double()[:, None]
    assert bool((err <= qm[:, 1].double()[:, None] * bd.double()[None, :] + 1e-12).all())
    # the packing is a bijection onto the MFMA fragment layout
    t = ops.q16_pack(hi[:288])
    assert t.shape == (18, 16, 64, 16)
    assert torch.equal(ops.q16_unpack(t), hi[:288])
    assert int(t[1, 2, 16 * 3 + 5, 7]) == int(hi[16 + 5, 64 * 2 + 16 * 3 + 7])


def _data(n, d=256, seed=1):
    g = np.random.default_rng(seed)
    v = g.standard_normal((n, d)).astype(np.float32)
    prio = [int(i % 4) for i in range(n)]
    tags = [{"even"} if i % 2 == 0 else {"odd"} for i in range(n)]
    exp = [None] * n
    return v, prio, tags, exp


@pytest.mark.parametrize("k", [1, 5, 20])
def test_q16_index_search_equals_float64_topk(k):
    n, d = 1500, 256
    v, prio, tags, exp = _data(n, d)
    idx = SemanticIndex(dim=d, capacity=256, device="cpu", storage="q16")
    idx.add(v, prio, tags, exp)
    assert idx.count == n and idx.capacity >= n
    q = np.random.default_rng(2).standard_normal((6, d)).astype(np.float32)
    qt = [(), ("even",), (), ("odd",), (), ()]
    qp = [0, 0, 2, 1, 0, 3]
    got = idx.search(q, k, qp, qt)
    # independent check: float64 cosine of the dequantised rows and queries
    rows = idx.read_rows(0, n).double().numpy()
    qv, qm = ops.q16_queries(torch.nn.functional.normalize(torch.from_numpy(q), dim=1))
    qd = ((256 * qv[:, 0].double() + qv[:, 1].double()) * qm[:, 0].double()[:, None]).numpy()
    sc = qd @ rows.T
    for i in range(len(q)):
        ok = np.array([prio[r] >= qp[i] and set(qt[i]) <= tags[r] for r in range(n)])
        s = np.where(ok, sc[i], -np.inf)
        want = list(np.argsort(-s, kind="stable")[:k])
        assert [r for r, _ in got[i]] == want
        np.testing.assert_allclose([x for _, x in got[i]], s[want], rtol=1e-6, atol=1e-7)


def test_q16_index_checkpoint_roundtrip(tmp_path):
    n, d = 700, 128
    v, prio, tags, exp = _data(n, d, seed=3)
    idx = SemanticIndex(dim=d, capacity=1024, device="cpu", storage="q16")
    idx.add(v, prio, tags, exp)
    idx.save(tmp_path / "ix")
    back = SemanticIndex.load(tmp_path / "ix", device="cpu")
    assert back.storage == "q16" and back.count == n
    assert torch.equal(back.hi[:(n + 15) // 16], idx.hi[:(n + 15) // 16])
    assert torch.equal(back.lo[:(n + 15) // 16], idx.lo[:(n + 15) // 16])
    assert torch.equal(back.rmeta[:n], idx.rmeta[:n])
    q = np.random.default_rng(4).standard_normal((3, d)).astype(np.float32)
    assert back.search(q, 5, [0, 0, 0], [(), (), ()]) == idx.search(q, 5, [0, 0, 0], [(), (), ()])

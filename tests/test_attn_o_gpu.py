"""Decode-sized steps: attention + O projection + residual in one launch
(csrc/ops/attention.hip attn_o_kernel) vs the two launches it replaces (8-wave paged
attention, packed decode GEMM with the residual epilogue) and vs fp32 references."""
import math

import numpy as np
import pytest
import torch

from pilottai_amd import ops
from pilottai_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _case(gpu, H, KV, q_lens, ctx_lens, part, seed, pad=20):
    torch.manual_seed(seed)
    G = H // KV
    blk = 16
    ns = len(q_lens)
    nbs = [(c + blk - 1) // blk for c in ctx_lens]
    total = sum(nbs) + 4
    kc = (torch.randn(total, KV, 16, blk, 8, device=gpu) * 0.5).to(torch.bfloat16)
    vc = torch.randn(total, KV, 128, blk, device=gpu).to(torch.bfloat16)
    perm = torch.randperm(total).tolist()
    bt = torch.zeros(ns, max(nbs), dtype=torch.int32)
    c = 0
    for s, nb in enumerate(nbs):
        bt[s, :nb] = torch.tensor(perm[c:c + nb], dtype=torch.int32)
        c += nb
    q_start = np.concatenate([[0], np.cumsum(q_lens)[:-1]]).astype(np.int32)
    T = int(sum(q_lens))
    q = torch.randn(T, H, 128, device=gpu).to(torch.bfloat16)
    items, _ = ops.build_attention_items(q_lens, ctx_lens, G, split=True, part=part, qcols=32, wide_min_tokens=0)
    it = torch.tensor(items + [(0, 0, 0, 0)] * pad, dtype=torch.int32, device=gpu)
    n_it = torch.tensor([len(items)], dtype=torch.int32, device=gpu)
    maxit = it.shape[0]
    dev_i = lambda a: torch.tensor(a, dtype=torch.int32, device=gpu)  # noqa: E731
    meta = dict(items=it, n_items=n_it, counters=torch.zeros(ns * KV, dtype=torch.int32, device=gpu),
                q_start=dev_i(q_start), q_len=dev_i(q_lens), ctx_len=dev_i(ctx_lens), block_table=bt.to(gpu),
                scale=1.0 / math.sqrt(128), part_size=dev_i([part]))
    ws = (ops.empty_handoff(maxit * KV * 16 * 128, torch.float32, gpu),
          ops.empty_handoff(maxit * KV * 16 * 2, torch.float32, gpu))
    N = H * 128
    w = (torch.randn(N, H * 128, device=gpu) * 0.02).to(torch.bfloat16)
    h = torch.randn(T, N, device=gpu).to(torch.bfloat16)
    return dict(q=q, kc=kc, vc=vc, meta=meta, ws=ws, w=w, wp=ops.pack_decode_weight(w), h=h, T=T,
                ref_att=ref.paged_attention(q.cpu(), kc.cpu(), vc.cpu(), q_start, q_lens, ctx_lens, bt,
                                            1.0 / math.sqrt(128)).float())


@pytest.mark.parametrize("H,KV,q_lens,ctx,part", [
    (32, 8, [1] * 8, [600, 650, 1, 17, 512, 513, 700, 999], 4096),        # the 8-token decode step
    (32, 8, [1] * 16, list(range(100, 1700, 100)), 4096),                # 16 rows
    (32, 8, [1] * 6 + [3], [5000, 4200, 300, 60, 4097, 8000, 900], 4096),  # split partitions (merge)
    (32, 8, [1, 1, 9, 1], [700, 64, 300, 2000], 4096),                    # a 9-token run (prefill item)
    (32, 8, [1] * 12, [600] * 12, 256),                                   # many small partitions
])
def test_attn_o_matches_two_launches_and_fp32(gpu, H, KV, q_lens, ctx, part):
    c = _case(gpu, H, KV, q_lens, ctx, part, seed=len(ctx) + part)
    m, (po, pm) = c["meta"], c["ws"]
    # two launches (the shipped decode path)
    att2 = torch.zeros(c["T"], H, 128, dtype=torch.bfloat16, device=gpu)
    h2 = c["h"].clone()
    ops.paged_attention(att2, po, pm, c["q"], c["kc"], c["vc"], m["items"], m["n_items"], m["counters"],
                        m["q_start"], m["q_len"], m["ctx_len"], m["block_table"], m["scale"],
                        part_size=m["part_size"], waves=8)
    ops.decode_gemm(att2.view(c["T"], -1), c["wp"], "resid", resid=h2, out=h2)
    # fused, twice (the counters must reset themselves)
    sync, err = ops.attn_o_workspace(gpu)
    for _ in range(2):
        att1 = torch.zeros(c["T"], H, 128, dtype=torch.bfloat16, device=gpu)
        h1 = c["h"].clone()
        assert ops.attn_o(att1, po, pm, c["q"], c["kc"], c["vc"], m["items"], m["n_items"], m["counters"],
                          m["q_start"], m["q_len"], m["ctx_len"], m["block_table"], m["scale"], c["wp"], h1,
                          part_size=m["part_size"])
        torch.cuda.synchronize()
        assert int(err[0]) == 0 and int(sync.abs().sum()) == 0 and int(m["counters"].abs().sum()) == 0
        torch.testing.assert_close(att1.cpu().float(), c["ref_att"], atol=2e-2, rtol=2e-2)
        assert torch.equal(att1, att2)  # the same attention code path
        want = c["h"].float() + att1.view(c["T"], -1).float() @ c["w"].float().T
        torch.testing.assert_close(h1.float(), want, atol=3e-2, rtol=2e-2)
        torch.testing.assert_close(h1.float(), h2.float(), atol=2e-2, rtol=1e-2)


def test_attn_o_in_a_graph_and_refuses_other_shapes(gpu):
    """Graph replay (the counters reset between replays) and a fallback answer (False,
    nothing launched) for a shape the fused launch does not take (O rows > 16)."""
    c = _case(gpu, 32, 8, [1] * 8, [600] * 8, 4096, seed=3)
    m, (po, pm) = c["meta"], c["ws"]
    att = torch.zeros(c["T"], 32, 128, dtype=torch.bfloat16, device=gpu)
    h = c["h"].clone()
    args = (att, po, pm, c["q"], c["kc"], c["vc"], m["items"], m["n_items"], m["counters"], m["q_start"],
            m["q_len"], m["ctx_len"], m["block_table"], m["scale"], c["wp"], h)
    ops.attn_o(*args, part_size=m["part_size"])
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ops.attn_o(*args, part_size=m["part_size"])
    h.copy_(c["h"])
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    sync, err = ops.attn_o_workspace(gpu)
    assert int(err[0]) == 0 and int(sync.abs().sum()) == 0
    want = c["h"].float() + 3 * (att.view(c["T"], -1).float() @ c["w"].float().T)
    torch.testing.assert_close(h.float(), want, atol=6e-2, rtol=3e-2)
    big = torch.zeros(20, 32, 128, dtype=torch.bfloat16, device=gpu)
    assert not ops.attn_o(big, po, pm, torch.zeros_like(big), c["kc"], c["vc"], m["items"], m["n_items"],
                          m["counters"], m["q_start"], m["q_len"], m["ctx_len"], m["block_table"], m["scale"],
                          c["wp"], torch.zeros(20, 4096, dtype=torch.bfloat16, device=gpu), part_size=m["part_size"])

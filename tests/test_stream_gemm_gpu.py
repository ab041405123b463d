"""Weight-streaming packed projections for 16 < M <= 256 (csrc/ops/gemm_stream.hip: exact
~256-workgroup decompositions, weights straight to VGPRs, x through LDS, cooperative
split-K reduction over uncached slabs, fused epilogues) vs fp32 PyTorch references."""
import pytest
import torch

from pilottai_amd import ops
from pilottai_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _bf(*shape, dev, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


def _ref(x, w, epi, norm, resid):
    N = w.shape[0]
    acc = x.float() @ w.float().T
    if norm:
        acc = acc * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-5)
    if epi == "silu":
        acc = torch.nn.functional.silu(acc[:, :N // 2]) * acc[:, N // 2:]
    elif epi == "resid":
        acc = acc + resid.float()
    return acc


def _check(gpu, M, N, K, epi, norm, plan, reps=3, rel=None):
    torch.manual_seed(31 + M)
    x = _bf(M, K, dev=gpu)
    w = _bf(N, K, dev=gpu, scale=0.05)
    resid = _bf(M, N, dev=gpu) if epi == "resid" else None
    pack = {"silu": ops.pack_decode_gate_up, "rope_perm": ops.pack_decode_qkv_rope}.get(epi, ops.pack_decode_weight)
    wp = pack(w)
    want = _ref(x, w, epi, norm, resid)
    _, _, err = ops.stream_workspace(gpu)
    for _ in range(reps):  # the group counters must reset themselves between launches
        y = ops.stream_gemm(x, wp, epi, resid=resid, norm=norm, plan=plan, rel=rel)
        torch.testing.assert_close(y.float(), want, atol=4e-2, rtol=2e-2)
    assert int(err[0]) == 0


# Llama-3-8B projections at the engine's mid-step sizes, default decompositions
@pytest.mark.parametrize("M", [17, 32, 48, 64, 96, 128, 160, 200, 256])
@pytest.mark.parametrize("N,K,epi,norm", [(6144, 4096, "rope_perm", True), (4096, 4096, "resid", False),
                                          (28672, 4096, "silu", True), (4096, 14336, "resid", False)])
def test_stream_gemm_llama8b_default_plans(gpu, M, N, K, epi, norm):
    _check(gpu, M, N, K, epi, norm, None)


# explicit decompositions: every instantiated wave shape, both ring depths, K splits 1-16,
# one and two row groups
@pytest.mark.parametrize("M,N,K,epi,norm,plan", [
    (64, 4096, 4096, "plain", False, (4, 1, 1, 4, 1, 4, 4)),
    (64, 4096, 4096, "plain", True, (4, 1, 2, 4, 1, 8, 2)),
    (40, 6144, 4096, "plain", False, (4, 1, 3, 4, 1, 8, 4)),
    (128, 4096, 4096, "resid", False, (8, 1, 4, 4, 1, 16, 2)),
    (100, 4096, 4096, "plain", False, (8, 1, 1, 4, 2, 4, 4)),
    (33, 4096, 4096, "plain", True, (4, 1, 2, 2, 2, 4, 2)),
    (250, 6144, 4096, "rope_perm", True, (8, 2, 3, 2, 2, 2, 2)),
    (64, 6144, 4096, "plain", False, (4, 1, 1, 6, 1, 4, 4)),
    (64, 6144, 4096, "plain", False, (4, 1, 2, 6, 1, 8, 4)),
    (160, 28672, 4096, "silu", True, (8, 2, 2, 7, 1, 1, 4)),
    (24, 4096, 14336, "resid", False, (2, 1, 2, 8, 1, 7, 4)),
    (200, 4096, 14336, "resid", False, (8, 2, 1, 8, 1, 4, 2)),
    (256, 4096, 14336, "resid", False, (8, 2, 2, 4, 1, 4, 4)),
    (96, 1280, 8192, "rope_perm", True, (8, 1, 2, 4, 1, 8, 2)),  # 70B TP=8 QKV shard
    (48, 128256, 4096, "plain", False, None),  # LM head
    (200, 128256, 4096, "plain", False, None),  # LM head, two row groups, no K split
])
def test_stream_gemm_plans(gpu, M, N, K, epi, norm, plan):
    _check(gpu, M, N, K, epi, norm, plan)


@pytest.mark.parametrize("M,N,K,epi,norm,plan", [
    (64, 6144, 4096, "rope_perm", True, None), (128, 4096, 14336, "resid", False, None),
    (48, 28672, 4096, "silu", True, None), (64, 4096, 4096, "plain", False, (4, 1, 2, 4, 1, 1, 4))])
def test_stream_gemm_rotated_chunk_order(gpu, M, N, K, epi, norm, plan):
    """rel bit 1: every workgroup streams its K slice from a different starting chunk (the
    accumulation order changes, the result must not beyond rounding)."""
    _check(gpu, M, N, K, epi, norm, plan, rel=2 | ops.kernels.STREAM_REL)


def test_stream_gemm_asymmetric_identity(gpu):
    """x = I (rows), W asymmetric: the output must be exactly W^T's rows (catches a transposed
    or permuted C write or a wrong fragment/slice mapping in the reduction)."""
    M, N, K = 128, 1024, 4096
    x = torch.zeros(M, K, device=gpu)
    x[torch.arange(M), (torch.arange(M) * 29) % K] = 1.0
    w = (torch.arange(N * K, device=gpu, dtype=torch.float32).view(N, K) % 251 / 64.0).to(torch.bfloat16)
    for plan in (None, (8, 1, 1, 4, 1, 8, 2), (8, 1, 2, 2, 2, 4, 4)):
        y = ops.stream_gemm(x.to(torch.bfloat16), ops.pack_decode_weight(w), "plain", plan=plan)
        want = w.float().T[(torch.arange(M) * 29) % K]
        assert torch.equal(y.float(), want.to(torch.bfloat16).float()), plan


@pytest.mark.parametrize("M,S", [(64, 4), (128, 8), (256, 4)])
def test_stream_gemm_resid_in_place_with_row_stats(gpu, M, S):
    """h += x W^T in place, accumulating the next norm's row statistics (ss_out) of the written
    bf16 rows and zeroing another buffer (ss_zero); a norm-folded projection consuming them
    matches rmsnorm + GEMM."""
    torch.manual_seed(32)
    N, K = 4096, 4096
    x = _bf(M, K, dev=gpu)
    w = _bf(N, K, dev=gpu, scale=0.05)
    h = _bf(M, N, dev=gpu)
    want = h.float() + x.float() @ w.float().T
    hh = h.clone()
    ss = torch.zeros(M, dtype=torch.float32, device=gpu)
    junk = torch.full((M,), 7.0, device=gpu)
    mg, rg = (8, 2) if M > 128 else ((4, 1) if M <= 64 else (8, 1))
    ops.stream_gemm(x, ops.pack_decode_weight(w), "resid", resid=hh, out=hh, ss_out=ss, ss_zero=junk,
                    plan=(mg, rg, 2, 4, 1, S, 2))
    torch.testing.assert_close(hh.float(), want, atol=4e-2, rtol=2e-2)
    torch.testing.assert_close(ss, hh.float().pow(2).sum(-1), rtol=1e-4, atol=1e-2)
    assert float(junk.abs().max()) == 0.0
    w2 = _bf(2048, N, dev=gpu, scale=0.05)
    g = (torch.rand(N, device=gpu) + 0.5).to(torch.bfloat16)
    wg = w2 * g[None, :]
    y = ops.stream_gemm(hh, ops.pack_decode_weight(wg), norm=True, ss_in=ss)
    xn = hh.float() * torch.rsqrt(hh.float().pow(2).mean(-1, keepdim=True) + 1e-5)
    torch.testing.assert_close(y.float(), xn @ wg.float().T, atol=4e-2, rtol=2e-2)


@pytest.mark.parametrize("M,H,KV,K,plan", [
    (64, 32, 8, 4096, None), (128, 32, 8, 4096, None), (211, 32, 8, 4096, None), (20, 32, 8, 4096, None),
    (96, 8, 1, 8192, (8, 1, 2, 4, 1, 8, 2)),  # 70B TP=8 shard
])
def test_stream_qkv_rope(gpu, M, H, KV, K, plan):
    """Norm-folded QKV with RoPE + paged KV write vs fp32 projection + reference rope_cache."""
    torch.manual_seed(33)
    N = (H + 2 * KV) * 128
    x = _bf(M, K, dev=gpu)
    w = _bf(N, K, dev=gpu, scale=0.05)
    g = (torch.rand(K, device=gpu) + 0.5).to(torch.bfloat16)
    wp = ops.pack_decode_qkv_rope(w * g[None, :])
    NB = (M + 15) // 16 + 4
    cos_sin = ref.rope_cos_sin(4096).to(gpu)
    pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=gpu)
    slots = torch.randperm(NB * 16, device=gpu)[:M].to(torch.int32)
    slots[1] = -1
    kc = torch.zeros(NB, KV, 16, 16, 8, dtype=torch.bfloat16, device=gpu)
    vc = torch.zeros(NB, KV, 128, 16, dtype=torch.bfloat16, device=gpu)
    q = torch.empty(M, H, 128, dtype=torch.bfloat16, device=gpu)
    for _ in range(2):
        ops.stream_qkv_rope(x, wp, 1e-5, q, kc, vc, pos, slots, cos_sin, H, KV, plan=plan)
    xn = x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-5) * g.float()
    qkv = (xn @ w.float().T).cpu()
    rq = torch.empty(M, H, 128, dtype=torch.float32)
    rk = torch.zeros(NB, KV, 16, 16, 8)
    rv = torch.zeros(NB, KV, 128, 16)
    ref.rope_cache(rq, rk, rv, qkv, pos.cpu(), slots.cpu(), cos_sin.cpu(), H, KV)
    torch.testing.assert_close(q.float().cpu(), rq, atol=4e-2, rtol=2e-2)
    torch.testing.assert_close(kc.float().cpu(), rk, atol=4e-2, rtol=2e-2)
    torch.testing.assert_close(vc.float().cpu(), rv, atol=4e-2, rtol=2e-2)


def test_stream_gemm_poisoned_handoff(gpu):
    """The cooperative split-K reduction under stress: fresh inputs each repetition, slabs
    NaN-poisoned before every launch, a side-stream GEMM beside every other launch; the
    result must equal the same plan's first (clean) result bit for bit."""
    torch.manual_seed(34)
    ws, _, err = ops.stream_workspace(gpu)
    side = torch.cuda.Stream()
    big = torch.randn(4096, 4096, device=gpu, dtype=torch.bfloat16)
    w = _bf(4096, 14336, dev=gpu, scale=0.02)
    wp = ops.pack_decode_weight(w)
    for rep in range(200):
        x = _bf(64, 14336, dev=gpu)
        base = ops.stream_gemm(x, wp, "plain", plan=(4, 1, 2, 4, 1, 8, 4)).clone()
        ws.fill_(float("nan"))
        if rep % 2:
            with torch.cuda.stream(side):
                torch.matmul(big, big)
        got = ops.stream_gemm(x, wp, "plain", plan=(4, 1, 2, 4, 1, 8, 4))
        torch.cuda.synchronize()
        assert torch.equal(got, base), rep
    assert int(err[0]) == 0


def test_stream_gemm_group_barrier_timeout_sets_err(gpu):
    """a split-K group whose partner never arrives (injected: the group's arrive
    counter starts far below zero, so no workgroup ever sees all S arrivals) must give up after
    its bounded spin and set the err word the engine reads back, not hang and not stay silent;
    the departure path then leaves the counters zeroed for the next launch."""
    torch.manual_seed(35)
    _, cnt, err = ops.stream_workspace(gpu)
    x = _bf(64, 4096, dev=gpu)
    w = _bf(4096, 4096, dev=gpu, scale=0.05)
    wp = ops.pack_decode_weight(w)
    plan = (4, 1, 1, 4, 1, 4, 4)  # 64 groups x 4 K-slices
    err.zero_()
    cnt[0] = -(1 << 20)  # group 0: its arrivals can never reach S
    ops.stream_gemm(x, wp, "plain", plan=plan)
    torch.cuda.synchronize()
    assert int(err[0]) == 1
    assert int(cnt[0]) == 0 and int(cnt[1]) == 0  # reset by the last departure
    err.zero_()
    y = ops.stream_gemm(x, wp, "plain", plan=plan)  # healthy again
    torch.testing.assert_close(y.float(), x.float() @ w.float().T, atol=4e-2, rtol=2e-2)
    assert int(err[0]) == 0


def _engine_stream_plans():
    """Every (kind, M, plan) the engine routes to the stream kernel with a K split (a hand-off):
    LlamaModel.STREAM_CFG at the first and last row count of each table row. LM_HEAD_STREAM
    plans have S = wk = 1 (direct epilogue, no slab) and are not listed."""
    from pilottai_amd.models.llama import LlamaModel

    out = []
    for kind, rows in LlamaModel.STREAM_CFG.items():
        lo = LlamaModel.DECODE_FUSED_MAX_T + 1
        for mmax, shape in rows:
            for M in sorted({lo, mmax}):
                plan = LlamaModel._stream_plan(M, shape)
                if plan[5] * plan[4] > 1:
                    out.append((kind, M, plan))
            lo = mmax + 1
    return out


_SHAPES = {"qkv": (6144, 4096, "rope_perm"), "o": (4096, 4096, "resid"), "down": (4096, 14336, "resid")}


@pytest.mark.parametrize("kind,M,plan", _engine_stream_plans())
def test_stream_handoff_shipping_default_no_release(gpu, kind, M, plan):
    """the SHIPPING hand-off (rel = 0: no producer release; the consumer
    polls, acquires, and reads with sc1 loads) on every plan the engine routes here, 2,000
    poisoned repetitions each: fresh inputs, the slabs NaN-poisoned before every launch, a
    side-stream GEMM beside every other launch; every result must equal the plan's clean
    result bit for bit (the group reduction sums the slabs in a fixed order), and the group
    barrier's err word must stay 0. tools/stream_handoff_stress.py runs the same at 100,000."""
    N, K, epi = _SHAPES[kind]
    torch.manual_seed(40 + M)
    ws, _, err = ops.stream_workspace(gpu)
    err.zero_()
    side = torch.cuda.Stream()
    big = torch.randn(4096, 4096, device=gpu, dtype=torch.bfloat16)
    w = _bf(N, K, dev=gpu, scale=0.02)
    wp = ops.pack_decode_qkv_rope(w) if epi == "rope_perm" else ops.pack_decode_weight(w)
    x = torch.empty(M, K, device=gpu, dtype=torch.bfloat16)
    r = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    base = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    got = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    bad = torch.zeros((), dtype=torch.int64, device=gpu)
    res = r if epi == "resid" else None
    for rep in range(2000):
        x.normal_()
        r.normal_()
        ops.stream_gemm(x, wp, epi, resid=res, out=base, plan=plan, rel=0)
        ws.fill_(float("nan"))
        got.fill_(float("nan"))
        if rep % 2:
            with torch.cuda.stream(side):
                torch.matmul(big, big)
        ops.stream_gemm(x, wp, epi, resid=res, out=got, plan=plan, rel=0)
        bad += (~((got == base) | (torch.isnan(got) & torch.isnan(base)))).any().to(torch.int64)
    torch.cuda.synchronize()
    assert int(bad) == 0 and int(err[0]) == 0

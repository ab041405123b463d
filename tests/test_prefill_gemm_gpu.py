"""Large-M packed-weight projections (csrc/ops/gemm_prefill.hip: 256 x 256, 256 x 192 and
256 x 128 MFMA tiles, LDS-DMA stages, fused epilogues) vs fp32 PyTorch references."""
import pytest
import torch

from pilottai_amd import ops
from pilottai_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _bf(*shape, dev, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


@pytest.mark.parametrize("M,N,K,epi,norm,full,splits", [
    # Llama-3-8B projections at prefill-step sizes (default plans: whole tiles + split tail)
    (2048, 28672, 4096, "silu", True, -1, 0), (2048, 6144, 4096, "rope_perm", True, -1, 0),
    (2048, 4096, 4096, "resid", False, -1, 0), (1024, 4096, 14336, "resid", False, -1, 0),
    # partial row tiles, explicit whole / split decompositions
    (300, 4096, 4096, "plain", False, -1, 1), (777, 6144, 4096, "plain", True, 0, 3),
    (513, 28672, 4096, "silu", True, 200, 2), (1536, 4096, 14336, "resid", False, 0, 4),
    (272, 2048, 1024, "plain", False, 3, 2), (64, 1024, 512, "silu", False, -1, 0),
    (1000, 1280, 8192, "rope_perm", True, 0, 2),  # 70B TP=8 QKV shard
    (17, 768, 128, "plain", True, -1, 1), (256, 512, 64, "resid", False, 0, 1),
    # more than one round of 256-wide tiles with a short tail (the default variant runs the
    # tail columns on 256 x 128 tiles in the same launch)
    (1024, 20480, 512, "rope_perm", True, -1, 0), (768, 24576, 256, "resid", False, -1, 0),
    (1000, 28672, 256, "plain", False, -1, 0)])
@pytest.mark.parametrize("bn,variant", [(256, 3), (256, 9), (256, 1), (128, 3), (128, 1)])
def test_prefill_gemm(gpu, M, N, K, epi, norm, full, splits, bn, variant):
    """Every epilogue and the folded row norm; run twice so the self-resetting tickets of
    the split tail are exercised. Ping-pong kernels (variant 3, the default: two-phase
    256-wide / three-buffer 128-wide schedules; 9: without the mixed 128-wide tail) and the
    read-ahead / 3-stage kernels (variant 1, the fallback for < 2 k-tiles)."""
    from pilottai_amd.ops import kernels

    kernels.require_native().prefill_set_variant(variant)
    try:
        _check_prefill_gemm(gpu, M, N, K, epi, norm, full, splits, bn)
    finally:
        kernels.require_native().prefill_set_variant(-1)


def _check_prefill_gemm(gpu, M, N, K, epi, norm, full, splits, bn):
    torch.manual_seed(21)
    x = _bf(M, K, dev=gpu)
    w = _bf(N, K, dev=gpu, scale=0.05)
    resid = _bf(M, N, dev=gpu) if epi == "resid" else None
    pack = {"silu": ops.pack_decode_gate_up, "rope_perm": ops.pack_decode_qkv_rope}.get(epi, ops.pack_decode_weight)
    wp = pack(w)
    acc = x.float() @ w.float().T
    if norm:
        acc = acc * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-5)
    if epi == "silu":
        acc = torch.nn.functional.silu(acc[:, :N // 2]) * acc[:, N // 2:]
    elif epi == "resid":
        acc = acc + resid.float()
    for _ in range(2):
        y = ops.prefill_gemm(x, wp, epi, resid=resid, norm=norm, full=full, splits=splits, bn=bn)
        torch.testing.assert_close(y.float(), acc, atol=4e-2, rtol=2e-2)


@pytest.mark.parametrize("M,N,K,epi,norm,full,splits", [
    # qkv of Llama-3-8B at 1,280 < M <= 2,048 (one round of 256 x 192 tiles)
    (2048, 6144, 4096, "rope_perm", True, -1, 0), (1536, 6144, 4096, "plain", False, -1, 1),
    (1300, 6144, 4096, "plain", True, -1, 0),
    # K-sliced items, every epilogue, partial row tiles, two k-tiles per item
    (777, 6144, 4096, "plain", True, 0, 3), (513, 6144, 4096, "silu", True, 10, 2),
    (1000, 6144, 14336, "resid", False, 0, 4), (300, 1536, 128, "resid", False, -1, 1),
    (2100, 11520, 512, "rope_perm", True, -1, 0), (64, 384, 256, "plain", False, 0, 2)])
def test_prefill_gemm_192(gpu, M, N, K, epi, norm, full, splits):
    """256 x 192 tiles (gemm_pingpong.h F = 6, `body6` schedule) vs fp32: whole tiles and
    K-slices, every register epilogue."""
    _check_prefill_gemm(gpu, M, N, K, epi, norm, full, splits, 192)


def test_prefill_gemm_192_refuses_other_widths(gpu):
    """bn = 192 needs N % 192 == 0 and the ping-pong schedule: anything else is refused at
    the launcher instead of running a partial tile."""
    x = _bf(512, 512, dev=gpu)
    wp = ops.pack_decode_weight(_bf(1024, 512, dev=gpu))
    with pytest.raises(ValueError, match="does not handle"):
        ops.prefill_gemm(x, wp, "plain", bn=192)


@pytest.mark.parametrize("bn,variant", [(256, -1), (192, -1), (128, -1), (256, 1)])
def test_prefill_gemm_asymmetric_identity(gpu, bn, variant):
    """x = I (rows), W asymmetric: the output must be exactly W^T's rows (catches a
    transposed or permuted C write, guide §3 'A = I-check with asymmetric B')."""
    M, N, K = 512, 1152 if bn == 192 else 1024, 512
    x = torch.zeros(M, K, device=gpu)
    x[torch.arange(M), torch.arange(M) % K] = 1.0
    w = (torch.arange(N * K, device=gpu, dtype=torch.float32).view(N, K) % 251 / 64.0).to(torch.bfloat16)
    y = ops.prefill_gemm(x.to(torch.bfloat16), ops.pack_decode_weight(w), "plain", full=-1, splits=1, bn=bn,
                         variant=variant)
    want = w.float().T[torch.arange(M) % K]
    assert torch.equal(y.float(), want.to(torch.bfloat16).float())


@pytest.mark.parametrize("M,S", [(700, 1), (700, 3), (2048, 2)])
@pytest.mark.parametrize("bn", [256, 128])
def test_prefill_gemm_resid_in_place_with_row_stats(gpu, M, S, bn):
    """h += x W^T in place, accumulating the next norm's row statistics (ss_out) of the
    written bf16 rows and zeroing another buffer (ss_zero); the following norm-folded
    projection consuming them matches rmsnorm + GEMM."""
    torch.manual_seed(22)
    N, K = 4096, 4096
    x = _bf(M, K, dev=gpu)
    w = _bf(N, K, dev=gpu, scale=0.05)
    h = _bf(M, N, dev=gpu)
    want = h.float() + x.float() @ w.float().T
    hh = h.clone()
    ss = torch.zeros(M, dtype=torch.float32, device=gpu)
    junk = torch.full((M,), 7.0, device=gpu)
    ops.prefill_gemm(x, ops.pack_decode_weight(w), "resid", resid=hh, out=hh, full=0 if S > 1 else -1,
                     splits=S, ss_out=ss, ss_zero=junk, bn=bn)
    torch.testing.assert_close(hh.float(), want, atol=4e-2, rtol=2e-2)
    torch.testing.assert_close(ss, hh.float().pow(2).sum(-1), rtol=1e-4, atol=1e-2)
    assert float(junk.abs().max()) == 0.0
    w2 = _bf(2048, N, dev=gpu, scale=0.05)
    g = (torch.rand(N, device=gpu) + 0.5).to(torch.bfloat16)
    wg = w2 * g[None, :]
    y = ops.prefill_gemm(hh, ops.pack_decode_weight(wg), norm=True, ss_in=ss, bn=bn)
    xn = hh.float() * torch.rsqrt(hh.float().pow(2).mean(-1, keepdim=True) + 1e-5)
    torch.testing.assert_close(y.float(), xn @ wg.float().T, atol=4e-2, rtol=2e-2)


@pytest.mark.parametrize("M,H,KV,K,full,splits", [
    (1024, 32, 8, 4096, -1, 0), (333, 32, 8, 4096, 0, 4), (600, 8, 2, 1024, -1, 1), (2048, 32, 8, 4096, 0, 2),
    (1792, 32, 8, 4096, -1, 0)])
@pytest.mark.parametrize("bn", [256, 192, 128])
def test_prefill_qkv_rope(gpu, M, H, KV, K, full, splits, bn):
    """Norm-folded QKV with RoPE + paged KV write vs fp32 projection + reference rope_cache."""
    torch.manual_seed(23)
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
        ops.prefill_qkv_rope(x, wp, 1e-5, q, kc, vc, pos, slots, cos_sin, H, KV, full=full, splits=splits, bn=bn)
    xn = x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-5) * g.float()
    qkv = (xn @ w.float().T).cpu()
    rq = torch.empty(M, H, 128, dtype=torch.float32)
    rk = torch.zeros(NB, KV, 16, 16, 8)
    rv = torch.zeros(NB, KV, 128, 16)
    ref.rope_cache(rq, rk, rv, qkv, pos.cpu(), slots.cpu(), cos_sin.cpu(), H, KV)
    torch.testing.assert_close(q.float().cpu(), rq, atol=4e-2, rtol=2e-2)
    torch.testing.assert_close(kc.float().cpu(), rk, atol=4e-2, rtol=2e-2)
    torch.testing.assert_close(vc.float().cpu(), rv, atol=4e-2, rtol=2e-2)


@pytest.mark.parametrize("epi", ["plain", "resid"])
def test_prefill_gemm_strided_views(gpu, epi):
    """The plain / residual epilogues store (and read the residual) 16 B per lane: a padded
    output view with 16-byte rows is written correctly, a view whose rows are only 8-byte
    aligned is refused at the binding instead of issuing misaligned wide accesses."""
    torch.manual_seed(5)
    M, N, K = 300, 1024, 512
    x = _bf(M, K, dev=gpu)
    w = _bf(N, K, dev=gpu, scale=0.05)
    wp = ops.pack_decode_weight(w)
    want = x.float() @ w.float().T
    big = torch.zeros(M, N + 8, dtype=torch.bfloat16, device=gpu)  # padded rows, 16-B aligned
    resid = None
    if epi == "resid":
        rbig = _bf(M, N + 16, dev=gpu)
        resid = rbig[:, 8:8 + N]
        want = want + resid.float()
    y = ops.prefill_gemm(x, wp, epi, resid=resid, out=big[:, :N])
    torch.testing.assert_close(y.float(), want, atol=4e-2, rtol=2e-2)
    assert torch.equal(big[:, N:], torch.zeros_like(big[:, N:]))  # the padding is untouched
    odd = torch.zeros(M, N + 4, dtype=torch.bfloat16, device=gpu)[:, 4:]  # 8-byte aligned only
    with pytest.raises(RuntimeError, match="16-byte"):
        ops.prefill_gemm(x, wp, epi, resid=resid, out=odd)

"""Plain-PyTorch fp32 reference implementations of every HIP kernel.

They define the semantics the CDNA4 kernels are tested against (GPU numerics
tests compare kernel output with these on the same inputs) and serve as the CPU
execution path for the control-plane tests that run without a GPU. On a GPU box
the native kernels are mandatory (see ops/kernels.py) — these are never a
silent fallback for device tensors.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch

# ---------------------------------------------------------------------------
# normalisation / activation
# ---------------------------------------------------------------------------


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    inv = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return ((xf * inv).to(x.dtype).float() * w.float()).to(x.dtype)


def fused_add_rmsnorm(resid: torch.Tensor, x: torch.Tensor, w: torch.Tensor, eps: float):
    """Returns (normed, new_resid); new_resid = bf16(resid + x)."""
    new_resid = (resid.float() + x.float()).to(resid.dtype)
    return rmsnorm(new_resid, w, eps), new_resid


def silu_mul(x: torch.Tensor) -> torch.Tensor:
    F = x.shape[-1] // 2
    g, u = x[..., :F].float(), x[..., F:].float()
    return (torch.nn.functional.silu(g).to(x.dtype).float() * u).to(x.dtype)


# ---------------------------------------------------------------------------
# RoPE + paged KV cache
# ---------------------------------------------------------------------------


def rope_cos_sin(max_pos: int, head_dim: int = 128, theta: float = 500000.0,
                 scaling: Optional[dict] = None) -> torch.Tensor:
    """fp32 [max_pos, head_dim] table: cos in [:, :hd/2], sin in [:, hd/2:].

    `scaling` follows the Llama-3.1 "llama3" rope_scaling dict (factor,
    low_freq_factor, high_freq_factor, original_max_position_embeddings).
    """
    half = head_dim // 2
    inv = 1.0 / (theta ** (torch.arange(0, half, dtype=torch.float64) / half))
    if scaling:
        factor = scaling.get("factor", 8.0)
        lo = scaling.get("low_freq_factor", 1.0)
        hi = scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        lo_wl, hi_wl = old / lo, old / hi
        wl = 2 * math.pi / inv
        smooth = (old / wl - lo) / (hi - lo)
        scaled = torch.where(wl > lo_wl, inv / factor, inv)
        mid = (wl <= lo_wl) & (wl >= hi_wl)
        scaled = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
        inv = scaled
    pos = torch.arange(max_pos, dtype=torch.float64)
    ang = torch.outer(pos, inv)
    return torch.cat([ang.cos(), ang.sin()], dim=1).float()


def apply_rope(x: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor) -> torch.Tensor:
    """x [T, heads, 128] -> rotated (bf16 rounding as in the kernel)."""
    half = x.shape[-1] // 2
    cs = cos_sin[positions.long()]
    c, s = cs[:, None, :half], cs[:, None, half:]
    x1, x2 = x[..., :half].float(), x[..., half:].float()
    o1 = x1 * c - x2 * s
    o2 = x2 * c + x1 * s
    return torch.cat([o1, o2], dim=-1).to(x.dtype)


def rope_cache(q_out, k_cache, v_cache, qkv, positions, slot_mapping, cos_sin, H, KV,
               apply: bool = True):
    T = qkv.shape[0]
    hd = 128
    q = qkv[:, : H * hd].reshape(T, H, hd)
    k = qkv[:, H * hd:(H + KV) * hd].reshape(T, KV, hd)
    v = qkv[:, (H + KV) * hd:(H + 2 * KV) * hd].reshape(T, KV, hd)
    if apply:
        q = apply_rope(q, positions[:T], cos_sin)
        k = apply_rope(k, positions[:T], cos_sin)
    q_out[:T].copy_(q.reshape(q_out[:T].shape))
    blk = k_cache.shape[3]  # K page: [KV, 128/8, block, 8] (fragment-major)
    for t in range(T):
        slot = int(slot_mapping[t])
        if slot < 0:
            continue
        b, o = divmod(slot, blk)
        k_cache[b, :, :, o, :] = k[t].reshape(KV, hd // 8, 8)
        v_cache[b, :, :, o] = v[t]


def paged_attention(q, k_cache, v_cache, q_start, q_len, ctx_len, block_table, scale):
    """q [T, H, 128]; returns out [T, H, 128] (fp32 math, causal within context)."""
    T, H, hd = q.shape
    KV = k_cache.shape[1]
    G = H // KV
    blk = k_cache.shape[3]
    out = torch.zeros_like(q)
    for s in range(len(q_len)):
        ql, ctx, q0 = int(q_len[s]), int(ctx_len[s]), int(q_start[s])
        if ql <= 0:
            continue
        nb = (ctx + blk - 1) // blk
        blocks = block_table[s, :nb].long()
        K = k_cache[blocks].permute(1, 0, 3, 2, 4).reshape(KV, nb * blk, hd)[:, :ctx].float()
        V = v_cache[blocks].permute(1, 0, 3, 2).reshape(KV, nb * blk, hd)[:, :ctx].float()
        Kh = K.repeat_interleave(G, dim=0)  # [H, ctx, hd]
        Vh = V.repeat_interleave(G, dim=0)
        qs = q[q0:q0 + ql].float().permute(1, 0, 2)  # [H, ql, hd]
        sc = torch.matmul(qs, Kh.transpose(1, 2)) * scale  # [H, ql, ctx]
        pos = torch.arange(ctx - ql, ctx)[:, None]
        keys = torch.arange(ctx)[None, :]
        sc = sc.masked_fill(keys > pos, float("-inf"))
        p = torch.softmax(sc, dim=-1)
        o = torch.matmul(p, Vh)  # [H, ql, hd]
        out[q0:q0 + ql] = o.permute(1, 0, 2).to(q.dtype)
    return out


# ---------------------------------------------------------------------------
# sampling — same counter-based hash as csrc/ops/common.h (uniform01)
# ---------------------------------------------------------------------------

_M32 = np.uint64(0xFFFFFFFF)


def _mix32(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64) & _M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & _M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & _M32
    x ^= x >> np.uint64(16)
    return x


def uniform01(seed: int, row_off: int, cols: np.ndarray) -> np.ndarray:
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    lo, hi = seed & 0xFFFFFFFF, seed >> 32
    a = _mix32(np.array([(row_off * 0x9E3779B9 + hi) & 0xFFFFFFFF], dtype=np.uint64))
    h = _mix32(np.uint64(lo) ^ a)
    c = (cols.astype(np.uint64) * np.uint64(0x85EBCA6B) + np.uint64(0x27D4EB2F)) & _M32
    h = _mix32(h ^ c)
    return ((h >> np.uint64(8)).astype(np.float64) + 0.5) * (1.0 / 16777216.0)


def topkp_threshold(logits: torch.Tensor, temperature, top_k, top_p, mask_class, class_masks):
    """Exact top-k / top-p logit threshold per row (fp64 math, sort based).

    Kept set = allowed tokens with logit >= tau; tau is the larger of the k-th
    largest allowed logit and the value at which the descending cumulative
    softmax(logit / T) mass first reaches p. -inf = no truncation."""
    rows, V = logits.shape
    out = torch.full((rows,), float("-inf"), dtype=torch.float32)
    lg = logits.float().cpu().numpy().astype(np.float64)
    cm = class_masks.cpu().numpy().view(np.uint32) if class_masks is not None else None
    for r in range(rows):
        T, k, p = float(temperature[r]), int(top_k[r]), float(top_p[r])
        if T <= 0 or ((k <= 0 or k >= V) and not p < 1.0):
            continue
        vals = lg[r]
        mc = int(mask_class[r])
        if mc >= 0 and cm is not None:
            idx = np.arange(V)
            ok = ((cm[mc][idx >> 5] >> (idx & 31).astype(np.uint32)) & 1).astype(bool)
            vals = vals[ok]
        if vals.size == 0:
            continue
        s = np.sort(vals)[::-1]
        t = -np.inf
        if 0 < k < s.size:
            t = max(t, s[k - 1])
        if p < 1.0:
            w = np.exp((s - s[0]) / T)
            c = np.cumsum(w)
            j = int(np.searchsorted(c, p * c[-1] * (1 - 1e-6)))
            t = max(t, s[min(j, s.size - 1)])
        out[r] = t
    return out


def sample(logits: torch.Tensor, temperature, mask_class, class_masks, seeds, offsets,
           forced=None, vocab_offset: int = 0, return_keys: bool = False, tau=None):
    """Gumbel-max sampling with grammar masks (and optional top-k/p threshold
    tau: logits below it are excluded); returns int32 tokens [rows]."""
    rows, V = logits.shape
    toks = torch.zeros(rows, dtype=torch.int32)
    keys_out = torch.zeros(rows, dtype=torch.float32)
    lg = logits.float().cpu().numpy().astype(np.float64)
    cm = class_masks.cpu().numpy().view(np.uint32) if class_masks is not None else None
    for r in range(rows):
        f = int(forced[r]) if forced is not None else -1
        T = float(temperature[r])
        mc = int(mask_class[r])
        idx = np.arange(V) + vocab_offset
        valid = np.ones(V, dtype=bool)
        if mc >= 0 and cm is not None:
            words = cm[mc][idx >> 5]
            valid = ((words >> (idx & 31).astype(np.uint32)) & 1).astype(bool)
        if T <= 0:
            key = lg[r].copy()
        else:
            key = lg[r] / T
            u = uniform01(int(seeds[r]), int(offsets[r]), idx)
            key = key + (-np.log(-np.log(u)))
        if tau is not None:
            valid &= lg[r] >= float(tau[r])
        key[~valid] = -np.inf
        best = int(np.argmax(key)) if valid.any() else 0
        keys_out[r] = float(key[best]) if valid.any() else float("-inf")
        toks[r] = f if f >= 0 else best + vocab_offset
    return (toks, keys_out) if return_keys else toks


# ---------------------------------------------------------------------------
# semantic index
# ---------------------------------------------------------------------------


def cosine_topk(queries, index, n_valid, K, row_priority, row_tags, row_expiry, q_min_priority,
                q_tags, now):
    """Returns (scores [Q,K] fp32, rows [Q,K] int32), rows -1 past the matches."""
    Q = queries.shape[0]
    sc = queries.float() @ index[:n_valid].float().T  # [Q, N]
    out_s = torch.full((Q, K), float("-inf"))
    out_r = torch.full((Q, K), -1, dtype=torch.int32)
    prio = row_priority[:n_valid].long()
    tags = row_tags[:n_valid].long()
    exp = row_expiry[:n_valid].float()
    alive = (exp == 0) | (exp > now)
    for q in range(Q):
        qt = int(q_tags[q])
        ok = (prio >= int(q_min_priority[q])) & ((tags & qt) == qt) & alive
        s = sc[q].masked_fill(~ok, float("-inf"))
        k = min(K, int(ok.sum()))
        if k == 0:
            continue
        v, i = torch.topk(s, k)
        out_s[q, :k] = v
        out_r[q, :k] = i.int()
    return out_s, out_r


def q16_topk(qv, qmeta, hi, lo, rmeta, n_valid, K, row_priority, row_tags, row_expiry, q_min_priority, q_tags,
             now):
    """Exact top-k over the 16-bit fixed-point index (csrc/ops/similarity_q16.hip semantics):
    score = float32(float64(v_q . v_r) * (float64(s_r) * float64(s_q))) with v = 256 hi + lo,
    the integer dot products exact in int64. qv [Q, 2, D] int8 (qh, ql), qmeta [Q, 2] (s_q, .),
    hi / lo fragment-major int8 tiles, rmeta [N, 2] (s_r, .)."""
    T, DS = hi.shape[0], hi.shape[1]
    unpack = lambda t: t.view(T, DS, 4, 16, 16).permute(0, 3, 1, 2, 4).reshape(T * 16, DS * 64)  # noqa: E731
    n = int(n_valid)
    vr = 256 * unpack(hi)[:n].long().cpu() + unpack(lo)[:n].long().cpu()
    vq = 256 * qv[:, 0].long().cpu() + qv[:, 1].long().cpu()
    dots = vq @ vr.T  # exact int64
    sc = (dots.double() * (rmeta[:n, 0].double().cpu()[None, :] * qmeta[:, 0].double().cpu()[:, None])).float()
    return cosine_topk_from_scores(sc, n, K, row_priority, row_tags, row_expiry, q_min_priority, q_tags, now)


def cosine_topk_from_scores(sc, n_valid, K, row_priority, row_tags, row_expiry, q_min_priority, q_tags, now):
    """The filtered top-k of precomputed scores [Q, n_valid] (the reference kernels' common tail)."""
    Q = sc.shape[0]
    out_s = torch.full((Q, K), float("-inf"))
    out_r = torch.full((Q, K), -1, dtype=torch.int32)
    prio = row_priority[:n_valid].long().cpu()
    tags = row_tags[:n_valid].long().cpu()
    exp = row_expiry[:n_valid].float().cpu()
    alive = (exp == 0) | (exp > now)
    for q in range(Q):
        qt = int(q_tags[q])
        ok = (prio >= int(q_min_priority[q])) & ((tags & qt) == qt) & alive
        s = sc[q].masked_fill(~ok, float("-inf"))
        k = min(K, int(ok.sum()))
        if k == 0:
            continue
        v, i = torch.topk(s, k)
        out_s[q, :k] = v
        out_r[q, :k] = i.int()
    return out_s, out_r


def pack_mask(allowed) -> torch.Tensor:
    """bool [V] -> int32 words, bit i of word i // 32 set iff token i is allowed."""
    a = np.asarray(allowed, dtype=bool)
    pad = (-len(a)) % 32
    if pad:
        a = np.concatenate([a, np.zeros(pad, dtype=bool)])
    return torch.from_numpy(np.packbits(a, bitorder="little").view(np.int32).copy())

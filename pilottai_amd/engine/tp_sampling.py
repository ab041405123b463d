"""Exact top-k / top-p thresholds over a vocab-parallel LM head without gathering the logits
(VERDICT r3 missing #3: the TP>1 sampler all-gathered the full logits).

The single-GPU threshold (csrc/ops/sampling.hip topkp_threshold_kernel) is a two-level radix
select on the 16-bit bf16 order key: 256-bin histograms of (count, softmax mass at the row's
temperature) of the allowed tokens, scanned top-down to the bin where the top-k count or the
top-p mass is reached, then the same inside that bin for the low byte. Histograms ADD across
vocabulary shards, so under tensor parallelism every rank builds the histograms of its own
V/tp slice, the group all-reduces them (rows x 512 floats per level, plus one rows-long max),
and every rank runs the identical scan: the same kept set as the single-GPU kernel on the
gathered logits, for ~4 KB per row of traffic instead of the 2 x V bytes per row an all-gather
of the logits moves (Llama-3: 256 KB per row at TP = 8).

On the GPU the passes are HIP kernels and the collectives run on the custom P2P buffers
(capturable, no RCCL in a step graph); on the CPU the same algorithm runs as torch ops.
"""
from __future__ import annotations

import torch

LOG2E = 1.4426950408889634


def _order_key(logits_bf16: torch.Tensor) -> torch.Tensor:
    """Monotone 16-bit key of bf16 values (as int32): larger key <=> larger value."""
    b = logits_bf16.contiguous().view(torch.int16).to(torch.int32) & 0xFFFF
    return torch.where((b & 0x8000) != 0, (~b) & 0xFFFF, b | 0x8000)


def _key_value(key: torch.Tensor) -> torch.Tensor:
    """Inverse of _order_key: the bf16 value (as fp32) of a 16-bit key."""
    b = torch.where((key & 0x8000) != 0, key & 0x7FFF, (~key) & 0xFFFF)
    return (b.to(torch.int32) << 16).view(torch.float32)


def _allowed(mask_class, class_masks, rows: int, vocab_offset: int, v_local: int, device) -> torch.Tensor:
    """[rows, v_local] bool: the grammar mask of each row's class over this shard's slice
    (class < 0: every token allowed)."""
    g = torch.arange(vocab_offset, vocab_offset + v_local, device=device)
    mc = mask_class[:rows].long()
    words = class_masks[mc.clamp(min=0)][:, (g >> 5)]          # [rows, v_local] int32
    bits = ((words >> (g & 31).to(torch.int32)) & 1) != 0
    return bits | (mc < 0).unsqueeze(1)


def _scan(cnt: torch.Tensor, mass: torch.Tensor, need_cnt: torch.Tensor, need_mass: torch.Tensor,
          above_cnt: torch.Tensor, above_mass: torch.Tensor):
    """Top-down scan of 256 bins (the kernel's loop, vectorised): the highest bin b where the
    count or the mass from the top reaches its need (bin 0 if none); returns (b, count and mass
    strictly above b)."""
    c_from = torch.flip(torch.cumsum(torch.flip(cnt, [1]), 1), [1]) + above_cnt.unsqueeze(1)  # >= b
    m_from = torch.flip(torch.cumsum(torch.flip(mass, [1]), 1), [1]) + above_mass.unsqueeze(1)
    hit = (c_from >= need_cnt.unsqueeze(1)) | (m_from >= need_mass.unsqueeze(1))
    idx = torch.arange(256, device=cnt.device).expand_as(hit)
    sel = torch.where(hit, idx, torch.full_like(idx, -1)).max(1).values.clamp(min=0)
    c_above = c_from.gather(1, sel.unsqueeze(1)).squeeze(1) - cnt.gather(1, sel.unsqueeze(1)).squeeze(1)
    m_above = m_from.gather(1, sel.unsqueeze(1)).squeeze(1) - mass.gather(1, sel.unsqueeze(1)).squeeze(1)
    return sel, c_above, m_above


def tkp_ws_floats(rows: int) -> int:
    """Workspace of the HIP phase kernels: mx (padded to 4 rows) | h0 | h1 | scan state."""
    return ((rows + 3) & ~3) + rows * 1028


def tp_topkp_threshold(logits: torch.Tensor, vocab_offset: int, V: int, temperature, top_k, top_p,
                       mask_class, class_masks, tp, out: torch.Tensor = None,
                       ws: torch.Tensor = None) -> torch.Tensor:
    """tau[row] for this rank's logit slice [rows, V / tp] (bf16): the threshold the single-GPU
    kernel computes on the whole vocabulary. Collective over the TP group `tp`
    (TPGroup: all_reduce_max / all_reduce_sum over fp32; on GPUs the custom P2P buffers, so a
    captured step graph holds no RCCL call). On the GPU: four launches of the HIP phase kernel
    (csrc/ops/sampling.hip tp_topkp_kernel: row max, high-byte histogram, scan + low-byte
    histogram, scan) with a MAX and two SUM all-reduces between them; `ws` (>= tkp_ws_floats(rows)
    fp32, allocate outside capture) is their workspace. CPU: the same algorithm as torch ops."""
    rows, vl = logits.shape
    if logits.is_cuda:
        from pilottai_amd.ops.kernels import require_native

        C = require_native()
        tau = out if out is not None else torch.empty(rows, dtype=torch.float32, device=logits.device)
        if ws is None:
            ws = torch.empty(tkp_ws_floats(rows), dtype=torch.float32, device=logits.device)
        args = (logits, int(vocab_offset), int(V), temperature, top_k, top_p, mask_class, class_masks)
        r4 = (rows + 3) & ~3
        mx = ws[:r4]
        h0 = ws[r4:r4 + rows * 512]
        h1 = ws[r4 + rows * 512:r4 + rows * 1024]
        C.tp_topkp_phase(0, tau, ws, *args)
        tp.all_reduce_max(mx)
        C.tp_topkp_phase(1, tau, ws, *args)
        tp.all_reduce_sum(h0)
        C.tp_topkp_phase(2, tau, ws, *args)
        tp.all_reduce_sum(h1)
        C.tp_topkp_phase(3, tau, ws, *args)
        return tau
    dev = logits.device
    T = temperature[:rows].float()
    k = top_k[:rows]
    p = top_p[:rows].float()
    active = (T > 0) & ~(((k <= 0) | (k >= V)) & ~(p < 1.0))
    ok = _allowed(mask_class, class_masks, rows, vocab_offset, vl, dev)
    key = _order_key(logits)
    val = _key_value(key)
    neg_inf = torch.full_like(val, float("-inf"))
    mx = torch.where(ok, val, neg_inf).max(1).values
    tp.all_reduce_max(mx)
    invT = torch.where(T > 0, LOG2E / T.clamp(min=1e-30), torch.zeros_like(T))
    w = torch.where(ok, torch.exp2((val - mx.unsqueeze(1)) * invT.unsqueeze(1)), torch.zeros_like(val))
    w = torch.nan_to_num(w, nan=0.0)  # rows with no allowed token (mx = -inf)
    one = ok.float()
    need_cnt = torch.where((k > 0) & (k < V), k.float(), torch.full_like(T, float("inf")))

    def hist(bins, keep):
        h = torch.zeros(rows, 512, dtype=torch.float32, device=dev)
        h[:, :256].scatter_add_(1, bins, one * keep)
        h[:, 256:].scatter_add_(1, bins, w * keep)
        tp.all_reduce_sum(h)
        return h[:, :256], h[:, 256:]

    cnt0, mass0 = hist(key >> 8, torch.ones_like(one))
    total = mass0.sum(1)
    need_mass = torch.where(p < 1.0, p * total, torch.full_like(total, float("inf")))
    zero = torch.zeros_like(total)
    hi, c_above, m_above = _scan(cnt0, mass0, need_cnt, need_mass, zero, zero)
    cnt1, mass1 = hist(key & 0xFF, ((key >> 8) == hi.unsqueeze(1)).float())
    lo, _, _ = _scan(cnt1, mass1, need_cnt, need_mass, c_above, m_above)
    tau = _key_value((hi << 8) | lo)
    tau = torch.where(active & (mx > float("-inf")), tau, torch.full_like(tau, float("-inf")))
    if out is not None:
        out[:rows].copy_(tau)
        return out
    return tau

"""Host-side work decomposition for the paged attention kernel.

Mirrors the C++ scheduler's builder (csrc/runtime/scheduler.cpp, `build_attention_items`)
so tests and the eager/CPU path can produce the same item lists. See the
header of csrc/ops/attention.hip for the meaning of an item.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

ATT_PART = 512  # keys per decode partition (must match csrc/ops/attention.hip)


def build_attention_items(q_lens: Sequence[int], ctx_lens: Sequence[int], group: int,
                          split: bool = True, part: int = ATT_PART,
                          qcols: int = 128, wide_min_tokens: int = 2048, split_keys: int = 0,
                          max_items: int = 1 << 30) -> Tuple[List[Tuple[int, int, int, int]], int]:
    """Return (items, n_partial_slots).

    item = (seq, q_begin, nq | part << 8 | nparts << 20, partial_slot); the
    partitions of a split decode row are merged in-kernel by the last to finish.
    split_keys > 0: wide prefill items with at least that many causal keys are cut into
    min(4, keys // split_keys) partitions of whole 32-key tiles (8 partial slots each, after the
    decode partitions' slots), as the scheduler's prefill_split_keys.
    """
    tpw = 16 // group  # query tokens per wave (kv-split path)
    # tokens per prefill item: qcols MFMA columns (128: the LDS-staged 4-wave path of
    # csrc/ops/attention.hip; 32: one wave per item)
    # (wide items only when the step's prefill tokens reach wide_min_tokens, as the scheduler)
    pre = [ql for ql in q_lens if ql > tpw]
    if sum(pre) < wide_min_tokens or (wide_min_tokens > 0 and len(pre) < 2):
        qcols = 32
    qtile = max(1, max(32, qcols) // group)
    # prefill tiles first, most keys first across all chunks; then the decode items,
    # longest partition first (as the scheduler: the attention work queue takes them in order)
    pre: List[Tuple[int, Tuple[int, int, int, int]]] = []
    for s, (ql, ctx) in enumerate(zip(q_lens, ctx_lens)):
        if ql > tpw:
            for qb in range(((ql - 1) // qtile) * qtile, -1, -qtile):
                nq = min(qtile, ql - qb)
                pre.append((ctx - ql + qb + nq, (s, qb, nq | (1 << 20), 0)))
    dec: List[Tuple[int, Tuple[int, int, int, int]]] = []
    slot = 0
    for s, (ql, ctx) in enumerate(zip(q_lens, ctx_lens)):
        if ql <= 0:
            continue
        if ql <= tpw:
            nparts = (ctx + part - 1) // part if split else 1
            nparts = max(1, nparts)
            if nparts > 1:
                for p in range(nparts):
                    dec.append((min(part, ctx - p * part), (s, 0, ql | (p << 8) | (nparts << 20), slot + p)))
                slot += nparts
            else:
                dec.append((ctx, (s, 0, ql | (1 << 20), 0)))
    if split_keys > 0 and qtile * group > 32:
        out, total = [], len(pre) + len(dec)
        for keys, it in pre:
            nq, np_ = it[2] & 0xFF, min(4, keys // split_keys)
            if nq > 32 // group and np_ >= 2 and slot + 8 * np_ <= max_items and total + np_ - 1 <= max_items:
                per = -(-((keys + 31) // 32) // np_) * 32
                out += [(per, (it[0], it[1], nq | (p << 8) | (np_ << 20), slot + 8 * p)) for p in range(np_)]
                slot += 8 * np_
                total += np_ - 1
            else:
                out.append((keys, it))
        pre = out
    pre.sort(key=lambda kv: -kv[0])  # stable
    items: List[Tuple[int, int, int, int]] = [it for _, it in pre]
    dec.sort(key=lambda kv: -kv[0])
    items += [it for _, it in dec]
    return items, slot

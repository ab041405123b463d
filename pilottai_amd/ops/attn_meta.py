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
                          qcols: int = 128, wide_min_tokens: int = 2048) -> Tuple[List[Tuple[int, int, int, int]], int]:
    """Return (items, n_partial_slots).

    item = (seq, q_begin, nq | part << 8 | nparts << 20, partial_slot); the
    partitions of a split decode row are merged in-kernel by the last to finish.
    """
    tpw = 16 // group  # query tokens per wave (kv-split path)
    # tokens per prefill item: qcols MFMA columns (128: the LDS-staged 4-wave path of
    # csrc/ops/attention.hip; 32: one wave per item)
    # (wide items only when the step's prefill tokens reach wide_min_tokens, as the scheduler)
    pre = [ql for ql in q_lens if ql > tpw]
    if sum(pre) < wide_min_tokens or (wide_min_tokens > 0 and len(pre) < 2):
        qcols = 32
    qtile = max(1, max(32, qcols) // group)
    items: List[Tuple[int, int, int, int]] = []
    # prefill tiles first, heaviest tile of each chunk first (as the scheduler)
    for s, (ql, ctx) in enumerate(zip(q_lens, ctx_lens)):
        if ql > tpw:
            for qb in range(((ql - 1) // qtile) * qtile, -1, -qtile):
                items.append((s, qb, min(qtile, ql - qb) | (1 << 20), 0))
    slot = 0
    for s, (ql, ctx) in enumerate(zip(q_lens, ctx_lens)):
        if ql <= 0:
            continue
        if ql <= tpw:
            nparts = (ctx + part - 1) // part if split else 1
            nparts = max(1, nparts)
            if nparts > 1:
                for p in range(nparts):
                    items.append((s, 0, ql | (p << 8) | (nparts << 20), slot + p))
                slot += nparts
            else:
                items.append((s, 0, ql | (1 << 20), 0))
    return items, slot

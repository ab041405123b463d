"""Host-side work decomposition for the paged attention kernel.

Mirrors the C++ scheduler's builder (csrc/runtime/scheduler.cpp, `build_attention_items`)
so tests and the eager/CPU path can produce the same item lists. See the
header of csrc/ops/attention.hip for the meaning of an item.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

ATT_PART = 512  # keys per decode partition (must match csrc/ops/attention.hip)


def build_attention_items(q_lens: Sequence[int], ctx_lens: Sequence[int], group: int,
                          split: bool = True) -> Tuple[List[Tuple[int, int, int, int]],
                                                       List[Tuple[int, int, int, int]], int]:
    """Return (items, reduce_items, n_partial_slots).

    item        = (seq, q_begin, nq | part << 8 | nparts << 20, partial_slot)
    reduce_item = (seq, first_partial_slot, nparts, q_begin | nq << 16)
    """
    tpw = 16 // group  # query tokens per wave
    items: List[Tuple[int, int, int, int]] = []
    ritems: List[Tuple[int, int, int, int]] = []
    slot = 0
    for s, (ql, ctx) in enumerate(zip(q_lens, ctx_lens)):
        if ql <= 0:
            continue
        if ql <= tpw:
            nparts = (ctx + ATT_PART - 1) // ATT_PART if split else 1
            nparts = max(1, nparts)
            if nparts > 1:
                for p in range(nparts):
                    items.append((s, 0, ql | (p << 8) | (nparts << 20), slot + p))
                ritems.append((s, slot, nparts, 0 | (ql << 16)))
                slot += nparts
            else:
                items.append((s, 0, ql | (1 << 20), 0))
        else:
            tile = 4 * tpw
            for qb in range(0, ql, tile):
                nq = min(tile, ql - qb)
                items.append((s, qb, nq | (1 << 20), 0))
    return items, ritems, slot

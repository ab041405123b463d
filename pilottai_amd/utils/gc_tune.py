"""Garbage-collector settings for a serving process.

CPython's cyclic collector stops the interpreter while it scans; a full (generation 2) pass
over a serving process's heap -- model and tokenizer objects, compiled grammars, thousands of
task records -- took 60-85 ms here (tools probe in BENCHMARKS.md), and while it runs the engine
thread cannot launch the next step: one such pause is a 61 ms device gap in the round-4
64-worker profile. `freeze_heap()` moves everything alive after start-up into the permanent
generation (`gc.freeze`), so later collections scan only what the serving loop allocates.
"""
from __future__ import annotations

import gc
import os


def freeze_heap() -> int:
    """Collect once, then exclude every surviving object from future collections.
    Returns the number of frozen objects. PILOTTAI_GC_FREEZE=0 turns it off."""
    if os.environ.get("PILOTTAI_GC_FREEZE", "1") == "0":
        return 0
    gc.collect()
    gc.freeze()
    return gc.get_freeze_count()

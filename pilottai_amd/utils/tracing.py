"""Tracing: roctx ranges for rocprofv3 and an in-process span recorder.

* `trace_range(name)` — a roctx range (torch.cuda.nvtx maps to roctx on ROCm)
  around engine phases (schedule / H2D / replay / commit), visible with
  `rocprofv3 --marker-trace`; enabled with PILOTTAI_TRACE=1 (no cost otherwise).
* `Tracer` — host-side spans (name, thread, start, end) exported as Chrome trace
  JSON (chrome://tracing, Perfetto): `with tracer.span("agent.analyze"): ...`.
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
import time
from typing import Dict, List, Optional

ENABLED = os.environ.get("PILOTTAI_TRACE", "0") == "1"


@contextlib.contextmanager
def trace_range(name: str):
    if not ENABLED:
        yield
        return
    import torch

    pushed = False
    if torch.cuda.is_available():
        try:
            torch.cuda.nvtx.range_push(name)
            pushed = True
        except Exception:  # noqa: BLE001 — tracing must never break the step
            pushed = False
    t0 = time.perf_counter_ns()
    try:
        yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()
        GLOBAL_TRACER.add(name, t0, time.perf_counter_ns())


class Tracer:
    def __init__(self, max_spans: int = 1 << 20):
        self.max_spans = max_spans
        self._spans: List[tuple] = []
        self._lock = threading.Lock()

    def add(self, name: str, t0_ns: int, t1_ns: int, args: Optional[Dict] = None):
        with self._lock:
            if len(self._spans) < self.max_spans:
                self._spans.append((name, threading.get_ident(), t0_ns, t1_ns, args))

    @contextlib.contextmanager
    def span(self, name: str, **args):
        t0 = time.perf_counter_ns()
        try:
            yield
        finally:
            self.add(name, t0, time.perf_counter_ns(), args or None)

    def chrome_trace(self) -> Dict:
        with self._lock:
            spans = list(self._spans)
        ev = [{"name": n, "ph": "X", "pid": os.getpid(), "tid": tid, "ts": t0 / 1e3, "dur": (t1 - t0) / 1e3,
               **({"args": a} if a else {})} for n, tid, t0, t1, a in spans]
        return {"traceEvents": ev, "displayTimeUnit": "ms"}

    def dump(self, path: str):
        with open(path, "w") as f:
            json.dump(self.chrome_trace(), f)

    def clear(self):
        with self._lock:
            self._spans.clear()


GLOBAL_TRACER = Tracer()


_HIP_NODE_TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "graph", 5: "empty",
                   6: "wait_event", 7: "event_record"}


def graph_node_counts(graph) -> dict:
    """Node counts by type of a captured torch.cuda.CUDAGraph made with keep_graph=True
    (hipGraphGetNodes / hipGraphNodeGetType): how many kernel launches one replay issues."""
    import ctypes

    lib = ctypes.CDLL("libamdhip64.so")
    g = ctypes.c_void_p(int(graph.raw_cuda_graph()))
    n = ctypes.c_size_t(0)
    if lib.hipGraphGetNodes(g, None, ctypes.byref(n)) != 0:
        raise RuntimeError("hipGraphGetNodes failed")
    nodes = (ctypes.c_void_p * n.value)()
    if lib.hipGraphGetNodes(g, nodes, ctypes.byref(n)) != 0:
        raise RuntimeError("hipGraphGetNodes failed")
    out: dict = {}
    t = ctypes.c_int(0)
    for i in range(n.value):
        if lib.hipGraphNodeGetType(ctypes.c_void_p(nodes[i]), ctypes.byref(t)) != 0:
            raise RuntimeError("hipGraphNodeGetType failed")
        k = _HIP_NODE_TYPES.get(t.value, f"type{t.value}")
        out[k] = out.get(k, 0) + 1
    return out

"""Hardware-counter driver for the paged attention decode path (one query token per sequence,
whole-context items: the engine's decode_part_target rule for 64 / 128 rows), 20 dispatches
per case, plus event-timed us per dispatch and the K/V bytes per dispatch.

    rocprofv3 --pmc <counters> --output-format csv -d OUT -- python3 tools/pmc_decode_attn.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from attn_bench import setup  # noqa: E402

from pilottai_amd import ops  # noqa: E402

torch.manual_seed(0)
for rows in (64, 128):
    args, _, _, _ = setup([1] * rows, [600] * rows, part=4096)
    for _ in range(2):
        ops.paged_attention(*args)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        ops.paged_attention(*args)
    e.record()
    e.synchronize()
    kv = rows * 600 * 8 * 128 * 2 * 2
    us = s.elapsed_time(e) * 1000 / 20
    print(json.dumps({"rows": rows, "ctx": 600, "us": round(us, 2), "kv_MB": round(kv / 1e6, 1),
                      "TBps": round(kv / us / 1e6, 2)}), flush=True)

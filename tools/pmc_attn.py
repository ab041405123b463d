"""Hardware-counter driver for the paged attention prefill paths (32- vs 128-column items),
20 dispatches per case: prefill8x256 (8 chunks x 256 new tokens, ctx 768) and prefill2048.

    rocprofv3 --pmc <counters> --output-format csv -d OUT -- python3 tools/pmc_attn.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from attn_bench import setup  # noqa: E402

from pilottai_amd import ops  # noqa: E402

torch.manual_seed(0)
for ql, cl in (([256] * 8, [768] * 8), ([2048], [2048])):
    for qcols in (32, 128):
        args, _, _, _ = setup(ql, cl, qcols=qcols)
        for _ in range(20):
            ops.paged_attention(*args)
        torch.cuda.synchronize()

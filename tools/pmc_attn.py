"""Hardware-counter driver for the paged attention prefill paths, 20 dispatches per case
(cases and item widths from tools/attn_bench.py; one case per rocprofv3 run keeps the
per-kernel counters of one shape).

    rocprofv3 --pmc <counters> --output-format csv -d OUT -- python3 tools/pmc_attn.py --case step2048
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from attn_bench import setup  # noqa: E402

from pilottai_amd import ops  # noqa: E402

CASES = {"prefill8x256": ([256] * 8, [768] * 8), "prefill2048": ([2048], [2048]),
         "prefill4x512": ([512] * 4, [768] * 4), "step2048": ([512] * 4 + [1] * 40, [768] * 4 + [600] * 40)}
ap = argparse.ArgumentParser()
ap.add_argument("--case", default="prefill8x256,prefill2048")
ap.add_argument("--qcols", default="32,128")
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
torch.manual_seed(0)
for c in a.case.split(","):
    ql, cl = CASES[c]
    for qcols in [int(x) for x in a.qcols.split(",")]:
        args, _, _, _ = setup(ql, cl, qcols=qcols)
        for _ in range(a.reps):
            ops.paged_attention(*args)
        torch.cuda.synchronize()

"""Hardware-counter driver for the 256 x 256 prefill GEMM (csrc/ops/gemm_prefill.hip) vs
hipBLASLt: gate_up at M = 2,048 (whole tiles only, 896 tiles) and down at M = 2,048, 10
dispatches each.

    rocprofv3 --pmc <counters> --output-format csv -d OUT -- python3 tools/pmc_prefill.py [--shapes M:N:K,...]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd.engine.gemm_tuning import load_tuned_gemms  # noqa: E402
from pilottai_amd.ops import kernels  # noqa: E402

load_tuned_gemms("llama-3-8b", 1)
torch.manual_seed(0)
ap = argparse.ArgumentParser()
ap.add_argument("--shapes", default="2048:28672:4096,2048:4096:14336")
ap.add_argument("--variants", default="-1", help="prefill kernel families to run, e.g. 3,10")
ap.add_argument("--no-lib", action="store_true")
a = ap.parse_args()
for spec in a.shapes.split(","):
    M, N, K, bn = ([int(v) for v in spec.split(":")] + [256])[:4]
    w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    wp = kernels.pack_decode_weight(w)
    x = torch.randn(M, K, device="cuda").bfloat16()
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for v in (int(t) for t in a.variants.split(",")):
        for _ in range(10):
            kernels.prefill_gemm(x, wp, out=y, full=-1, splits=1, bn=bn, variant=v)
    for _ in range(0 if a.no_lib else 10):
        torch.nn.functional.linear(x, w)
    torch.cuda.synchronize()

"""Hardware-counter driver for the mid-size GEMM (csrc/ops/gemm_mid.hip) vs hipBLASLt,
cache-cold (weights rotate over >= 1 GB of copies), 20 dispatches per case:

  v1_gu256   variant 1 (2x2 waves, both operands LDS-DMA), gate_up M = 256, 256x128 tile
  v2_gu256   variant 2 (1x8 waves, weight VGPR ring), gate_up M = 256, 128x256 tile
  lib_gu256  hipBLASLt gate_up M = 256
  v2_dn256   variant 2, down M = 256, split-K 4
  lib_dn256  hipBLASLt down M = 256

    rocprofv3 --pmc <counters> --output-format csv -d OUT -- python3 tools/pmc_mid.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd.engine.gemm_tuning import load_tuned_gemms  # noqa: E402
from pilottai_amd.ops import kernels  # noqa: E402

load_tuned_gemms("llama-3-8b", 1)
torch.manual_seed(0)


def copies(N, K):
    n = max(2, int(1.0e9 / (N * K * 2)) + 1)
    return [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(n)]


def run(fn, n, iters=20):
    for i in range(iters):
        fn(i % n)
    torch.cuda.synchronize()


M = 256
ws = copies(28672, 4096)
wp = [kernels.pack_decode_weight(w) for w in ws]
x = torch.randn(M, 4096, device="cuda").bfloat16()
y = torch.empty(M, 28672, device="cuda", dtype=torch.bfloat16)
run(lambda i: kernels.mid_gemm(x, wp[i], out=y, fm=8, fn=4, splits=1, variant=1), len(wp))
run(lambda i: kernels.mid_gemm(x, wp[i], out=y, fm=8, fn=2, splits=1, variant=2, waves=8), len(wp))
run(lambda i: torch.nn.functional.linear(x, ws[i]), len(ws))
del ws, wp
torch.cuda.empty_cache()
ws = copies(4096, 14336)
wp = [kernels.pack_decode_weight(w) for w in ws]
x = torch.randn(M, 14336, device="cuda").bfloat16()
y = torch.empty(M, 4096, device="cuda", dtype=torch.bfloat16)
run(lambda i: kernels.mid_gemm(x, wp[i], out=y, fm=8, fn=1, splits=4, variant=2, waves=8), len(wp))
run(lambda i: torch.nn.functional.linear(x, ws[i]), len(ws))

"""Driver for hardware-counter passes (rocprofv3 --pmc) over the hot kernels, one
case each, cache-cold (weights rotate over >= 1.5 GB of copies):

  dec_gateup_m8   packed decode GEMM, gate_up + norm + SwiGLU, M = 8   (top kernel at 8 workers)
  dec_o_m8        packed decode GEMM, o_proj + residual, M = 8
  mid_down_m32    mid-size packed GEMM, down + residual, M = 32
  mid_down_m128   mid-size packed GEMM, down + residual, M = 128
  lib_down_m128   hipBLASLt (F.linear), down, M = 128
  attn_dec8       paged attention, 8 decode rows, ctx 1000, 256-key partitions
  attn_mix        paged attention, 64 decode rows (ctx 512) + 2 x 320 prefill

    rocprofv3 --pmc <counters> --output-format csv -d OUT -- python3 tools/pmc_kernels.py
"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd import ops  # noqa: E402
from pilottai_amd.ops import kernels  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from attn_bench import setup as attn_setup  # noqa: E402

ITERS = 20
torch.manual_seed(0)


def copies(N, K):
    n = max(2, int(1.5e9 / (N * K * 2)) + 1)
    return [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(n)]


def run(fn, n):
    for i in range(ITERS):
        fn(i % n)
    torch.cuda.synchronize()


# packed decode GEMMs
ws = copies(28672, 4096)
wp = [kernels.pack_decode_gate_up(w) for w in ws]
del ws
x = torch.randn(8, 4096, device="cuda").bfloat16()
run(lambda i: kernels.decode_gemm(x, wp[i], "silu", norm=True), len(wp))
del wp
ws = copies(4096, 4096)
wp = [kernels.pack_decode_weight(w) for w in ws]
r = torch.randn(8, 4096, device="cuda").bfloat16()
run(lambda i: kernels.decode_gemm(x, wp[i], "resid", resid=r), len(wp))
del ws, wp
torch.cuda.empty_cache()

# down projection: mid-size packed kernel at M = 32 and 128, hipBLASLt at 128
ws = copies(4096, 14336)
wp = [kernels.pack_decode_weight(w) for w in ws]
for M in (32, 128):
    xm = torch.randn(M, 14336, device="cuda").bfloat16()
    rm = torch.randn(M, 4096, device="cuda").bfloat16()
    run(lambda i: kernels.mid_gemm(xm, wp[i], "resid", resid=rm), len(wp))
run(lambda i: torch.nn.functional.linear(xm, ws[i]), len(ws))
del ws, wp
torch.cuda.empty_cache()

# attention
for ql, cl, part in (([1] * 8, [1000] * 8, 256), ([1] * 64 + [320, 320], [512] * 64 + [480, 480], 512)):
    args, _, _, _ = attn_setup(ql, cl, part=part)
    for _ in range(ITERS):
        ops.paged_attention(*args)
    torch.cuda.synchronize()
print("done", flush=True)

"""Hardware-counter driver: the packed decode GEMM with default-policy (variant 0) and
non-temporal (variant 1) weight loads, gate_up + norm + SwiGLU and down + residual at M = 8,
cache-cold (weights rotate over >= 1.5 GB of copies), 20 dispatches each. The two variants
are different kernel instantiations, so the counter summary separates them by name.

    rocprofv3 --pmc <counters> --output-format csv -d OUT -- python3 tools/pmc_nt.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd.ops import kernels  # noqa: E402

C = kernels.require_native()
torch.manual_seed(0)
M = 8
for N, K, epi, norm, pack in ((28672, 4096, "silu", True, kernels.pack_decode_gate_up),
                              (4096, 14336, "resid", False, kernels.pack_decode_weight)):
    n = max(2, int(1.5e9 / (N * K * 2)) + 1)
    wps = [pack((torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)) for _ in range(n)]
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    resid = torch.randn(M, N, device="cuda").to(torch.bfloat16) if epi == "resid" else None
    for v in (0, 1):
        C.decode_set_variant(v)
        for i in range(20):
            kernels.decode_gemm(x, wps[i % n], epi, norm=norm, resid=resid)
        torch.cuda.synchronize()
    del wps
    torch.cuda.empty_cache()
C.decode_set_variant(1)

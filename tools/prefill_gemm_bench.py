"""Prefill-shape GEMM survey (Llama-3-8B projections) on hipBLASLt: TFLOP/s per M.

    python tools/prefill_gemm_bench.py [M list] > out.jsonl

For each projection and token count M it times F.linear(x, W) with W stored
[N, K] (the engine's layout) and x @ Wt with W stored [K, N], so the table
shows both which M the library handles well and whether the layout matters.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

shapes = [(6144, 4096, "qkv"), (4096, 4096, "o"), (28672, 4096, "gate_up"), (4096, 14336, "down")]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / iters


Ms = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "128,256,512,768,1024,2048").split(",")]
for N, K, name in shapes:
    w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    wt = w.t().contiguous()
    for M in Ms:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        t_nk = timeit(lambda: torch.nn.functional.linear(x, w))
        t_kn = timeit(lambda: x @ wt)
        t_sw = timeit(lambda: torch.nn.functional.linear(w, x))  # C^T = W X^T (M <-> N swapped)
        fl = 2.0 * M * N * K
        print(json.dumps({"shape": name, "M": M, "us_NK": round(t_nk, 1), "us_KN": round(t_kn, 1),
                          "us_swap": round(t_sw, 1),
                          "TF_NK": round(fl / t_nk / 1e6, 1), "TF_KN": round(fl / t_kn / 1e6, 1),
                          "TF_swap": round(fl / t_sw / 1e6, 1)}), flush=True)

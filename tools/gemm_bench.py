"""Decode-shape GEMM micro-benchmark, cache-cold: own skinny MFMA kernel (variants) vs hipBLASLt.

Each measurement rotates over enough weight copies (>= 1.5 GB) that no weight is
served from the 256 MB Infinity Cache, as in a real 15 GB decode step.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd.ops import kernels  # noqa: E402

C = kernels.require_native()
shapes = [(6144, 4096, "qkv"), (4096, 4096, "o"), (28672, 4096, "gate_up"), (4096, 14336, "down"),
          (128256, 4096, "lm_head")]


def timeit(fn, ncopies, iters=40):
    for i in range(3):
        fn(i % ncopies)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i % ncopies)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / iters


Ms = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "8,16,32,64,128").split(",")]
for N, K, name in shapes:
    gb = N * K * 2 / 1e9
    ncopies = max(2, int(1.5 / gb) + 1)
    ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(ncopies)]
    for M in Ms:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        row = {"M": M, "shape": name}
        row["lib"] = round(timeit(lambda i: torch.nn.functional.linear(x, ws[i]), ncopies), 1)
        for v in range(4):
            C.skinny_set_variant(v)
            row[f"v{v}"] = round(timeit(lambda i: C.skinny_gemm(y, x, ws[i]), ncopies), 1)
        C.skinny_set_variant(0)
        best = min(row[f"v{v}"] for v in range(4))
        row["lib_TBps"] = round(gb / row["lib"] * 1e3, 2)
        row["best_TBps"] = round(gb / best * 1e3, 2)
        print(json.dumps(row), flush=True)
    del ws
    torch.cuda.empty_cache()

"""Does a weight stream from the Infinity Cache (MALL) instead of HBM make the decode
projections faster? Per Llama-3-8B decode projection at M=8: the packed decode GEMM
(csrc/ops/gemm_decode.hip) cache-cold (rotating over >= 1.5 GB of copies), warm (the same
copy again), and right after a strided "touch" pass over its weights (one 2-byte read per
128-B line, the GEMM timed alone) — the case a side-stream prefetch during attention
would create.

    python tools/mall_warm_bench.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd.ops import kernels  # noqa: E402

shapes = [(6144, 4096, "qkv"), (4096, 4096, "o"), (28672, 4096, "gate_up"), (4096, 14336, "down")]
M = 8
ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731


def gemm_time(fn, pre=None, iters=20):
    ts = []
    for i in range(iters + 3):
        if pre is not None:
            pre(i)
        a, b = ev(), ev()
        a.record()
        fn(i)
        b.record()
        torch.cuda.synchronize()
        if i >= 3:
            ts.append(a.elapsed_time(b) * 1000)
    ts.sort()
    return round(ts[len(ts) // 2], 1)


for N, K, name in shapes:
    gb = N * K * 2 / 1e9
    nc = max(2, int(1.5 / gb) + 1)
    ws = [kernels.pack_decode_weight((torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)) for _ in range(nc)]
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    flat = [w.view(-1) for w in ws]
    sink = torch.empty((), device="cuda")
    cold = gemm_time(lambda i: kernels.decode_gemm(x, ws[i % nc], "plain", out=y))
    warm = gemm_time(lambda i: kernels.decode_gemm(x, ws[0], "plain", out=y),
                     pre=lambda i: kernels.decode_gemm(x, ws[0], "plain", out=y))
    touched = gemm_time(lambda i: kernels.decode_gemm(x, ws[i % nc], "plain", out=y),
                        pre=lambda i: sink.copy_(flat[i % nc][::64].float().sum()))
    a, b = ev(), ev()
    a.record()
    for i in range(10):
        sink.copy_(flat[i % nc][::64].float().sum())
    b.record()
    torch.cuda.synchronize()
    print(json.dumps({"shape": name, "M": M, "MB": round(gb * 1e3, 1), "cold_us": cold, "warm_us": warm,
                      "after_touch_us": touched, "touch_pass_us": round(a.elapsed_time(b) * 100, 1),
                      "cold_TBps": round(gb / cold * 1e3, 2), "warm_TBps": round(gb / warm * 1e3, 2)}), flush=True)
    del ws, flat
    torch.cuda.empty_cache()

"""Would splitting a 2,048-token step into two independent 1,024-token halves on two HIP
streams fill the GPU better? Times, per Llama-3-8B projection: one M=2048 GEMM, two
M=1024 GEMMs back to back, and two M=1024 GEMMs on two streams at once (hipBLASLt with
the shipped tuned solutions, cache-warm).

    python tools/dual_stream_gemm.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from pilottai_amd.engine.gemm_tuning import load_tuned_gemms  # noqa: E402

load_tuned_gemms("llama-3-8b", 1)
shapes = [(6144, 4096, "qkv"), (4096, 4096, "o"), (28672, 4096, "gate_up"), (4096, 14336, "down")]
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def t(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) * 1000 / iters, 1)


for N, K, name in shapes:
    w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    x = torch.randn(2048, K, device="cuda").to(torch.bfloat16)
    xa, xb = x[:1024].contiguous(), x[1024:].contiguous()
    full = t(lambda: F.linear(x, w))
    seq = t(lambda: (F.linear(xa, w), F.linear(xb, w)))

    def dual():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            F.linear(xa, w)
        with torch.cuda.stream(s2):
            F.linear(xb, w)
        cur.wait_stream(s1)
        cur.wait_stream(s2)
    print(json.dumps({"shape": name, "m2048_us": full, "two_m1024_seq_us": seq, "two_m1024_dual_us": t(dual)}),
          flush=True)

"""A/B of packed decode-GEMM kernel variants (csrc/ops/gemm_decode.hip g_dg_variant) on the
model's fused forms, cache-cold (weights rotated over >= 1.5 GB), interleaved rounds in
one process; prints one JSON line per (shape, M) with the per-variant median us.

    python tools/decode_variant_ab.py [--variants 0,1] [--ms 8,16,32] [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd.ops import kernels  # noqa: E402

C = kernels.require_native()
ap = argparse.ArgumentParser()
ap.add_argument("--variants", default="0,1")
ap.add_argument("--ms", default="8,16,32")
ap.add_argument("--rounds", type=int, default=5)
a = ap.parse_args()
variants = [int(v) for v in a.variants.split(",")]
shapes = [(6144, 4096, "qkv", "plain", True), (4096, 4096, "o", "resid", False),
          (28672, 4096, "gate_up", "silu", True), (4096, 14336, "down", "resid", False),
          (128256, 4096, "lm_head", "plain", False)]


def timeit(fn, ncopies, iters=30):
    for i in range(3):
        fn(i % ncopies)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for i in range(iters):
        fn(i % ncopies)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / iters


torch.manual_seed(0)
for N, K, name, epi, norm in shapes:
    gb = N * K * 2 / 1e9
    ncopies = max(2, int(1.5 / gb) + 1)
    ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(ncopies)]
    pack = kernels.pack_decode_gate_up if epi == "silu" else kernels.pack_decode_weight
    wps = [pack(w) for w in ws]
    del ws
    for M in [int(m) for m in a.ms.split(",")]:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        resid = torch.randn(M, N, device="cuda").to(torch.bfloat16) if epi == "resid" else None
        NO = N // 2 if epi == "silu" else N
        yo = torch.empty(M, NO, dtype=torch.bfloat16, device="cuda")
        fn = lambda i: kernels.decode_gemm(x, wps[i], epi, norm=norm, resid=resid, out=yo)  # noqa: E731
        times = {v: [] for v in variants}
        outs = {}
        for _ in range(a.rounds):
            for v in variants:
                C.decode_set_variant(v)
                times[v].append(timeit(fn, ncopies))
        for v in variants:
            C.decode_set_variant(v)
            outs[v] = kernels.decode_gemm(x, wps[0], epi, norm=norm, resid=resid).float()
        row = {"shape": name, "M": M, "GB": round(gb, 3)}
        for v in variants:
            med = statistics.median(times[v])
            row[f"v{v}_us"] = round(med, 2)
            row[f"v{v}_TBps"] = round(gb / med * 1e3, 2)
            row[f"v{v}_same"] = bool(torch.equal(outs[v], outs[variants[0]]))
        print(json.dumps(row), flush=True)
    del wps
    torch.cuda.empty_cache()
C.decode_set_variant(1)  # the library default

"""Decode-shape projection micro-benchmark, cache-cold (Llama-3-8B shapes).

Compares, per (M, projection): hipBLASLt (torch linear), the row-major skinny
MFMA kernel (csrc/ops/gemm_skinny.hip) and the packed-weight decode kernel
(csrc/ops/gemm_decode.hip) over its (tile width, waves) configurations, plus the
fused forms the model uses (norm-folded QKV, norm+SwiGLU gate_up, residual O/down).
Every measurement rotates over >= 1.5 GB of weight copies so W streams from
HBM, not the 256 MB Infinity Cache. Also checks each result against fp32.

    python tools/decode_gemm_bench.py [M list, default 1,8,16,32,64] > out.jsonl
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd.ops import kernels  # noqa: E402

C = kernels.require_native()
# (N, K, name, epi, norm)
shapes = [(6144, 4096, "qkv", "plain", True), (4096, 4096, "o", "resid", False),
          (28672, 4096, "gate_up", "silu", True), (4096, 14336, "down", "resid", False),
          (128256, 4096, "lm_head", "plain", False)]
CFGS = [(1, 8, 1), (1, 16, 1), (2, 8, 1), (2, 16, 1), (4, 8, 1), (2, 8, 2), (2, 8, 4), (2, 16, 2), (4, 8, 2),
        (4, 8, 4), (1, 8, 2), (1, 8, 4), (2, 4, 4), (4, 4, 4)]


def timeit(fn, ncopies, iters=30):
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


Ms = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,8,16,32,64").split(",")]
torch.manual_seed(0)
for N, K, name, epi, norm in shapes:
    gb = N * K * 2 / 1e9
    ncopies = max(2, int(1.5 / gb) + 1)
    ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(ncopies)]
    pack = kernels.pack_decode_gate_up if epi == "silu" else kernels.pack_decode_weight
    wps = [pack(w) for w in ws]
    for M in Ms:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        resid = torch.randn(M, N, device="cuda").to(torch.bfloat16) if epi == "resid" else None
        y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        row = {"M": M, "shape": name, "GB": round(gb, 3)}
        row["lib"] = round(timeit(lambda i: torch.nn.functional.linear(x, ws[i]), ncopies), 1)
        if M <= 128:
            row["skinny"] = round(timeit(lambda i: C.skinny_gemm(y, x, ws[i]), ncopies), 1)
        # plain packed kernel over configs
        best = None
        bestk = None
        for nt, wv, sp in CFGS:
            if (N // 16) % nt:
                continue
            try:
                t = timeit(lambda i: kernels.decode_gemm(x, wps[i], "plain", out=y, nt=nt, waves=wv, splits=sp),
                           ncopies)
            except (ValueError, RuntimeError):
                continue
            row[f"p{nt}x{wv}s{sp}"] = round(t, 1)
            if best is None or t < best:
                best, bestk = t, f"p{nt}x{wv}s{sp}"
        row["best_cfg"] = bestk
        row["auto"] = round(timeit(lambda i: kernels.decode_gemm(x, wps[i], "plain", out=y), ncopies), 1)
        ref = x.float() @ ws[0].float().T
        got = kernels.decode_gemm(x, wps[0], "plain").float()
        row["plain_err"] = float((got - ref).abs().max() / ref.abs().max())
        # fused form used by the model
        if epi != "plain" or norm:
            NO = N // 2 if epi == "silu" else N
            yo = torch.empty(M, NO, dtype=torch.bfloat16, device="cuda")
            row["fused"] = round(timeit(lambda i: kernels.decode_gemm(x, wps[i], epi, norm=norm, resid=resid,
                                                                       out=yo), ncopies), 1)
            acc = ref
            if norm:
                acc = acc * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-5)
            if epi == "silu":
                acc = torch.nn.functional.silu(acc[:, :NO]) * acc[:, NO:]
            elif epi == "resid":
                acc = acc + resid.float()
            got = kernels.decode_gemm(x, wps[0], epi, norm=norm, resid=resid).float()
            row["fused_err"] = float((got - acc).abs().max() / acc.abs().max())
        row["lib_TBps"] = round(gb / row["lib"] * 1e3, 2)
        row["best_TBps"] = round(gb / best * 1e3, 2) if best else None
        row["auto_TBps"] = round(gb / row["auto"] * 1e3, 2)
        print(json.dumps(row), flush=True)
    del ws, wps
    torch.cuda.empty_cache()

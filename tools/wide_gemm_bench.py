"""Small-batch projection micro-benchmark (Llama-3-8B shapes), cache-cold:
hipBLASLt (with the shipped tuned solutions) vs csrc/ops/gemm_wide.hip over its
(ntw, waves, splits) configurations, with an fp32 check.

    python tools/wide_gemm_bench.py [M list, default 24,32,48,64,96,128] > out.jsonl
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd.engine.gemm_tuning import load_tuned_gemms  # noqa: E402
from pilottai_amd.ops import kernels  # noqa: E402

load_tuned_gemms("llama-3-8b", 1)
shapes = [(6144, 4096, "qkv"), (4096, 4096, "o"), (28672, 4096, "gate_up"), (4096, 14336, "down")]
FUSED = {"qkv": ("rope_perm", True), "o": ("resid", False), "gate_up": ("silu", True), "down": ("resid", False)}
CFGS = [(1, 4, 0), (2, 4, 0), (1, 8, 0), (1, 4, 1), (1, 4, 2), (1, 4, 4), (1, 4, 8), (2, 4, 1), (2, 4, 2)]


def timeit(fn, ncopies, iters=20):
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


Ms = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "24,32,48,64,96,128").split(",")]
torch.manual_seed(0)
for N, K, name in shapes:
    gb = N * K * 2 / 1e9
    ncopies = max(2, int(1.5 / gb) + 1)
    ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(ncopies)]
    wps = [kernels.pack_decode_weight(w) for w in ws]
    epi, nrm = FUSED[name]
    fpack = {"silu": kernels.pack_decode_gate_up, "rope_perm": kernels.pack_decode_qkv_rope}.get(epi)
    fps = [fpack(w) for w in ws] if fpack else wps
    for M in Ms:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        row = {"M": M, "shape": name}
        row["lib"] = round(timeit(lambda i: torch.nn.functional.linear(x, ws[i]), ncopies), 1)
        best = None
        for ntw, wv, sp in CFGS:
            key = f"n{ntw}w{wv}s{sp}"
            try:
                t = timeit(lambda i: kernels.wide_gemm(x, wps[i], out=y, ntw=ntw, waves=wv, splits=sp), ncopies)
            except (ValueError, RuntimeError):
                continue
            row[key] = round(t, 1)
            best = (t, key) if best is None or t < best[0] else best
        row["auto"] = round(timeit(lambda i: kernels.wide_gemm(x, wps[i], out=y), ncopies), 1)
        resid = torch.randn(M, N, device="cuda").to(torch.bfloat16) if epi == "resid" else None
        yo = torch.empty(M, N // 2 if epi == "silu" else N, dtype=torch.bfloat16, device="cuda")
        row["fused"] = round(timeit(lambda i: kernels.wide_gemm(x, fps[i], epi, resid=resid, norm=nrm, out=yo),
                                    ncopies), 1)
        ref = x.float() @ ws[0].float().T
        got = kernels.wide_gemm(x, wps[0]).float()
        row["err"] = float((got - ref).abs().max() / ref.abs().max())
        row["best"] = best[1] if best else None
        row["lib_TBps"] = round(gb / row["lib"] * 1e3, 2)
        row["auto_TBps"] = round(gb / row["auto"] * 1e3, 2)
        print(json.dumps(row), flush=True)
    del ws, wps, fps
    torch.cuda.empty_cache()

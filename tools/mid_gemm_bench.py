"""Mid-size projection micro-benchmark (Llama-3-8B shapes, 48 < M <= 512), cache-cold:
hipBLASLt (shipped tuned solutions) vs csrc/ops/gemm_mid.hip over its (fm, fn, splits)
configurations, with an fp32 check of every configuration.

    python tools/mid_gemm_bench.py [M list] [--quick] [--fused-sweep] > out.jsonl

Each row: M, shape, lib (us), every config "f{fm}x{fn}s{S}" (us), auto (the default
plan), fused (the engine's epilogue: norm + rope_perm / silu / resid), err of the worst
config (max |err| / max |ref|), TB/s of weight traffic for lib and the best config.
"""
import json
import re
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd.engine.gemm_tuning import load_tuned_gemms  # noqa: E402
from pilottai_amd.ops import kernels  # noqa: E402

load_tuned_gemms("llama-3-8b", 1)
shapes = [(6144, 4096, "qkv"), (4096, 4096, "o"), (28672, 4096, "gate_up"), (4096, 14336, "down")]
FUSED = {"qkv": ("rope_perm", True), "o": ("resid", False), "gate_up": ("silu", True), "down": ("resid", False)}


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


args = [a for i, a in enumerate(sys.argv[1:], 1) if not a.startswith("--") and not sys.argv[i - 1].startswith("--")]
quick = "--quick" in sys.argv
fused_sweep = "--fused-sweep" in sys.argv  # time every config in the engine's epilogue form
Ms = [int(v) for v in (args[0] if args else "64,96,128,192,256,384,512").split(",")]
def _opt(name, default):
    for i, v in enumerate(sys.argv):
        if v == name and i + 1 < len(sys.argv):
            return [int(x) for x in sys.argv[i + 1].split(",")]
    return default


_FMS, _FNS, _SS = _opt("--fms", (1, 2, 4, 8)), _opt("--fns", (2, 4)), _opt("--splits", (1, 2, 3, 4, 6))
_SHAPES = None
for _i, _v in enumerate(sys.argv):
    if _v == "--shapes" and _i + 1 < len(sys.argv):
        _SHAPES = sys.argv[_i + 1].split(",")
if _SHAPES:
    shapes = [s for s in shapes if s[2] in _SHAPES]
CFGS = [(1, fm, fn, 4, S) for fm in _FMS for fn in _FNS for S in _SS]
torch.manual_seed(0)
for N, K, name in shapes:
    gb = N * K * 2 / 1e9
    ncopies = max(2, int(1.0 / gb) + 1)
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
        ref = x.float() @ ws[0].float().T
        resid = torch.randn(M, N, device="cuda").to(torch.bfloat16) if epi == "resid" else None
        yo = torch.empty(M, N // 2 if epi == "silu" else N, dtype=torch.bfloat16, device="cuda")
        ssv = kernels.row_sumsq(x)
        best, worst_err = None, 0.0
        for var, fm, fn, wv, S in ([] if quick else CFGS):
            bm = (32 if var == 1 else 16) * fm
            if bm > 2 * max(64, M) or (bm < M / 4 and bm < 256):  # row tile far from the step size: skip
                continue
            key = f"v{var}f{fm}x{fn}w{wv}s{S}"
            try:
                got = kernels.mid_gemm(x, wps[0], out=y, fm=fm, fn=fn, splits=S).float()
            except (ValueError, RuntimeError):
                continue
            worst_err = max(worst_err, float((got - ref).abs().max() / ref.abs().max()))
            if fused_sweep:
                t = timeit(lambda i: kernels.mid_gemm(x, fps[i], epi, resid=resid, norm=nrm, out=yo, ss_in=ssv,
                                                      fm=fm, fn=fn, splits=S), ncopies)
            else:
                t = timeit(lambda i: kernels.mid_gemm(x, wps[i], out=y, fm=fm, fn=fn, splits=S), ncopies)
            row[key] = round(t, 1)
            best = (t, key) if best is None or t < best[0] else best
        row["plan"] = kernels.require_native().mid_gemm_plan(M, N, K, kernels.MID_EPI["plain"])
        got = kernels.mid_gemm(x, wps[0], out=y).float()
        worst_err = max(worst_err, float((got - ref).abs().max() / ref.abs().max()))
        row["auto"] = round(timeit(lambda i: kernels.mid_gemm(x, wps[i], out=y), ncopies), 1)
        bfm, bfn, bS = (int(v) for v in re.match(r"v1f(\d+)x(\d+)w4s(\d+)", best[1]).groups()) if best else (0, 0, 0)
        row["fused"] = round(timeit(lambda i: kernels.mid_gemm(x, fps[i], epi, resid=resid, norm=nrm, out=yo,
                                                               ss_in=ssv, fm=bfm, fn=bfn, splits=bS), ncopies), 1)
        row["err"] = worst_err
        row["best"] = best[1] if best else "auto"
        tb = best[0] if best else row["auto"]
        row["lib_TBps"] = round(gb / row["lib"] * 1e3, 2)
        row["best_TBps"] = round(gb / tb * 1e3, 2)
        row["speedup"] = round(row["lib"] / tb, 2)
        print(json.dumps(row), flush=True)
    del ws, wps, fps
    torch.cuda.empty_cache()

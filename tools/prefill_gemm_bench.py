"""Large-M projection benchmark (Llama-3-8B shapes, prefill-heavy steps): tuned hipBLASLt vs
the mid path (csrc/ops/gemm_mid.hip) vs the 256 x 256 prefill kernel
(csrc/ops/gemm_prefill.hip) over its (whole tiles, K-slices) decompositions, each checked
against fp32. Variants are timed in interleaved rounds in one process (guide §5.4 rule 24).

    python tools/prefill_gemm_bench.py [--M 512,1024,2048] [--rounds 3] [--out file.jsonl]

Row: M, shape, us per variant (median of rounds), TFLOP/s of the best, err of pf_default.
"fused" variants run the engine's epilogue (norm + rope_perm / silu / resid).
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd.engine.gemm_tuning import load_tuned_gemms  # noqa: E402
from pilottai_amd.ops import kernels  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--M", default="512,768,1024,1536,2048")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--shapes", default="qkv,o,gate_up,down")
ap.add_argument("--variants", default="")
ap.add_argument("--out", default="")
ap.add_argument("--cold-mb", type=int, default=0,
                help="rotate enough weight copies that their total exceeds this many MB (e.g. 1024: more than the "
                     "256 MB Infinity Cache, as in the engine, where every step streams 15 GB of weights)")
a = ap.parse_args()
load_tuned_gemms("llama-3-8b", 1)
SHAPES = {"sq": (4096, 4096), "qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
FUSED = {"sq": ("resid", False), "qkv": ("rope_perm", True), "o": ("resid", False), "gate_up": ("silu", True), "down": ("resid", False)}
out_f = open(a.out, "a") if a.out else None


def timeit(fn, ncopies):
    for i in range(2):
        fn(i % ncopies)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(a.iters):
        fn(i % ncopies)
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1000 / a.iters


C = kernels.require_native()


def v0(fn, v=1):  # prefill kernel family v for this call (1 read-ahead, 3 ping-pong, 8 / 9 tail forms)
    C.prefill_set_variant(v)
    try:
        return fn()
    finally:
        C.prefill_set_variant(-1)


torch.manual_seed(0)
for name in a.shapes.split(","):
    N, K = SHAPES[name]
    gb = N * K * 2 / 1e9
    ncopies = max(2, -(-a.cold_mb * 1_000_000 // (N * K * 2))) if a.cold_mb else 2
    ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(ncopies)]
    wps = [kernels.pack_decode_weight(w) for w in ws]
    epi, nrm = FUSED[name]
    fpack = {"silu": kernels.pack_decode_gate_up, "rope_perm": kernels.pack_decode_qkv_rope}.get(epi)
    fps = [fpack(w) for w in ws] if fpack else wps
    for M in [int(v) for v in a.M.split(",")]:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        NO = N // 2 if epi == "silu" else N
        yf = torch.empty(M, NO, dtype=torch.bfloat16, device="cuda")
        resid = torch.randn(M, N, device="cuda").to(torch.bfloat16) if epi == "resid" else None
        ss = kernels.row_sumsq(x)
        full_default, s_default, _, bn_default = kernels.require_native().prefill_gemm_plan(M, N, K)
        variants = {
            "lib": lambda i: torch.nn.functional.linear(x, ws[i]),
            "mid": lambda i: kernels.mid_gemm(x, wps[i], "plain", out=y),
            "pf_default": lambda i: kernels.prefill_gemm(x, wps[i], "plain", out=y),
            "pf256": lambda i: kernels.prefill_gemm(x, wps[i], "plain", out=y, bn=256),
            "pf128": lambda i: v0(lambda: kernels.prefill_gemm(x, wps[i], "plain", out=y, bn=128), 1),
            "pp128": lambda i: v0(lambda: kernels.prefill_gemm(x, wps[i], "plain", out=y, full=-1, splits=1, bn=128), 3),
            "pp128_fused": lambda i: v0(lambda: kernels.prefill_gemm(x, fps[i], epi, out=yf if epi == "silu" else y,
                                                                    resid=resid, norm=nrm, ss_in=ss if nrm else None,
                                                                    full=-1, splits=1, bn=128), 3),
            "pf128_s2": lambda i: kernels.prefill_gemm(x, wps[i], "plain", out=y, bn=128, full=0, splits=2),
            "pf128_fused": lambda i: kernels.prefill_gemm(x, fps[i], epi, out=yf if epi == "silu" else y, resid=resid,
                                                          norm=nrm, ss_in=ss if nrm else None, bn=128),
            "pp": lambda i: v0(lambda: kernels.prefill_gemm(x, wps[i], "plain", out=y, bn=256), 9),
            "pp_mix": lambda i: v0(lambda: kernels.prefill_gemm(x, wps[i], "plain", out=y, bn=256), 8),
            "pp_mix_fused": lambda i: v0(lambda: kernels.prefill_gemm(x, fps[i], epi, out=yf if epi == "silu" else y,
                                                                     resid=resid, norm=nrm, ss_in=ss if nrm else None,
                                                                     bn=256), 8),
            "pp_whole": lambda i: v0(lambda: kernels.prefill_gemm(x, wps[i], "plain", out=y, full=-1, splits=1, bn=256), 3),
            "pp_s2": lambda i: v0(lambda: kernels.prefill_gemm(x, wps[i], "plain", out=y, full=0, splits=2, bn=256), 3),
            "pp_fused": lambda i: v0(lambda: kernels.prefill_gemm(x, fps[i], epi, out=yf if epi == "silu" else y,
                                                                 resid=resid, norm=nrm, ss_in=ss if nrm else None,
                                                                 bn=256), 3),
            "pf_whole": lambda i: kernels.prefill_gemm(x, wps[i], "plain", out=y, full=-1, splits=1, bn=256),
            "pf_s2": lambda i: kernels.prefill_gemm(x, wps[i], "plain", out=y, full=0, splits=2),
            "pf_s3": lambda i: kernels.prefill_gemm(x, wps[i], "plain", out=y, full=0, splits=3),
            "pf_s4": lambda i: kernels.prefill_gemm(x, wps[i], "plain", out=y, full=0, splits=4),
            "pf_fused": lambda i: kernels.prefill_gemm(x, fps[i], epi, out=yf if epi == "silu" else y, resid=resid,
                                                       norm=nrm, ss_in=ss if nrm else None),
            "mid_fused": lambda i: kernels.mid_gemm(x, fps[i], epi, out=yf if epi == "silu" else y, resid=resid,
                                                    norm=nrm, ss_in=ss if nrm else None),
        }
        for bn_ in (192, 256, 128):  # 256 x bn_ ping-pong tiles, plain and fused
            if N % bn_ == 0:
                variants[f"pp{bn_}w"] = (lambda bn_: lambda i: v0(lambda: kernels.prefill_gemm(
                    x, wps[i], "plain", out=y, bn=bn_), 3))(bn_)
                variants[f"pp{bn_}w_fused"] = (lambda bn_: lambda i: v0(lambda: kernels.prefill_gemm(
                    x, fps[i], epi, out=yf if epi == "silu" else y, resid=resid, norm=nrm,
                    ss_in=ss if nrm else None, bn=bn_), 3))(bn_)
        # the 3-stage 256 x 128 kernel (variant 1) with the engine's epilogue
        variants["n128v1_fused"] = lambda i: v0(lambda: kernels.prefill_gemm(
            x, fps[i], epi, out=yf if epi == "silu" else y, resid=resid, norm=nrm, ss_in=ss if nrm else None,
            bn=128), 1)
        if name == "qkv":  # the engine's qkv call: RMSNorm folded, RoPE + paged KV write epilogue
            from pilottai_amd.ops import reference as _ref
            H, KV = 32, 8
            NB = (M + 15) // 16 + 4
            cs = _ref.rope_cos_sin(8192).cuda()
            pos = torch.arange(M, dtype=torch.int32, device="cuda")
            slots = torch.arange(M, dtype=torch.int32, device="cuda")
            kc = torch.zeros(NB, KV, 16, 16, 8, dtype=torch.bfloat16, device="cuda")
            vc = torch.zeros(NB, KV, 128, 16, dtype=torch.bfloat16, device="cuda")
            qo = torch.empty(M, H, 128, dtype=torch.bfloat16, device="cuda")
            for bn_ in (192, 256, 128):
                variants[f"ropekv{bn_}"] = (lambda bn_: lambda i: kernels.prefill_qkv_rope(
                    x, fps[i], 1e-5, qo, kc, vc, pos, slots, cs, H, KV, ss_in=ss, bn=bn_, variant=3))(bn_)
        for bn_ in (128, 256):  # fused epilogue on an explicit (whole tiles, K-slices) decomposition
            for S_ in (1, 2, 3, 4, 6, 8, 10):
                variants[f"pf{bn_}_s{S_}_fused"] = (lambda bn_, S_: lambda i: kernels.prefill_gemm(
                    x, fps[i], epi, out=yf if epi == "silu" else y, resid=resid, norm=nrm,
                    ss_in=ss if nrm else None, bn=bn_, full=0 if S_ > 1 else -1, splits=S_))(bn_, S_)
        if a.variants:
            variants = {k: v for k, v in variants.items() if k in a.variants.split(",")}
        times = {k: [] for k in variants}
        for _ in range(a.rounds):
            for k, fn in variants.items():
                try:
                    times[k].append(timeit(fn, ncopies))
                except (ValueError, RuntimeError):
                    times[k].append(float("nan"))
        row = {"M": M, "shape": name, "plan": [full_default, s_default, bn_default]}
        for k in variants:
            row[k] = round(statistics.median(times[k]), 1)
        flop = 2.0 * M * N * K
        best = min((v, k) for k, v in row.items() if k in variants and v == v)
        row["best"] = best[1]
        row["tflops_best"] = round(flop / best[0] / 1e6, 1)
        row["tflops_lib"] = round(flop / row["lib"] / 1e6, 1) if "lib" in row else None
        if "pf_default" in row:
            row["tflops_pf"] = round(flop / row["pf_default"] / 1e6, 1)
            ref = x.float() @ ws[0].float().T
            for bn in (256, 128):
                yy = kernels.prefill_gemm(x, wps[0], "plain", out=y, bn=bn)
                row[f"err_pf{bn}"] = float(((yy.float() - ref).abs().max() / ref.abs().max()))
        if "pp128" in variants:
            ref = x.float() @ ws[0].float().T
            y.fill_(float("nan"))
            yy = v0(lambda: kernels.prefill_gemm(x, wps[0], "plain", out=y, full=-1, splits=1, bn=128), 3)
            row["err_pp128"] = float(((yy.float() - ref).abs().max() / ref.abs().max()))
        for bn_ in (192, 256, 128):
            if f"pp{bn_}w" in variants:
                ref = x.float() @ ws[0].float().T
                y.fill_(float("nan"))
                yy = v0(lambda: kernels.prefill_gemm(x, wps[0], "plain", out=y, bn=bn_), 3)
                row[f"err_pp{bn_}w"] = float(((yy.float() - ref).abs().max() / ref.abs().max()))
        if any(k.startswith("pp") for k in variants):
            ref = x.float() @ ws[0].float().T
            for nm, kw, vv in (("pp", {}, 3), ("pp_whole", dict(full=-1, splits=1), 3), ("pp_s2", dict(full=0, splits=2), 3),
                               ("pp_mix", {}, 8)):
                if nm not in variants:
                    continue
                try:
                    y.fill_(float("nan"))
                    yy = v0(lambda: kernels.prefill_gemm(x, wps[0], "plain", out=y, bn=256, **kw), vv)
                    row[f"err_{nm}"] = float(((yy.float() - ref).abs().max() / ref.abs().max()))
                except (ValueError, RuntimeError):
                    row[f"err_{nm}"] = None
        print(json.dumps(row), flush=True)
        if out_f:
            out_f.write(json.dumps(row) + "\n")
            out_f.flush()

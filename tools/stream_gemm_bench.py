"""Mid-step projection benchmark (Llama-3-8B shapes, 16 < M <= 256): the weight-streaming
kernel (csrc/ops/gemm_stream.hip) over its decompositions vs the round-3 engine choice (mid
kernel / 256 x 128 prefill kernel per LlamaModel.PF_CFG), every variant with the engine's
fused epilogue (norm + RoPE-perm / SwiGLU / residual). Weights are rotated over enough copies
to exceed the 256 MB Infinity Cache (cold, as in the engine, where every step streams 15 GB).
Variants are timed in interleaved rounds in one process (guide §5.4 rule 24).

    python tools/stream_gemm_bench.py [--M 32,64,128,256] [--shapes qkv,o,gate_up,down] [--sweep]
        [--out file.jsonl]

Row: M, shape, us of the engine's round-3 choice, of the stream default plan, of the best
swept plan (with the plan), and the weight-stream rate of the best (TB/s).
"""
import argparse
import itertools
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd.models.llama import LlamaModel  # noqa: E402
from pilottai_amd.ops import kernels  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--M", default="32,48,64,96,128,160,192,256")
ap.add_argument("--shapes", default="qkv,o,gate_up,down")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--slabs", default="uncached", help="comma list of slab memories to time: uncached (shipped), "
                "cached_rel (cached memory + producer release), cached (cached, no release: timing only)")
ap.add_argument("--cold-mb", type=int, default=1024)
ap.add_argument("--sweep", action="store_true", help="time every valid stream decomposition too")
ap.add_argument("--row-groups", action="store_true", help="sweep also splits the rows into 2-4 groups")
ap.add_argument("--krot", action="store_true", help="also time the default plan with rotated K-chunk order")
ap.add_argument("--rel-ab", action="store_true",
                help="also time the default plan without the producer release (rel 0; shipped: ops.STREAM_REL)")
ap.add_argument("--out", default="")
a = ap.parse_args()
SHAPES = {"qkv": (6144, 4096, "rope_perm", True), "o": (4096, 4096, "resid", False),
          "gate_up": (28672, 4096, "silu", True), "down": (4096, 14336, "resid", False),
          "lm_head": (128256, 4096, "plain", False)}
WAVE_SHAPES = [(1, 4, 1), (2, 4, 1), (3, 4, 1), (4, 4, 1), (1, 4, 2), (2, 2, 2), (3, 2, 2), (1, 6, 1), (2, 6, 1),
               (2, 7, 1), (2, 8, 1), (1, 8, 1)]
out_f = open(a.out, "a") if a.out else None


def timeit(fn, ncopies):
    """Device time per call: one hipGraph holds `ncopies` calls (rotating the weight copies,
    cache-cold like the engine's layer chain) and is replayed; eager launches from Python
    would measure the host (~15 us per call) for kernels this short."""
    for i in range(2):
        fn(i % ncopies)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(ncopies):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        g.replay()
    e.record()
    e.synchronize()
    del g
    return s.elapsed_time(e) * 1000 / (a.iters * ncopies)


def plans_for(M, N, K, epi):
    rgs = []
    for mg in (2, 4, 8):  # every row split into <= 4 groups whose last group holds rows
        rg = (M + 16 * mg - 1) // (16 * mg)
        if rg <= (4 if a.row_groups else 1 if mg < 8 or M <= 128 else 2) and 16 * mg * (rg - 1) < M:
            rgs.append((mg, rg))
    if not a.row_groups:  # the single-group plan of the smallest sufficient mg (round-4 sweeps)
        rgs = rgs[:1] if rgs else [(8, (M + 127) // 128)]
    out = []
    tiles, KS = N // 16, K // 32
    for (mg_, rg), (tpw, wt, wk), S, D in itertools.product(rgs, WAVE_SHAPES, (1, 2, 4, 7, 8, 14, 16), (2, 4, 8, 16)):
        CT = tpw * wt
        if tiles % CT or (epi == "silu" and CT % 2) or KS % S or (KS // S) % (2 * wk):
            continue
        nch = KS // S // (2 * wk)
        if nch < D or nch % D:
            continue
        grid = tiles // CT * rg * S
        if (S > 1 and grid > 256) or grid < 96:
            continue
        out.append((mg_, rg, tpw, wt, wk, S, D))
    return out


_cached_ws = {}


def with_slabs(kind, fn):
    """Run fn with the stream kernel's slabs in ordinary cached memory (comparison only)."""
    key = str(torch.device("cuda", torch.cuda.current_device()))
    shipped = kernels.stream_workspace(key)
    if key not in _cached_ws:
        _cached_ws[key] = (torch.zeros(kernels.STREAM_WS_FLOATS, dtype=torch.float32, device=key),) + shipped[1:]
    kernels._stream_ws[key] = _cached_ws[key]
    try:
        return fn()
    finally:
        kernels._stream_ws[key] = shipped


torch.manual_seed(0)
for name in a.shapes.split(","):
    N, K, epi, nrm = SHAPES[name]
    ncopies = max(2, -(-a.cold_mb * 1_000_000 // (N * K * 2)))
    ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(ncopies)]
    pack = {"silu": kernels.pack_decode_gate_up, "rope_perm": kernels.pack_decode_qkv_rope}.get(epi,
                                                                                               kernels.pack_decode_weight)
    wps = [pack(w) for w in ws]
    if name != "lm_head":
        del ws
    for M in [int(v) for v in a.M.split(",")]:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        NO = N // 2 if epi == "silu" else N
        y = torch.empty(M, NO, dtype=torch.bfloat16, device="cuda")
        resid = torch.randn(M, N, device="cuda").to(torch.bfloat16) if epi == "resid" else None
        ss = kernels.row_sumsq(x)
        kw = dict(out=y, resid=resid, norm=nrm, ss_in=ss if nrm else None)
        variants = {}
        if name == "lm_head":  # round 3: packed decode kernel up to 32 logit rows, hipBLASLt above
            if M <= 32:
                variants["r3"] = lambda i: kernels.decode_gemm(x, wps[i], "plain", out=y)
            else:
                variants["r3"] = lambda i: torch.nn.functional.linear(x, ws[i], out=y)
        elif M <= 16:  # decode-sized steps: the packed decode kernel
            dep = {"rope_perm": "plain", "silu": "silu", "resid": "resid", "plain": "plain"}[epi]
            variants["r3"] = lambda i: kernels.decode_gemm(x, wps[i], dep, out=y if epi != "rope_perm" else y,
                                                           resid=resid, norm=nrm)
        else:
            model = LlamaModel.__new__(LlamaModel)  # only the per-shape tables are used
            model.device = torch.device("cuda")
            model.STREAM_CFG = {}  # the round-3 choice, whatever the current tables route
            path, cfg = LlamaModel._proj_path(model, name, M)
            f = kernels.prefill_gemm if path == "pf" else kernels.mid_gemm
            variants["r3"] = lambda i, f=f, cfg=cfg: f(x, wps[i], epi, **kw, **cfg)
        variants["stream"] = lambda i: kernels.stream_gemm(x, wps[i], epi, **kw)
        if a.rel_ab:  # the sc1-only group hand-off, for the cost of the shipped release
            variants["stream_rel0"] = lambda i: kernels.stream_gemm(x, wps[i], epi, rel=0, **kw)
        if a.krot:  # default plan, rotated K-chunk order per workgroup
            variants["stream_krot"] = lambda i: kernels.stream_gemm(x, wps[i], epi, rel=2, **kw)
        for sl in a.slabs.split(","):
            if sl == "uncached":
                continue
            variants["stream_" + sl] = (lambda sl: lambda i: with_slabs(sl, lambda: kernels.stream_gemm(
                x, wps[i], epi, rel=1 if sl == "cached_rel" else 0, **kw)))(sl)
        if a.sweep:
            for p in plans_for(M, N, K, epi):
                variants["s" + ".".join(map(str, p))] = lambda i, p=p: kernels.stream_gemm(x, wps[i], epi, plan=p, **kw)
        times = {k: [] for k in variants}
        for _ in range(a.rounds):
            for k, fn in variants.items():
                try:
                    times[k].append(timeit(fn, ncopies))
                except (ValueError, RuntimeError):
                    times[k].append(float("nan"))
        med = {k: statistics.median(v) for k, v in times.items()}
        best = min((v, k) for k, v in med.items() if k.startswith("s") and not k.startswith("stream_") and v == v)
        row = {"M": M, "shape": name, "r3_us": round(med.get("r3", float("nan")), 2),
               "stream_default_us": round(med["stream"], 2),
               "default_plan": list(kernels.stream_gemm_plan(M, N, K, "rope_kv" if name == "qkv" else epi)),
               "best_us": round(best[0], 2), "best": best[1],
               "best_TBps": round(N * K * 2 / best[0] / 1e6, 2)}
        for k in med:
            if k.startswith("stream_"):
                row[k + "_us"] = round(med[k], 2)
        if a.sweep:
            row["top5"] = sorted(((round(v, 2), k) for k, v in med.items() if k.startswith("s") and v == v))[:5]
        print(json.dumps(row), flush=True)
        if out_f:
            out_f.write(json.dumps(row) + "\n")
            out_f.flush()

"""What the agent-scope fences of the in-launch hand-offs cost (common.h handoff_last):
times the engine's split-K / partition-merge launches with the round-2 sc1-only consumer
(mode 0), the acquire by the last arriver (mode 1) and producer release + acquire
(mode 2), interleaved in one process (guide §5.4 rule 24), each with the hand-off buffers in
uncached memory (ops.empty_handoff, shipped from round 4) and in ordinary cached memory.

    python tools/handoff_cost.py [--rounds 15] [--out file.jsonl]
"""
import argparse
import json
import math
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd import ops  # noqa: E402
from pilottai_amd.ops import kernels  # noqa: E402

C = kernels.require_native()
ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=15)
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--out", default="")
a = ap.parse_args()
dev = torch.device("cuda")


def timer(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(a.iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1000.0 / a.iters  # us


def gemm(M, N, K, kind, **kw):
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    wp = ops.pack_decode_weight(w)
    r = torch.randn(M, N, device=dev).to(torch.bfloat16)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    if kind == "decode":
        return lambda: ops.decode_gemm(x, wp, "resid", resid=r, out=out, **kw)
    return lambda: ops.mid_gemm(x, wp, "resid", resid=r, out=out, **kw)


ALLOC = {"uncached": kernels.empty_handoff,
         "cached": lambda n, dt=torch.float32, device=None: torch.zeros(int(n), dtype=dt, device=device)}
WS = {}
for kind, fn in ALLOC.items():  # one split-K workspace set per allocation kind
    WS[kind] = {"decode": (fn(kernels.DECODE_WS_FLOATS, torch.float32, dev), torch.zeros(16384, dtype=torch.int32, device=dev)),
                "mid": (fn(kernels.MID_WS_FLOATS, torch.float32, dev), torch.zeros(16384, dtype=torch.int32, device=dev))}


def use_ws(kind):
    kernels._decode_ws[str(dev)] = WS[kind]["decode"]
    kernels._mid_ws[str(dev)] = WS[kind]["mid"]


def attention(nseq, ctx_len, part, alloc="uncached"):
    H, KV, blk = 32, 8, 16
    nb = (ctx_len + blk - 1) // blk
    total = nseq * nb + 4
    kc = torch.randn(total, KV, 16, blk, 8, device=dev).to(torch.bfloat16)
    vc = torch.randn(total, KV, 128, blk, device=dev).to(torch.bfloat16)
    bt = torch.randperm(total)[:nseq * nb].view(nseq, nb).to(torch.int32).to(dev)
    items, _ = ops.build_attention_items([1] * nseq, [ctx_len] * nseq, H // KV, split=True, part=part,
                                         qcols=128, wide_min_tokens=0)
    it = torch.tensor(items + [(0, 0, 0, 0)], dtype=torch.int32, device=dev)
    n_it = torch.tensor([len(items)], dtype=torch.int32, device=dev)
    part_o = ALLOC[alloc](it.shape[0] * KV * 16 * 128, torch.float32, dev)
    part_ml = ALLOC[alloc](it.shape[0] * KV * 16 * 2, torch.float32, dev)
    cnt = torch.zeros(nseq * KV, dtype=torch.int32, device=dev)
    q = torch.randn(nseq, H, 128, device=dev).to(torch.bfloat16)
    out = torch.empty(nseq, H, 128, device=dev, dtype=torch.bfloat16)
    i32 = lambda v: torch.tensor(v, dtype=torch.int32, device=dev)  # noqa: E731
    qs, ql, cl, ps = i32(list(range(nseq))), i32([1] * nseq), i32([ctx_len] * nseq), i32([part])
    return lambda: ops.paged_attention(out, part_o, part_ml, q, kc, vc, it, n_it, cnt, qs, ql, cl, bt,
                                       1.0 / math.sqrt(128), part_size=ps)


cases = {}
for alloc in ALLOC:
    use_ws(alloc)
    cases.update({
        (alloc, "decode down_resid M16 S2 (engine, 9-16-row steps)"): (gemm(16, 4096, 14336, "decode", nt=2, waves=16, splits=2), alloc),
        (alloc, "mid o_resid M32 fm1 fn2 S4 (engine)"): (gemm(32, 4096, 4096, "mid", fm=1, fn=2, splits=4), alloc),
        (alloc, "mid down_resid M64 fm2 fn2 S4 (engine)"): (gemm(64, 4096, 14336, "mid", fm=2, fn=2, splits=4), alloc),
        (alloc, "mid down_resid M256 fm4 fn2 S2 (engine)"): (gemm(256, 4096, 14336, "mid", fm=4, fn=2, splits=2), alloc),
        (alloc, "attention decode 64 x ctx 1000 part 256"): (attention(64, 1000, 256, alloc), alloc),
        (alloc, "attention decode 8 x ctx 2000 part 512"): (attention(8, 2000, 512, alloc), alloc),
    })
MODES = (0, 1, 2)
res = {k: {m: [] for m in MODES} for k in cases}
for _ in range(a.rounds):
    for k, (fn, alloc) in cases.items():
        use_ws(alloc)
        for mode in MODES:
            C.handoff_set_acquire(mode)
            res[k][mode].append(timer(fn))
C.handoff_set_modes(2, 1)
use_ws("uncached")
f = open(a.out, "a") if a.out else None
for k in cases:
    m0, m1, m2 = (statistics.median(res[k][m]) for m in MODES)
    rec = {"alloc": k[0], "case": k[1], "sc1_only_us": round(m0, 2), "acquire_us": round(m1, 2),
           "release_acquire_us": round(m2, 2),
           "delta_acquire_us": round(m1 - m0, 2), "delta_release_acquire_us": round(m2 - m0, 2)}
    print(json.dumps(rec), flush=True)
    if f:
        f.write(json.dumps(rec) + "\n")

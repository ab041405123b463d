#!/usr/bin/env python3
"""Engine-exact epilogue cost of the QKV and O / down projections, mid vs prefill kernels.

prefill_gemm_bench.py times the fused epilogues without the engine's side outputs (QKV: RoPE
into a q buffer only; residual: no row statistics). The engine's QKV epilogue also writes
K / V into the paged cache (EP_ROPEKV), and its residual epilogues accumulate the next
RMSNorm's row statistics (ss_out, one atomic per row and workgroup) and zero the other
statistics buffer (ss_zero). This tool times, per M and kernel:

  plain   the projection with no epilogue
  engine  the engine's exact call (llama.py _forward_mid: _qkv_rope / _gemm "resid")

with cold weights (rotating copies > the 256 MB Infinity Cache), so engine - plain is the
epilogue's price inside the step.

    python tools/epilogue_bench.py [--M 96,128,192,256,2048] [--out file.jsonl]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd.ops import kernels, reference as ref  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--M", default="96,128,192,256,512,2048")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--cold-mb", type=int, default=1024)
ap.add_argument("--out", default="")
a = ap.parse_args()
out_f = open(a.out, "a") if a.out else None
torch.manual_seed(0)
dev = "cuda"
H, KVH, HD, D = 32, 8, 128, 4096


def timeit(fn, n):
    for i in range(2):
        fn(i % n)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(a.iters):
        fn(i % n)
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1000 / a.iters


def copies(N, K):
    return max(2, -(-a.cold_mb * 1_000_000 // (N * K * 2)))


cos_sin = ref.rope_cos_sin(8192, HD, 500000.0).to(dev)
for M in [int(v) for v in a.M.split(",")]:
    x = (torch.randn(M, D, device=dev)).to(torch.bfloat16)
    ss = kernels.row_sumsq(x)
    # ---- QKV: rope-packed weights, paged KV write (contiguous pages, positions 256 + t)
    nq = copies(6144, D)
    wq = [kernels.pack_decode_qkv_rope((torch.randn(6144, D, device=dev) * 0.02).to(torch.bfloat16))
          for _ in range(nq)]
    nb = (M + 256) // 16 + 8
    kc = torch.zeros(nb, KVH, 16, 16, 8, dtype=torch.bfloat16, device=dev)
    vc = torch.zeros(nb, KVH, 128, 16, dtype=torch.bfloat16, device=dev)
    pos = torch.arange(256, 256 + M, dtype=torch.int32, device=dev)
    slots = pos.clone()
    q = torch.empty(M, H, HD, dtype=torch.bfloat16, device=dev)
    yq = torch.empty(M, 6144, dtype=torch.bfloat16, device=dev)
    # ---- O: residual epilogue with row statistics
    no = copies(4096, D)
    wo = [kernels.pack_decode_weight((torch.randn(4096, D, device=dev) * 0.02).to(torch.bfloat16))
          for _ in range(no)]
    h = torch.randn(M, D, device=dev).to(torch.bfloat16)
    ss_a = torch.zeros(M, dtype=torch.float32, device=dev)
    ss_b = torch.zeros(M, dtype=torch.float32, device=dev)
    yo = torch.empty(M, 4096, dtype=torch.bfloat16, device=dev)
    pf = {"bn": 128, "variant": 1}
    variants = {
        ("qkv", "mid", "plain"): (nq, lambda i: kernels.mid_gemm(x, wq[i], "plain", out=yq)),
        ("qkv", "mid", "engine"): (nq, lambda i: kernels.mid_qkv_rope(x, wq[i], 1e-5, q, kc, vc, pos, slots, cos_sin,
                                                                      H, KVH, ss_in=ss)),
        ("qkv", "pf", "plain"): (nq, lambda i: kernels.prefill_gemm(x, wq[i], "plain", out=yq, **pf)),
        ("qkv", "pf", "engine"): (nq, lambda i: kernels.prefill_qkv_rope(x, wq[i], 1e-5, q, kc, vc, pos, slots,
                                                                         cos_sin, H, KVH, ss_in=ss, **pf)),
        ("o", "mid", "plain"): (no, lambda i: kernels.mid_gemm(x, wo[i], "plain", out=yo)),
        ("o", "mid", "engine"): (no, lambda i: kernels.mid_gemm(x, wo[i], "resid", resid=h, out=h, ss_out=ss_b,
                                                                ss_zero=ss_a)),
        ("o", "pf", "plain"): (no, lambda i: kernels.prefill_gemm(x, wo[i], "plain", out=yo, **pf)),
        ("o", "pf", "engine"): (no, lambda i: kernels.prefill_gemm(x, wo[i], "resid", resid=h, out=h, ss_out=ss_b,
                                                                   ss_zero=ss_a, **pf)),
    }
    times = {k: [] for k in variants}
    for _ in range(a.rounds):
        for k, (n, fn) in variants.items():
            try:
                times[k].append(timeit(fn, n))
            except (ValueError, RuntimeError):
                times[k].append(float("nan"))
    for proj in ("qkv", "o"):
        row = {"M": M, "proj": proj}
        for kern in ("mid", "pf"):
            p_, e_ = (statistics.median(times[(proj, kern, w)]) for w in ("plain", "engine"))
            row[f"{kern}_plain_us"] = round(p_, 1)
            row[f"{kern}_engine_us"] = round(e_, 1)
            row[f"{kern}_epilogue_us"] = round(e_ - p_, 1)
        print(json.dumps(row), flush=True)
        if out_f:
            out_f.write(json.dumps(row) + "\n")
            out_f.flush()

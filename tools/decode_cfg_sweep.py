"""Decode-path projection configs (csrc/ops/gemm_decode.hip) at decode row counts, cache-cold
(weight copies rotated past the 256 MB Infinity Cache), interleaved rounds in one process
(guide §5.4 rule 24). Each row: M, projection, us per (nt, waves, splits) config and TB/s of
the best.

    python tools/decode_cfg_sweep.py [--M 8,16,24,32] [--proj down,o,qkv,gate_up] [--out f.jsonl]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd.ops import kernels  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--M", default="8,16,24,32")
ap.add_argument("--proj", default="down,o,gate_up")
ap.add_argument("--cfgs", default="1:8:1,1:16:1,2:16:2,1:8:2,2:8:1,1:16:2,2:16:1,4:16:1")
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--out", default="")
a = ap.parse_args()
SH = {"qkv": (6144, 4096, "plain", True), "o": (4096, 4096, "resid", False),
      "gate_up": (28672, 4096, "silu", True), "down": (4096, 14336, "resid", False)}
out_f = open(a.out, "a") if a.out else None
kernels.require_native()
torch.manual_seed(0)
cfgs = [tuple(int(v) for v in c.split(":")) for c in a.cfgs.split(",")]
for name in a.proj.split(","):
    N, K, epi, norm = SH[name]
    gb = N * K * 2 / 1e9
    ncopies = max(2, int(0.6 / gb) + 1)
    pack = kernels.pack_decode_gate_up if epi == "silu" else kernels.pack_decode_weight
    wps = [pack((torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)) for _ in range(ncopies)]
    for M in [int(v) for v in a.M.split(",")]:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        NO = N // 2 if epi == "silu" else N
        resid = torch.randn(M, N, device="cuda").to(torch.bfloat16) if epi == "resid" else None
        out = torch.empty(M, NO, dtype=torch.bfloat16, device="cuda")
        times = {c: [] for c in cfgs}
        ok = {}
        for _ in range(a.rounds):
            for c in cfgs:
                nt, wv, sp = c
                fn = lambda i: kernels.decode_gemm(x, wps[i], epi, norm=norm, resid=resid, out=out, nt=nt, waves=wv,
                                                   splits=sp)
                try:
                    for i in range(2):
                        fn(i % ncopies)
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for i in range(20):
                        fn(i % ncopies)
                    e.record()
                    e.synchronize()
                    times[c].append(s.elapsed_time(e) * 1000 / 20)
                    ok[c] = True
                except (ValueError, RuntimeError):
                    ok[c] = False
        row = {"M": M, "proj": name, "MB": round(gb * 1000, 1)}
        for c in cfgs:
            if ok.get(c) and times[c]:
                row["nt%d_w%d_s%d" % c] = round(statistics.median(times[c]), 2)
        best = min((v, k) for k, v in row.items() if k.startswith("nt"))
        row["best"] = best[1]
        row["TBps_best"] = round(gb * 1e3 / best[0], 2)
        print(json.dumps(row), flush=True)
        if out_f:
            out_f.write(json.dumps(row) + "\n")

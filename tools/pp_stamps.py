"""Cycle anatomy of the ping-pong prefill GEMM (csrc/ops/gemm_pingpong.h, STAMP build =
prefill variant 4): per workgroup, s_memtime at entry, after the prologue, after the k-loop
and after the epilogue, plus s_memrealtime (100 MHz) for the in-kernel clock
(MI355X_MICROARCH.md "DVFS give-back" item 6). Runs >= 2 s of back-to-back launches on
random data first, then one stamped launch per shape.

    python tools/pp_stamps.py [--shapes sq:4096,gate_up:2048] [--out file.jsonl]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd.ops import kernels  # noqa: E402

SHAPES = {"sq": (4096, 4096), "qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096),
          "down": (4096, 14336)}
ap = argparse.ArgumentParser()
ap.add_argument("--shapes", default="sq:4096,sq:2048,gate_up:2048,gate_up:1024,down:2048")
ap.add_argument("--out", default="")
a = ap.parse_args()
C = kernels.require_native()
out_f = open(a.out, "a") if a.out else None
torch.manual_seed(0)
for spec in a.shapes.split(","):
    name, M = spec.split(":")
    M = int(M)
    N, K = SHAPES[name]
    w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    wp = kernels.pack_decode_weight(w)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    ws, _ = kernels.prefill_workspace(x.device)
    C.prefill_set_variant(3)
    try:
        t_end = time.time() + 2.0
        n = 0
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        while time.time() < t_end:
            for _ in range(20):
                kernels.prefill_gemm(x, wp, "plain", out=y, full=-1, splits=1, bn=256)
            n += 20
            torch.cuda.synchronize()
        e.record()
        e.synchronize()
        us = s.elapsed_time(e) * 1000 / n
        C.prefill_set_variant(4)  # the stamp build
        ws[: 8 * 4096 * 9].zero_()
        kernels.prefill_gemm(x, wp, "plain", out=y, full=-1, splits=1, bn=256)
        torch.cuda.synchronize()
    finally:
        C.prefill_set_variant(-1)
    tiles = ((M + 255) // 256) * (N // 256)
    st = ws[: tiles * 16].view(torch.int64).view(tiles, 8).cpu()
    pro = (st[:, 1] - st[:, 0]).tolist()
    loop = (st[:, 2] - st[:, 1]).tolist()
    epi = (st[:, 3] - st[:, 2]).tolist()
    tot = (st[:, 3] - st[:, 0]).tolist()
    real = (st[:, 5] - st[:, 4]).tolist()
    clk = [t / r * 100 / 1000 for t, r in zip(tot, real) if r > 0]  # GHz
    start_spread_us = (st[:, 4].max() - st[:, 4].min()).item() / 100
    end_spread_us = (st[:, 5].max() - st[:, 5].min()).item() / 100
    span_us = (st[:, 5].max() - st[:, 4].min()).item() / 100
    row = {"variant": 3, "shape": name, "M": M, "N": N, "K": K, "tiles": tiles, "us_per_launch": round(us, 1),
           "tflops": round(2 * M * N * K / us / 1e6, 1),
           "prologue_cyc_med": statistics.median(pro), "loop_cyc_med": statistics.median(loop),
           "epilogue_cyc_med": statistics.median(epi), "epilogue_cyc_max": max(epi), "total_cyc_med": statistics.median(tot),
           "clock_ghz_med": round(statistics.median(clk), 3), "loop_cyc_per_ktile": round(statistics.median(loop) / (K // 64), 1),
           "start_spread_us": start_spread_us, "end_spread_us": end_spread_us, "stamped_span_us": span_us}
    print(json.dumps(row), flush=True)
    if out_f:
        out_f.write(json.dumps(row) + "\n")

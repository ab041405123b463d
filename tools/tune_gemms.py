#!/usr/bin/env python3
"""Tune the engine's projection GEMMs with PyTorch TunableOp (hipBLASLt/rocBLAS
solution search) and write the results file the engine loads at start-up.

For every token bucket M of the engine and every Llama projection shape, each
registered hipBLASLt/rocBLAS solution is timed and the fastest is recorded.
Prints default-vs-tuned timings (cache-warm, µs) per shape.

    python tools/tune_gemms.py --model llama-3-8b --out pilottai_amd/tuned/gemm_llama-3-8b_tp1.csv \
        [--ms 256,576,768] [--tp 1]
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def shapes(model: str, tp: int):
    from pilottai_amd.models.llama import get_config

    c = get_config(model)
    d, hd = c.hidden_size, c.head_dim
    return {
        "qkv": ((c.num_heads + 2 * c.num_kv_heads) * hd // tp, d),
        "o": (d, c.num_heads * hd // tp),
        "gate_up": (2 * c.intermediate_size // tp, d),
        "down": (d, c.intermediate_size // tp),
        "lm_head": (c.vocab_size // tp, d),
    }


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / iters


def main():
    from pilottai_amd.engine.engine import DEFAULT_BUCKETS
    from pilottai_amd.ops.kernels import SKINNY_MAX_M

    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--out", required=True)
    ap.add_argument("--ms", default="")
    ap.add_argument("--max-m", type=int, default=2048)
    ap.add_argument("--max-seqs", type=int, default=128, help="lm_head rows are min(bucket, max_seqs)")
    ap.add_argument("--duration-ms", type=int, default=30)
    a = ap.parse_args()
    ms = [int(x) for x in a.ms.split(",")] if a.ms else [b for b in DEFAULT_BUCKETS if b <= a.max_m]
    dev = torch.device("cuda", 0)
    sh = shapes(a.model, a.tp)
    ws = {k: (torch.randn(n, kk, device=dev) * 0.02).to(torch.bfloat16) for k, (n, kk) in sh.items()}
    tun = torch.cuda.tunable
    jobs = []
    for m in ms:
        for k, (n, kk) in sh.items():
            rows = min(m, a.max_seqs) if k == "lm_head" else m
            if rows <= SKINNY_MAX_M.get(k, 0):
                continue  # served by the skinny kernel, not the library
            jobs.append((k, rows, kk))
    jobs = sorted(set(jobs))
    xs = {}
    base = {}
    for k, rows, kk in jobs:
        x = (torch.randn(rows, kk, device=dev)).to(torch.bfloat16)
        xs[(k, rows)] = x
        base[(k, rows)] = bench(lambda: F.linear(x, ws[k]))
    os.makedirs(os.path.dirname(os.path.abspath(a.out)) or ".", exist_ok=True)
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(a.duration_ms)
    tun.set_filename(a.out, insert_device_ordinal=False)
    t0 = time.time()
    for k, rows, kk in jobs:
        F.linear(xs[(k, rows)], ws[k])
    torch.cuda.synchronize()
    tune_s = time.time() - t0
    tun.tuning_enable(False)
    # TunableOp writes the results file at interpreter exit
    tot_b = tot_t = 0.0
    for k, rows, kk in jobs:
        x = xs[(k, rows)]
        t = bench(lambda: F.linear(x, ws[k]))
        tot_b += base[(k, rows)]
        tot_t += t
        print(json.dumps({"shape": k, "M": rows, "default_us": round(base[(k, rows)], 1),
                          "tuned_us": round(t, 1), "speedup": round(base[(k, rows)] / t, 3)}), flush=True)
    print(json.dumps({"jobs": len(jobs), "tune_s": round(tune_s, 1), "default_total_us": round(tot_b),
                      "tuned_total_us": round(tot_t), "out": a.out}), flush=True)


if __name__ == "__main__":
    main()

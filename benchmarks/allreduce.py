#!/usr/bin/env python3
"""TP all-reduce latency: custom P2P kernel (one-shot / two-shot) vs RCCL, per message size.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        benchmarks/allreduce.py                       # one rank per GPU, RCCL + custom over xGMI
    PILOTTAI_DIST_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 \\
        --master-addr 127.0.0.1 benchmarks/allreduce.py --share-gpu
                                                      # 1-GPU rehearsal: custom kernel only (peers are
                                                      # local HBM, so this times the barrier machinery)

Messages are bf16 [tokens, 8192] (Llama-3-70B hidden size, the TP=8 row-parallel
output): 1 token = 16 KiB. Each size is timed over `--iters` back-to-back calls
between two barriers; rank 0 prints one JSON line per (size, method) with the
per-call latency in microseconds and the algorithm bandwidth (bytes / time).
Every method's result is checked against the RCCL / fp32 sum before timing.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", default="1,4,8,16,32,64,128,256,512")
    ap.add_argument("--hidden", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--share-gpu", action="store_true", help="all ranks on GPU 0 (gloo control plane)")
    a = ap.parse_args()

    import torch
    import torch.distributed as dist

    from pilottai_amd.parallel import comm
    from pilottai_amd.parallel.custom_ar import CustomAllReduce

    rank, world, local = comm.init_distributed()
    dev = torch.device("cuda", 0 if a.share_gpu else local)
    torch.cuda.set_device(dev)
    rccl = dist.get_backend() == "nccl"
    ctrl = dist.new_group(list(range(world)), backend="gloo") if rccl else dist.group.WORLD
    car = CustomAllReduce.create(ctrl, rank, world, dev)

    def barrier():
        dist.barrier(group=ctrl)

    def timed(fn, t):
        for _ in range(5):
            fn(t)
        torch.cuda.synchronize()
        barrier()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            fn(t)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.iters
        m = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(m, op=dist.ReduceOp.MAX, group=ctrl)
        return float(m.item())

    methods = {}
    if rccl:
        methods["rccl"] = lambda t: dist.all_reduce(t)
    if car is not None:
        methods["custom_1shot"] = lambda t: car.all_reduce(t, two_shot=False)
        methods["custom_2shot"] = lambda t: car.all_reduce(t, two_shot=True)
        methods["custom_auto"] = lambda t: car.all_reduce(t)
    g = torch.Generator(device=dev).manual_seed(rank)
    for ntok in [int(x) for x in a.tokens.split(",")]:
        n = ntok * a.hidden
        x = torch.randn(n, device=dev, generator=g).bfloat16()
        parts = [torch.empty_like(x).cpu() for _ in range(world)]
        dist.all_gather(parts, x.cpu(), group=ctrl)
        want = torch.stack([p.float() for p in parts]).sum(0).bfloat16().to(dev)
        for name, fn in methods.items():
            if name.startswith("custom") and not car.eligible(x):
                continue
            t = x.clone()
            fn(t)
            torch.cuda.synchronize()
            err = float((t.float() - want.float()).abs().max())
            sec = timed(fn, x.clone())
            if rank == 0:
                print(json.dumps({"tokens": ntok, "bytes": n * 2, "method": name, "ranks": world,
                                  "share_gpu": a.share_gpu, "us": round(sec * 1e6, 2),
                                  "algbw_GBps": round(n * 2 / sec / 1e9, 2), "max_abs_err": err}), flush=True)
    if car is not None:
        ok = car.healthy()
        if rank == 0:
            print(json.dumps({"custom_healthy": ok}), flush=True)
        barrier()
        car.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

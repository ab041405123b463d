#!/usr/bin/env python3
"""Paged-attention microbenchmark (Llama-3-8B heads: H=32, KV=8, head_dim 128).

Cases mirror the agent-serving steps seen in bench.py profiles:
  decode64   64 decode tokens, ctx 512            (pure KV streaming)
  prefill    2 prompts x 320 new tokens, ctx 480  (prefix-cached task text)
  mix        decode64 + prefill in one launch     (a typical bench step)
Each case is timed with the exact item count and with the grid padded to what
the engine's hipGraph bucket reserves (`--pad`), to expose empty-workgroup cost.

    python tools/attn_bench.py [--iters 50]
"""
import argparse
import json
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pilottai_amd import ops  # noqa: E402


def setup(q_lens, ctx_lens, H=32, KV=8, pad_items=0, dev="cuda", part=512, qcols=128, split_keys=0):
    G = H // KV
    blk = 16
    ns = len(q_lens)
    nbs = [(c + blk - 1) // blk for c in ctx_lens]
    total = sum(nbs) + 4
    mb = max(nbs)
    kc = (torch.randn(total, KV, 16, blk, 8, device=dev) * 0.5).to(torch.bfloat16)
    vc = (torch.randn(total, KV, 128, blk, device=dev) * 0.5).to(torch.bfloat16)
    perm = torch.randperm(total).tolist()
    bt = torch.zeros(ns, mb, dtype=torch.int32)
    c = 0
    for s, nb in enumerate(nbs):
        bt[s, :nb] = torch.tensor(perm[c:c + nb], dtype=torch.int32)
        c += nb
    q_start = np.concatenate([[0], np.cumsum(q_lens)[:-1]]).astype(np.int32)
    T = int(sum(q_lens))
    q = (torch.randn(T, H, 128, device=dev) * 0.5).to(torch.bfloat16)
    items, nslots = ops.build_attention_items(q_lens, ctx_lens, G, part=part, qcols=qcols, wide_min_tokens=0,
                                              split_keys=split_keys)
    n_items = len(items)
    items = items + [(0, 0, 0, 0)] * max(1, pad_items - len(items), nslots - len(items))
    it = torch.tensor(items, dtype=torch.int32, device=dev)
    # ticket room for split prefill items only when splitting (as the engine): without it the
    # kernel runs the instantiation with the partition hand-off compiled out
    cnt = torch.zeros((ns + (it.shape[0] if split_keys else 0)) * KV, dtype=torch.int32, device=dev)
    di = lambda a: torch.tensor(a, dtype=torch.int32, device=dev)  # noqa: E731
    n_it = di([n_items])
    part_o = torch.empty(it.shape[0] * KV * 16 * 128, dtype=torch.float32, device=dev)
    part_ml = torch.empty(it.shape[0] * KV * 16 * 2, dtype=torch.float32, device=dev)
    out = torch.zeros(T, H, 128, dtype=torch.bfloat16, device=dev)
    args = (out, part_o, part_ml, q, kc, vc, it, n_it, cnt, di(q_start), di(q_lens), di(ctx_lens),
            bt.to(dev), 1.0 / math.sqrt(128), None, di([part]))
    kv_bytes = sum(ctx_lens) * KV * 128 * 2 * 2
    flops = sum(4 * ql * (c - ql + (ql + 1) / 2) * H * 128 for ql, c in zip(q_lens, ctx_lens))
    return args, kv_bytes, flops, n_items


def timeit(args, iters, waves=4):
    for _ in range(3):
        ops.paged_attention(*args, waves=waves)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        ops.paged_attention(*args, waves=waves)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--pad", type=int, default=2228, help="items reserved by the 768-token bucket")
    ap.add_argument("--scan", action="store_true", help="prefill length scan instead of the step cases")
    ap.add_argument("--small", action="store_true", help="small-batch decode (8/16 rows) over partition sizes")
    ap.add_argument("--cases", default="", help="comma-separated subset of the step cases")
    ap.add_argument("--qcols", default="32,128", help="prefill item widths to time")
    ap.add_argument("--waves", default="4", help="waves per workgroup to time (4, 8), comma-separated")
    ap.add_argument("--split-keys", default="0", help="prefill item split thresholds to time (0 = off), comma-separated")
    a = ap.parse_args()
    torch.manual_seed(0)
    cases = {
        "decode64": ([1] * 64, [512] * 64),
        "decode64_long": ([1] * 64, [2048] * 64),
        "prefill": ([320, 320], [480, 480]),
        "prefill_cold": ([480], [480]),
        "mix": ([1] * 64 + [320, 320], [512] * 64 + [480, 480]),
        "prefill8x256": ([256] * 8, [768] * 8),
        "prefill2048": ([2048], [2048]),
        # the bench's dominant step: 4 prompts x 512 new tokens on a 256-token cached prefix
        "prefill4x512": ([512] * 4, [768] * 4),
        # ... as it really runs: beside ~40 decode / forced-run rows
        "step2048": ([512] * 4 + [1] * 40, [768] * 4 + [600] * 40),
        # follow-up turns on long cached contexts: few items, each a long serial key chain
        "cont256x4096": ([256], [4352]),
        "cont2x256x2048": ([256] * 2, [2304] * 2),
        "cont512x3072": ([512], [3584]),
    }
    if a.scan:
        cases = {f"pf{n}": ([n], [n]) for n in (8, 32, 128, 256, 512, 1024, 2048, 4096)}
        cases.update({f"pf8x{n}": ([n] * 8, [n] * 8) for n in (128, 512)})
    if a.small:
        for ns in (8, 16):
            for ctx in (600, 1000):
                for part in (128, 256, 512, 4096):
                    for w in [int(x) for x in a.waves.split(",")]:
                        args, kvb, fl, n = setup([1] * ns, [ctx] * ns, part=part, pad_items=141)
                        us = timeit(args, a.iters, waves=w)
                        print(json.dumps({"case": f"decode{ns}_ctx{ctx}", "part": part, "waves": w, "items": n,
                                          "us": round(us, 1), "kv_TBps": round(kvb / us / 1e6, 2)}), flush=True)
        return
    if a.cases:
        cases = {k: v for k, v in cases.items() if k in a.cases.split(",")}
    for name, (ql, cl) in cases.items():
        for qcols in [int(x) for x in a.qcols.split(",")]:
            for sk in [int(x) for x in a.split_keys.split(",")]:
                for pad in ((0,) if a.scan else (0, a.pad)):
                    args, kvb, fl, n = setup(ql, cl, pad_items=pad, qcols=qcols, split_keys=sk)
                    us = timeit(args, a.iters)
                    print(json.dumps({"case": name, "qcols": qcols, "split_keys": sk, "items": n,
                                      "grid_items": args[6].shape[0], "us": round(us, 1),
                                      "kv_TBps": round(kvb / us / 1e6, 2), "TFLOPs": round(fl / us / 1e6, 1)}),
                          flush=True)


if __name__ == "__main__":
    main()

"""Kernel anatomy of the engine's R-row decode steps (Llama-3-8B, 1 GPU), bounded by marker
kernels so that `tools/prof_summary.py --between-markers` keeps only the timed steps.

R prompts of --ctx random tokens (prefix caching off) are prefilled first; once every row is
decoding, marker 0, --steps engine steps of exactly R tokens (bucket R), marker 1. Prints the
mean step time from the engine's own bucket clock.

    rocprofv3 --kernel-trace --stats -d out -- python3 tools/rows_anatomy.py --rows 64 --ctx 600
    python tools/prof_summary.py --between-markers out
"""
import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=64)
    ap.add_argument("--ctx", type=int, default=600)
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch

    from pilottai_amd.engine.engine import EngineConfig, LLMEngine
    from pilottai_amd.ops import kernels

    eng = LLMEngine(EngineConfig(model="llama-3-8b", max_num_seqs=max(64, a.rows), max_num_batched_tokens=2048,
                                 kv_cache_gb=16, prefix_caching=False, capture_on_start=True))
    rng = random.Random(0)
    done = []
    for _ in range(a.rows):
        eng.submit([rng.randrange(1000, 100000) for _ in range(a.ctx)], done.append, temperature=0.0,
                   max_tokens=a.steps + 64, ignore_eos=True)
    R = a.rows
    b = min(x for x in eng.buckets if x >= R)
    guard = 0
    while eng.bucket_hist.get(b, [0])[0] < 2:  # every row is decoding: steps of exactly R tokens
        eng.step()
        guard += 1
        assert guard < 10000, "rows never reached the decode phase"
    torch.cuda.synchronize()
    h0 = list(eng.bucket_hist[b])
    C = kernels.require_native()
    C.timeline_marker(0)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.step()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    C.timeline_marker(1)
    torch.cuda.synchronize()
    h1 = eng.bucket_hist[b]
    n = h1[0] - h0[0]
    rec = {"rows": R, "bucket": b, "ctx": a.ctx, "steps": n, "step_ms": round(1000 * (h1[1] - h0[1]) / max(n, 1), 3),
           "wall_ms_per_step": round(1000 * wall / a.steps, 3)}
    print(json.dumps(rec), flush=True)
    if a.out:
        with open(a.out, "a") as f:
            f.write(json.dumps(rec) + "\n")
    while eng.sched.has_work():
        eng.step()


if __name__ == "__main__":
    main()

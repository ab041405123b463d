"""Kernel anatomy of one engine step shape (run under rocprofv3 --kernel-trace).

Builds the Llama-3-8B engine, then runs R repetitions of a step made of `--seqs` prompts
of `--new` new tokens each on top of a `--cached`-token shared prefix (prefix-cache hit),
i.e. the 2,048-token prefill steps of the 64-worker bench. Each repetition uses fresh
suffixes so nothing but the shared prefix is cached. Markers on stdout give the wall
time per step; the kernel table comes from rocprofv3.

    rocprofv3 --kernel-trace --stats -d out -- python3 tools/step_anatomy.py --seqs 4 --new 512
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seqs", type=int, default=4)
    ap.add_argument("--new", type=int, default=512)
    ap.add_argument("--cached", type=int, default=256)
    ap.add_argument("--reps", type=int, default=6)
    a = ap.parse_args()
    import random

    import torch

    from pilottai_amd.engine.engine import EngineConfig, LLMEngine

    eng = LLMEngine(EngineConfig(model="llama-3-8b", max_num_seqs=64, max_num_batched_tokens=2048, kv_cache_gb=32))
    rng = random.Random(0)
    prefix = [rng.randrange(1000, 100000) for _ in range(a.cached)]
    eng.generate([prefix], temperature=0.0, max_tokens=1, ignore_eos=True)  # cache the prefix
    from pilottai_amd.ops import kernels

    C = kernels.require_native()
    times = []
    for r in range(a.reps):
        prompts = [prefix + [rng.randrange(1000, 100000) for _ in range(a.new)] for _ in range(a.seqs)]
        torch.cuda.synchronize()
        if r == 1:  # rep 0 warms up; markers bound the rest (prof_summary.py --between-markers)
            C.timeline_marker(0)
        s0 = eng.stats["steps"]
        t0 = time.perf_counter()
        eng.generate(prompts, temperature=0.0, max_tokens=1, ignore_eos=True)
        torch.cuda.synchronize()
        times.append((time.perf_counter() - t0) * 1e3)
        print(json.dumps({"rep": r, "ms": round(times[-1], 2), "steps": eng.stats["steps"] - s0}), flush=True)
    C.timeline_marker(1)
    torch.cuda.synchronize()
    print(json.dumps({"seqs": a.seqs, "new": a.new, "cached": a.cached, "ms_median": sorted(times)[len(times) // 2],
                      "buckets": {str(k): v for k, v in eng.bucket_hist.items()}}), flush=True)


if __name__ == "__main__":
    main()

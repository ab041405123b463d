"""Engine micro-benchmark: decode step time, prefill throughput, grammar calls.

    python tools/engine_bench.py --model llama-3-8b --batch 64 --ctx 512 --gen 128

Prints one JSON line per phase. Used to profile the per-token path
(rocprofv3 --kernel-trace --stats -- python tools/engine_bench.py ...).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pilottai_amd.engine.engine import EngineConfig, LLMEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--ctx", type=int, default=512)
    ap.add_argument("--gen", type=int, default=128)
    ap.add_argument("--kv-gb", type=float, default=32.0)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--max-batched", type=int, default=2048)
    ap.add_argument("--phases", default="decode,prefill,grammar")
    ap.add_argument("--buckets", default=None, help="comma-separated token buckets to capture")
    a = ap.parse_args()
    t0 = time.time()
    eng = LLMEngine(EngineConfig(model=a.model, max_num_seqs=max(64, a.batch), kv_cache_gb=a.kv_gb,
                                 max_num_batched_tokens=a.max_batched, use_graphs=not a.no_graphs,
                                 token_buckets=[int(x) for x in a.buckets.split(",")] if a.buckets else None))
    print(json.dumps({"phase": "init", "seconds": round(time.time() - t0, 2),
                      "graphs": len(eng._graphs), "weights_gb": round(eng.model.weight_bytes() / 2**30, 2),
                      "kv_blocks": eng.num_kv_blocks}), flush=True)
    tok = eng.tok
    phases = a.phases.split(",")
    if "decode" in phases:
        prompts = [[(i * 7919 + j * 31) % 120000 for j in range(a.ctx)] for i in range(a.batch)]
        eng.generate(prompts[:2], temperature=0.7, max_tokens=4, ignore_eos=True)  # warm
        st0 = dict(eng.stats)
        t = time.perf_counter()
        outs = eng.generate(prompts, temperature=0.7, max_tokens=a.gen, ignore_eos=True)
        dt = time.perf_counter() - t
        steps = eng.stats["steps"] - st0["steps"]
        gen = sum(len(o.token_ids) for o in outs)
        print(json.dumps({"phase": "decode", "batch": a.batch, "ctx": a.ctx, "gen": a.gen,
                          "seconds": round(dt, 3), "steps": steps, "ms_per_step": round(1e3 * dt / max(1, steps), 3),
                          "gen_tok_s": round(gen / dt, 1),
                          "prompt_tok_s": round(a.batch * a.ctx / dt, 1)}), flush=True)
    if "prefill" in phases:
        prompts = [[(i * 104729 + j * 17) % 120000 for j in range(1024)] for i in range(32)]
        t = time.perf_counter()
        eng.generate(prompts, temperature=0.7, max_tokens=1, ignore_eos=True)
        dt = time.perf_counter() - t
        print(json.dumps({"phase": "prefill", "tokens": 32 * 1024, "seconds": round(dt, 3),
                          "tok_s": round(32 * 1024 / dt, 1)}), flush=True)
    if "grammar" in phases:
        segs = eng.grammar.compile("agent.task_analysis")
        prompts = [tok.encode(f"You act as worker {i}. Analyse the following task: summarize report {i}")
                   for i in range(a.batch)]
        t = time.perf_counter()
        outs = eng.generate(prompts, temperature=0.7, max_tokens=512, grammar=segs)
        dt = time.perf_counter() - t
        ok = 0
        for o in outs:
            try:
                json.loads(o.text)
                ok += 1
            except Exception:
                pass
        print(json.dumps({"phase": "grammar", "calls": a.batch, "seconds": round(dt, 3),
                          "parsed": ok, "sampled": sum(o.sampled_tokens for o in outs),
                          "forced": sum(o.forced_tokens for o in outs)}), flush=True)
    print(json.dumps({"phase": "metrics", **{k: (round(v, 3) if isinstance(v, float) else v)
                                             for k, v in eng.metrics().items()}}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""In-engine A/B of per-step kernel choices (LlamaModel tunables, e.g. PF_MIDRANGE).

One Llama-3-8B engine per configuration (random-init weights, 16 GB each, all resident on one
MI355X); every repetition sends the same fresh T-token prompt (max_tokens = 1: one prefill
step of exactly T tokens through the step's hipGraph) to each engine in turn, so the
configurations alternate and see the same box state. Reported: median step wall time (the
engine's own per-bucket clock, bucket_hist) per configuration and T.

    python tools/midrange_ab.py [--T 96,128,160,192,256] [--reps 12] [--configs none;gate_up;all]
    python tools/midrange_ab.py --T 32,48,64 --overrides '[{}, {"DEC_QKV_MAX_T": 64}]'
"""
import argparse
import json
import os
import random
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", default="96,128,160,192,256")
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--configs", default="none;gate_up;qkv,o,gate_up,down")
    ap.add_argument("--overrides", default="",
                    help="JSON list of LlamaModel tunable overrides, one engine each (replaces --configs)")
    ap.add_argument("--decode", default="",
                    help="decode mode: 'R,CTX,N' = R concurrent prompts of CTX tokens, N generated tokens each; "
                         "the timed steps are the R-row decode steps (bucket T = the --T value, e.g. 8 or 16)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from pilottai_amd.engine.engine import EngineConfig, LLMEngine

    Ts = [int(t) for t in a.T.split(",")]
    seqs = max(64, int(a.decode.split(",")[0])) if a.decode else 64
    engines = {}
    if a.overrides:
        ovs = json.load(open(a.overrides)) if a.overrides.endswith(".json") else json.loads(a.overrides)
        cfgs = [f"cfg{i}" for i in range(len(ovs))]
        for c, o in zip(cfgs, ovs):
            # UPPER-case keys: LlamaModel tunables; lower-case: EngineConfig fields
            eng_kw = {k: v for k, v in o.items() if not k.isupper()}
            mod = {k: v for k, v in o.items() if k.isupper()}
            engines[c] = LLMEngine(EngineConfig(model="llama-3-8b", max_num_seqs=seqs, max_num_batched_tokens=2048,
                                                kv_cache_gb=8, prefix_caching=False, token_buckets=sorted(set(Ts)),
                                                model_overrides=mod, capture_on_start=True, **eng_kw))
    else:
        cfgs = [c for c in a.configs.split(";")]
        for c in cfgs:
            kinds = [k for k in c.split(",") if k and k != "none"]
            engines[c] = LLMEngine(EngineConfig(model="llama-3-8b", max_num_seqs=seqs, max_num_batched_tokens=2048,
                                                kv_cache_gb=8, prefix_caching=False, token_buckets=sorted(set(Ts)),
                                                pf_midrange=kinds, capture_on_start=True))
    rng = random.Random(0)
    res = {c: {T: [] for T in Ts} for c in cfgs}
    if a.decode:
        R, CTX, N = (int(v) for v in a.decode.split(","))
        for r in range(a.reps + 1):
            prompts = [[rng.randrange(1000, 100000) for _ in range(CTX)] for _ in range(R)]
            order = cfgs if r % 2 == 0 else cfgs[::-1]
            for c in order:
                e = engines[c]
                h0 = {T: list(e.bucket_hist.get(T, [0, 0.0])) for T in Ts}
                e.generate(prompts, temperature=0.7, max_tokens=N, ignore_eos=True)
                for T in Ts:
                    h1 = e.bucket_hist.get(T, [0, 0.0])
                    if r > 0 and h1[0] > h0[T][0]:
                        res[c][T].append(1000 * (h1[1] - h0[T][1]) / (h1[0] - h0[T][0]))
    for r in range(0 if a.decode else a.reps + 1):
        for T in Ts:
            prompt = [rng.randrange(1000, 100000) for _ in range(T - 1)]
            order = cfgs if r % 2 == 0 else cfgs[::-1]
            for c in order:
                e = engines[c]
                h0 = list(e.bucket_hist.get(T, [0, 0.0]))
                e.generate([prompt], temperature=0.0, max_tokens=1, ignore_eos=True)
                h1 = e.bucket_hist[T]
                if r > 0 and h1[0] - h0[0] == 1:  # rep 0 warms up
                    res[c][T].append(1000 * (h1[1] - h0[1]))
    out = open(a.out, "a") if a.out else None
    for T in Ts:
        row = {"T": T}
        for c in cfgs:
            v = res[c][T]
            row[c] = round(statistics.median(v), 3) if v else None
        print(json.dumps(row), flush=True)
        if out:
            out.write(json.dumps(row) + "\n")
    for e in engines.values():
        e.stop()


if __name__ == "__main__":
    main()

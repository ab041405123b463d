"""Decode-step anatomy (8 / 16 rows, Llama-3-8B): where an engine decode step's time goes
against the weight-stream floor.

  1. engine decode steps: 8 prompts of --ctx random tokens, --gen tokens each (greedy,
     ignore_eos); the mean 8-row step time from the engine's bucket histogram. Run under
     `rocprofv3 --kernel-trace --stats` for the per-kernel durations inside the graphs.
  2. the same packed projections, launched eagerly in layer order over ALL 32 layers'
     weights (the engine's 15 GB stream: nothing is re-read from the Infinity Cache), and
  3. rotating two layers only (what a microbenchmark with few weight copies measures).

    python tools/decode_anatomy.py [--ctx 1000] [--gen 96] [--out file.jsonl]
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
    ap.add_argument("--ctx", type=int, default=1000)
    ap.add_argument("--gen", type=int, default=96)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="")
    ap.add_argument("--part", choices=["all", "engine", "proj"], default="all")
    a = ap.parse_args()
    from pilottai_amd.engine.engine import EngineConfig, LLMEngine

    eng = LLMEngine(EngineConfig(model="llama-3-8b", max_num_seqs=64, max_num_batched_tokens=2048,
                                 kv_cache_fraction=0.85))
    rng = random.Random(0)
    out = []
    if a.part != "proj":
        out.append(engine_part(a, eng, rng))
    if a.part != "engine":
        out.extend(proj_part(a, eng))
    if a.out:
        with open(a.out, "a") as f:
            for r in out:
                f.write(json.dumps(r) + "\n")


def engine_part(a, eng, rng):
    prompts = [[rng.randrange(1000, 100000) for _ in range(a.ctx)] for _ in range(8)]
    eng.generate(prompts, temperature=0.0, max_tokens=4, ignore_eos=True)  # warm the graphs
    h0 = {b: list(v) for b, v in eng.bucket_hist.items()}
    t0 = time.perf_counter()
    prompts = [[rng.randrange(1000, 100000) for _ in range(a.ctx)] for _ in range(8)]
    eng.generate(prompts, temperature=0.0, max_tokens=a.gen, ignore_eos=True)
    wall = time.perf_counter() - t0
    steps = {b: (v[0] - h0.get(b, [0, 0.0])[0], v[1] - h0.get(b, [0, 0.0])[1]) for b, v in eng.bucket_hist.items()}
    rec = {"what": "engine", "wall_s": round(wall, 3),
           "step_ms": {str(b): [n, round(1000 * t / n, 3)] for b, (n, t) in sorted(steps.items()) if n}}
    print(json.dumps(rec), flush=True)
    return rec


def proj_part(a, eng):
    import torch

    from pilottai_amd import ops

    out = []
    m = eng.model
    layers = m.layers
    eps = m.cfg.rms_eps

    def timed(fn, n_calls):
        """Device time per call: the calls are captured in one hipGraph (eager launches
        from Python would leave the GPU idle between 10-us kernels)."""
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        g.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            g.replay()
        e.record()
        e.synchronize()
        del g
        return s.elapsed_time(e) * 1000.0 / (a.reps * n_calls)

    torch.cuda.set_device(m.device)
    for M in (8, 16):
        h = torch.randn(M, 4096, device=m.device).to(torch.bfloat16)
        a2 = torch.randn(M, 4096, device=m.device).to(torch.bfloat16)
        act = torch.randn(M, m.f_local, device=m.device).to(torch.bfloat16)
        qkv_out = torch.empty(M, layers[0]["wqkv_p"].shape[0] * 16, device=m.device, dtype=torch.bfloat16)
        projs = {
            "qkv(plain,norm)": lambda L: ops.decode_gemm(h, L["wqkv_p"], "plain", norm=True, eps=eps, out=qkv_out),
            "o(resid)": lambda L: ops.decode_gemm(a2, L["wo_p"], "resid", resid=h, out=h),
            "gate_up(silu,norm)": lambda L: ops.decode_gemm(h, L["w13_p"], "silu", norm=True, eps=eps, out=act),
            "down(resid)": lambda L: ops.decode_gemm(act, L["w2_p"], "resid", resid=h, out=h, **m._down_cfg(M)),
        }
        for name, f in projs.items():
            gb = {"qkv(plain,norm)": "wqkv_p", "o(resid)": "wo_p", "gate_up(silu,norm)": "w13_p",
                  "down(resid)": "w2_p"}[name]
            nbytes = layers[0][gb].numel() * 2
            all_l = timed(lambda: [f(L) for L in layers], len(layers))
            two_l = timed(lambda: [f(layers[i & 1]) for i in range(len(layers))], len(layers))
            rec = {"what": "projection", "M": M, "proj": name, "MB": round(nbytes / 1e6, 1),
                   "us_all_layers": round(all_l, 2), "TBps_all_layers": round(nbytes / all_l / 1e6, 2),
                   "us_two_layers": round(two_l, 2), "TBps_two_layers": round(nbytes / two_l / 1e6, 2)}
            print(json.dumps(rec), flush=True)
            out.append(rec)
        # the four projections back to back in layer order (the step minus attention)
        chain = timed(lambda: [[f(L) for f in projs.values()] for L in layers], len(layers))
        rec = {"what": "layer_chain", "M": M, "us_per_layer": round(chain, 2),
               "floor_us_at_6TBps": round(sum(layers[0][k].numel() * 2 for k in ("wqkv_p", "wo_p", "w13_p", "w2_p"))
                                          / 6e6, 2)}
        print(json.dumps(rec), flush=True)
        out.append(rec)
    return out


if __name__ == "__main__":
    main()

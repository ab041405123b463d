"""Host cost of launching one engine step's hipGraph, and the device time it buys.

For a few token buckets: wall time of `graph.replay()` on the host (the GPU idles
for it between engine steps: copy of the step metadata -> first graph kernel), the
device time of the replay (events), and the same with the step split into S
graph segments launched back-to-back (the device starts on segment 1 while the host
is still launching the rest).

    python tools/graph_launch_bench.py [--buckets 8,64,256]
"""
import argparse
import json
import time

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--buckets", default="8,64,256")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--model", default="llama-3-8b")
    a = ap.parse_args()
    from pilottai_amd.engine.engine import EngineConfig, LLMEngine as Engine

    bks = [int(x) for x in a.buckets.split(",")]
    eng = Engine(EngineConfig(model=a.model, capture_on_start=False, max_num_seqs=64))
    eng.capture_graphs(bks)
    for b in bks:
        g = eng._graphs[(b, False, False)]
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        host, dev = [], []
        for i in range(a.iters):
            torch.cuda.synchronize()
            ev0.record()
            t0 = time.perf_counter()
            g.replay()
            t1 = time.perf_counter()
            ev1.record()
            torch.cuda.synchronize()
            if i >= 3:
                host.append(1e6 * (t1 - t0))
                dev.append(1e3 * ev0.elapsed_time(ev1))
        host.sort()
        dev.sort()
        print(json.dumps({"bucket": b, "replay_host_us_p50": round(host[len(host) // 2], 1),
                          "replay_host_us_min": round(host[0], 1),
                          "device_us_p50": round(dev[len(dev) // 2], 1)}), flush=True)


if __name__ == "__main__":
    main()

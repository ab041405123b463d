"""What a kernel boundary costs inside a hipGraph, and whether it grows with the data the
previous kernel WROTE (dirty L2 lines written back by the end-of-kernel release).

A graph holds R launches of a fill kernel (csrc/ops/markers.hip store_test) that writes B bytes
with plain, non-temporal or write-through (sc1) stores; per launch time = graph time / R.
An empty chain (B = 0 via an empty marker) gives the bare boundary.

    python tools/launch_gap.py [--out file.jsonl]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd.ops import kernels  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    C = kernels.require_native()
    out = open(a.out, "a") if a.out else None
    buf = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(a.reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(5):
            s.record()
            g.replay()
            e.record()
            e.synchronize()
            best = min(best, s.elapsed_time(e) * 1000 / a.reps)
        return round(best, 3)

    rows = [{"case": "empty marker kernel", "us": timed(lambda: C.timeline_marker(0))}]
    for nbytes in (4 << 10, 64 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20):
        v = buf[:nbytes]
        for mode, name in ((0, "plain"), (1, "nontemporal"), (2, "write-through sc1")):
            rows.append({"case": f"write {nbytes >> 10} KiB, {name}", "bytes": nbytes, "mode": mode,
                         "us": timed(lambda v=v, m=mode: C.store_test(v, m))})
    for r in rows:
        print(json.dumps(r), flush=True)
        if out:
            out.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()

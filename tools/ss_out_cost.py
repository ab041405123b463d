"""Cost of the residual epilogue's row statistics (ss_out: the next RMSNorm's sum(h^2) per row,
accumulated with float atomics) on the mid-step projections the engine routes to the stream
kernel, graph-replayed with cold weights: the engine's call (with ss_out / ss_zero) vs the
same call without them.

    python tools/ss_out_cost.py [--out file.jsonl]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd.models.llama import LlamaModel  # noqa: E402
from pilottai_amd.ops import kernels  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    out = open(a.out, "a") if a.out else None
    for name, N, K in (("o", 4096, 4096), ("down", 4096, 14336)):
        nc = max(2, -(-1024 * 1_000_000 // (N * K * 2)))
        wps = [kernels.pack_decode_weight((torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16))
               for _ in range(nc)]
        for M in (32, 64, 128, 192, 256):
            m = LlamaModel.__new__(LlamaModel)
            m.device = torch.device("cuda")
            path, cfg = LlamaModel._proj_path(m, name, M, N, K)
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            h = torch.randn(M, N, device="cuda").to(torch.bfloat16)
            ss_a = torch.zeros(M, device="cuda")
            ss_b = torch.zeros(M, device="cuda")
            fn = {"pf": kernels.prefill_gemm, "stream": kernels.stream_gemm}.get(path, kernels.mid_gemm)

            def timed(with_ss):
                def call(i):
                    kw = dict(ss_out=ss_a, ss_zero=ss_b) if with_ss else {}
                    fn(x, wps[i], "resid", resid=h, out=h, **kw, **cfg)
                for i in range(nc):
                    call(i)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for i in range(nc):
                        call(i)
                g.replay()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                best = 1e9
                for _ in range(3):
                    s.record()
                    for _ in range(5):
                        g.replay()
                    e.record()
                    e.synchronize()
                    best = min(best, s.elapsed_time(e) * 1000 / (5 * nc))
                return round(best, 2)

            rec = {"shape": name, "M": M, "path": path, "cfg": str(cfg), "us_with_ss_out": timed(True),
                   "us_without": timed(False)}
            print(json.dumps(rec), flush=True)
            if out:
                out.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()

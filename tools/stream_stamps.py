"""Phase anatomy of the weight-streaming GEMM (csrc/ops/gemm_stream.hip) from in-kernel
wall-clock stamps (s_memrealtime, 100 MHz; diagnostics build path: Args.stamps).

For each (shape, M, plan): the kernel runs inside a hipGraph over rotating cold weight copies
(as tools/stream_gemm_bench.py), then once more with stamps; per workgroup
  [0] start  [1] first chunk in LDS  [2] main loop done  [3] group barrier passed  [4] end
Reported (us): kernel span, start skew, time to the first chunk, main loop, barrier wait,
epilogue — medians and maxima over workgroups — plus the weight rate of the loop alone.

    python tools/stream_stamps.py [--cases qkv:64:4,1,1,4,1,2,4;o:64:...] [--out file.jsonl]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd.ops import kernels  # noqa: E402

SHAPES = {"qkv": (6144, 4096, "rope_perm", True), "o": (4096, 4096, "resid", False),
          "gate_up": (28672, 4096, "silu", True), "down": (4096, 14336, "resid", False)}
DEFAULT = ("qkv:64:4,1,1,4,1,2,4;qkv:64:4,1,3,2,2,4,4;qkv:64:4,1,1,6,1,4,4;o:64:4,1,1,4,1,4,4;"
           "gate_up:64:4,1,2,4,1,1,4;down:64:4,1,1,4,1,4,4;qkv:128:8,1,1,8,1,4,4;down:128:8,1,1,8,1,8,4")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default=DEFAULT)
    ap.add_argument("--cold-mb", type=int, default=1024)
    ap.add_argument("--out", default="")
    ap.add_argument("--rel", type=int, default=0, help="stream_gemm rel bits (2: rotated K-chunk order)")
    a = ap.parse_args()
    out_f = open(a.out, "a") if a.out else None
    stamps = torch.zeros(8 * 8192, dtype=torch.int64, device="cuda")
    cache = {}
    for case in a.cases.split(";"):
        name, M, plan = case.split(":")
        M = int(M)
        plan = tuple(int(v) for v in plan.split(","))
        N, K, epi, nrm = SHAPES[name]
        if name not in cache:
            nc = max(2, -(-a.cold_mb * 1_000_000 // (N * K * 2)))
            pack = {"silu": kernels.pack_decode_gate_up, "rope_perm": kernels.pack_decode_qkv_rope}.get(
                epi, kernels.pack_decode_weight)
            cache = {name: [pack((torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)) for _ in range(nc)]}
        wps = cache[name]
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        y = torch.empty(M, N // 2 if epi == "silu" else N, dtype=torch.bfloat16, device="cuda")
        resid = torch.randn(M, N, device="cuda").to(torch.bfloat16) if epi == "resid" else None
        ss = kernels.row_sumsq(x)
        kw = dict(out=y, resid=resid, norm=nrm, ss_in=ss if nrm else None, plan=plan)

        def call(i, st=None):
            kernels.stream_gemm(x, wps[i], epi, stamps=st, rel=a.rel, **kw)

        for i in range(len(wps)):
            call(i)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(len(wps) - 1):
                call(i)
            call(len(wps) - 1, stamps)  # the last call of the chain stamps (cold weights, busy chip)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        stamps.zero_()
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        per_call = e0.elapsed_time(e1) * 1000 / len(wps)
        mg, rg, tpw, wt, wk, S, D = plan
        grid = N // 16 // (tpw * wt) * rg * S
        t = stamps[: grid * 8].view(grid, 8).cpu().double() * 10e-3  # 100 MHz ticks -> us
        t0 = t[:, 0].min()
        rel = t - t0

        def med(v):
            return round(float(statistics.median(v.tolist())), 2)

        first = rel[:, 1] - rel[:, 0]
        loop = rel[:, 2] - rel[:, 1]
        bar = rel[:, 3] - rel[:, 2]
        epi_t = rel[:, 4] - rel[:, 3]
        rec = {"shape": name, "M": M, "plan": list(plan), "grid": grid, "us_per_call_graph": round(per_call, 2),
               "span_us": round(float(rel[:, 4].max()), 2), "start_skew_us": round(float(rel[:, 0].max()), 2),
               "first_chunk_us": [med(first), round(float(first.max()), 2)],
               "loop_us": [med(loop), round(float(loop.max()), 2)],
               "barrier_wait_us": [med(bar), round(float(bar.max()), 2)],
               "epilogue_us": [med(epi_t), round(float(epi_t.max()), 2)],
               "loop_end_spread_us": round(float(rel[:, 2].max() - rel[:, 2].min()), 2),
               "rel": a.rel,
               # per XCD (workgroup id % 8, the dispatcher's round robin): median loop time and
               # median loop end, to tell a slow XCD from slow CUs spread over all of them
               "loop_by_xcd_us": [med(loop[x::8]) for x in range(8)],
               "loop_end_by_xcd_us": [med(rel[x::8, 2]) for x in range(8)],
               "weights_TBps_in_loop": round(N * K * 2 / 1e6 / max(1e-3, float(rel[:, 2].max() - rel[:, 1].min())), 2)}
        print(json.dumps(rec), flush=True)
        if out_f:
            out_f.write(json.dumps(rec) + "\n")
            out_f.flush()


if __name__ == "__main__":
    main()

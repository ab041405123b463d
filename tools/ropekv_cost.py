"""Cost of the QKV projection's RoPE + paged-KV-write epilogue (EP_ROPEKV, packed_epi.h) against
the same projection with the rope_perm epilogue (no cache write) and without any epilogue
work beyond the store, on the engine's plans (LlamaModel.PF_CFG), cold weights, graph-replayed.

    python tools/ropekv_cost.py [--M 512,1024,2048] [--out file.jsonl]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd import ops  # noqa: E402
from pilottai_amd.models.llama import LlamaModel  # noqa: E402
from pilottai_amd.ops import kernels, reference as ref  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="512,1024,2048")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = torch.device("cuda")
    H, KV, K = 32, 8, 4096
    N = (H + 2 * KV) * 128
    ncopies = 6  # 6 x 50 MB > the 256 MB Infinity Cache
    ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(ncopies)]
    wps = [ops.pack_decode_qkv_rope(w) for w in ws]
    cos_sin = ref.rope_cos_sin(8192).to(dev)
    out = []
    for M in [int(v) for v in a.M.split(",")]:
        cfg = next(c for mmax, path, c in LlamaModel.PF_CFG["qkv"] if M <= mmax)
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        ss = kernels.row_sumsq(x)
        NB = (M + 15) // 16 + 8
        kc = torch.zeros(NB, KV, 16, 16, 8, dtype=torch.bfloat16, device=dev)
        vc = torch.zeros(NB, KV, 128, 16, dtype=torch.bfloat16, device=dev)
        q = torch.empty(M, H, 128, dtype=torch.bfloat16, device=dev)
        y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        pos = torch.arange(500, 500 + M, dtype=torch.int32, device=dev)
        slots = torch.arange(32, 32 + M, dtype=torch.int32, device=dev)  # one sequence's consecutive slots

        def ropekv(i):
            ops.prefill_qkv_rope(x, wps[i], 1e-5, q, kc, vc, pos, slots, cos_sin, H, KV, ss_in=ss, **cfg)

        def ropeperm(i):
            ops.prefill_gemm(x, wps[i], "rope_perm", out=y, norm=True, ss_in=ss, **cfg)

        def plain(i):
            ops.prefill_gemm(x, wps[i], "plain", out=y, norm=True, ss_in=ss, **cfg)

        rec = {"M": M, "cfg": cfg}
        for name, fn in (("ropekv", ropekv), ("rope_perm", ropeperm), ("plain", plain)) * 2:
            fn(0)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for r in range(a.reps):
                    fn(r % ncopies)
            g.replay()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            g.replay()
            e.record()
            e.synchronize()
            rec[name] = round(s.elapsed_time(e) * 1000 / a.reps, 1)  # second pass overwrites the first
            del g
        print(json.dumps(rec), flush=True)
        out.append(rec)
    if a.out:
        with open(a.out, "a") as f:
            for r in out:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()

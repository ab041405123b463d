"""Phase anatomy of the fused attention + O launch (csrc/ops/attention.hip attn_o_kernel) on
an 8-row decode step (ctx 600), from per-workgroup s_memrealtime stamps, next to the two
launches it replaces (graph-replayed, us per call).

    python tools/attn_o_stamps.py [--rows 8] [--ctx 600] [--out file.jsonl]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402

from pilottai_amd import ops  # noqa: E402
from pilottai_amd.ops import kernels  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8)
    ap.add_argument("--ctx", type=int, default=600)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from test_attn_o_gpu import _case

    gpu = torch.device("cuda")
    c = _case(gpu, 32, 8, [1] * a.rows, [a.ctx] * a.rows, 4096, seed=1)
    m, (po, pm) = c["meta"], c["ws"]
    att = torch.zeros(c["T"], 32, 128, dtype=torch.bfloat16, device=gpu)
    h = c["h"].clone()
    args = (att, po, pm, c["q"], c["kc"], c["vc"], m["items"], m["n_items"], m["counters"], m["q_start"],
            m["q_len"], m["ctx_len"], m["block_table"], m["scale"])

    def fused():
        ops.attn_o(*args, c["wp"], h, part_size=m["part_size"])

    def two():
        ops.paged_attention(*args, part_size=m["part_size"], waves=8)
        ops.decode_gemm(att.view(c["T"], -1), c["wp"], "resid", resid=h, out=h)

    def timed(fn, reps=50):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        e.synchronize()
        return round(s.elapsed_time(e) * 1000 / reps, 2)

    rec = {"rows": a.rows, "ctx": a.ctx, "two_launches_us": timed(two), "fused_us": timed(fused)}
    st = torch.zeros(8 * 256, dtype=torch.int64, device=gpu)
    C = kernels.require_native()
    C.attn_o_set_stamps(st)
    fused()
    torch.cuda.synchronize()
    C.attn_o_set_stamps(None)
    t = st.view(256, 8).cpu().double() * 10e-3
    t0 = t[:, 0].min()
    rel = t - t0
    units = a.rows * 8
    phases = {"start": 0, "att_or_issue_done": 1, "w_issued": 2, "wait_passed": 3, "w_landed": 4, "end": 5}
    for grp, sl in (("attention_wgs", slice(0, units)), ("o_only_wgs", slice(units, 256))):
        rec[grp] = {k: round(statistics.median(rel[sl, i].tolist()), 2) for k, i in phases.items()}
        rec[grp + "_max"] = {k: round(float(rel[sl, i].max()), 2) for k, i in phases.items()}
    print(json.dumps(rec), flush=True)
    if a.out:
        with open(a.out, "a") as f:
            f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()

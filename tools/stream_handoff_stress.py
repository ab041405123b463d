"""Poisoned, varied-input stress of the weight-streaming GEMM's split-K group hand-off
(csrc/ops/gemm_stream.hip) on EVERY plan the engine routes to it (LlamaModel.STREAM_CFG, at
the row counts where each table row applies), including the RoPE + paged-KV epilogue
(>= 100,000 repetitions per case).

Per repetition:
  * fresh random activations (a stale slab from the previous launch holds a WRONG value);
  * the slab workspace and the outputs NaN-poisoned before the launch (a slab read before
    its write lands, or a lost store, shows up as NaN);
  * every other repetition runs beside a 4096^3 GEMM on a side stream (uneven load);
  * the result is compared with the same projection on the mid kernel without a K split
    (no hand-off), with the bf16 tolerance of the numerics tests.
Bad-run counts are accumulated on the device and read back every --sync reps.

    python tools/stream_handoff_stress.py [--reps 100000] [--rel 1] [--only qkv] [--out f.jsonl]

LM_HEAD_STREAM plans have S = 1 (no hand-off) and are not stressed here.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilottai_amd import ops  # noqa: E402
from pilottai_amd.models.llama import LlamaModel  # noqa: E402
from pilottai_amd.ops import kernels, reference as ref  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=100000)
ap.add_argument("--rel", default="1", help="comma-separated rel values (bit 0: producer release)")
ap.add_argument("--only", default="")
ap.add_argument("--sync", type=int, default=2000)
ap.add_argument("--out", default="")
a = ap.parse_args()
dev = torch.device("cuda")
NAN = float("nan")
side = torch.cuda.Stream()
big_a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
big_b = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
out_f = open(a.out, "a") if a.out else None
ws = kernels.stream_workspace(dev)


def emit(rec):
    line = json.dumps(rec)
    print(line, flush=True)
    if out_f:
        out_f.write(line + "\n")
        out_f.flush()


H, KV, D = 32, 8, 4096
NQKV = (H + 2 * KV) * 128
cos_sin = ref.rope_cos_sin(4096).to(dev)
NB = 32


def bad_count(got, base, acc):
    """acc[0] += 1 if any element is off (or NaN where base is not), acc[1] += #NaN."""
    nan = torch.isnan(got) & ~torch.isnan(base)
    bad = ((got - base).abs() > 3e-2 + 2e-2 * base.abs()) | nan
    acc[0] += bad.any().to(torch.int64)
    acc[1] += nan.sum()


def gemm_case(M, N, K, epi, plan, rel):
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    wp = ops.pack_decode_gate_up(w) if epi == "silu" else ops.pack_decode_weight(w)
    no = N // 2 if epi == "silu" else N
    x = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    r = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    base = torch.empty(M, no, device=dev, dtype=torch.bfloat16)
    out = torch.empty(M, no, device=dev, dtype=torch.bfloat16)

    def rep(acc):
        x.normal_()
        r.normal_()
        ops.mid_gemm(x, wp, epi, resid=r if epi == "resid" else None, out=base, norm=(epi == "silu"), splits=1)
        ws[0].fill_(NAN)
        out.fill_(NAN)
        ops.stream_gemm(x, wp, epi, resid=r if epi == "resid" else None, out=out, norm=(epi == "silu"),
                        plan=plan, rel=rel)
        bad_count(out.float(), base.float(), acc)
    return rep


def qkv_rope_case(M, plan, rel):
    w = (torch.randn(NQKV, D, device=dev) * 0.05).to(torch.bfloat16)
    wp = ops.pack_decode_qkv_rope(w)
    x = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    bufs = {}
    for k in ("base", "got"):
        bufs[k] = (torch.empty(M, H, 128, dtype=torch.bfloat16, device=dev),
                   torch.empty(NB, KV, 16, 16, 8, dtype=torch.bfloat16, device=dev),
                   torch.empty(NB, KV, 128, 16, dtype=torch.bfloat16, device=dev))

    def flat(b, used):
        q, kc, vc = b
        return torch.cat([q.flatten().float(),
                          kc.permute(0, 3, 1, 2, 4).reshape(NB * 16, -1)[used].flatten().float(),
                          vc.permute(0, 3, 1, 2).reshape(NB * 16, -1)[used].flatten().float()])

    def rep(acc):
        x.normal_()
        pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=dev)
        slots = torch.randperm(NB * 16, device=dev)[:M].to(torch.int32)
        for k in ("base", "got"):
            for t in bufs[k]:
                t.fill_(NAN)
        q, kc, vc = bufs["base"]
        ops.mid_qkv_rope(x, wp, 1e-5, q, kc, vc, pos, slots, cos_sin, H, KV, splits=1)
        ws[0].fill_(NAN)
        q, kc, vc = bufs["got"]
        ops.stream_qkv_rope(x, wp, 1e-5, q, kc, vc, pos, slots, cos_sin, H, KV, plan=plan, rel=rel)
        used = slots.long()
        bad_count(flat(bufs["got"], used), flat(bufs["base"], used), acc)
    return rep


SHAPES = {"qkv": (NQKV, D, "rope_kv"), "o": (4096, 4096, "resid"), "down": (4096, 14336, "resid"),
          "gate_up": (28672, 4096, "silu")}
cases = []
for kind, rows in LlamaModel.STREAM_CFG.items():
    N, K, epi = SHAPES[kind]
    lo = LlamaModel.DECODE_FUSED_MAX_T + 1
    for mmax, shape in rows:
        for M in sorted({lo, mmax}):
            plan = LlamaModel._stream_plan(M, shape)
            if plan[5] * plan[4] == 1:
                continue  # no K split: no hand-off
            for rel in (int(v) for v in a.rel.split(",")):
                nm = f"stream {kind} {epi} M{M} plan{plan} rel{rel}"
                if epi == "rope_kv":
                    cases.append((nm, lambda M=M, plan=plan, rel=rel: qkv_rope_case(M, plan, rel)))
                else:
                    cases.append((nm, lambda M=M, N=N, K=K, epi=epi, plan=plan, rel=rel:
                                  gemm_case(M, N, K, epi, plan, rel)))
        lo = mmax + 1

for name, mk in cases:
    if a.only and a.only not in name:
        continue
    torch.manual_seed(len(name))
    rep = mk()
    acc = torch.zeros(2, dtype=torch.int64, device=dev)
    ws[2].zero_()
    t0 = time.time()
    done = 0
    while done < a.reps:
        n = min(a.sync, a.reps - done)
        for i in range(n):
            if (done + i) % 2:
                with torch.cuda.stream(side):
                    torch.matmul(big_a, big_b)
            rep(acc)
        torch.cuda.synchronize()
        done += n
    bad, nan = (int(v) for v in acc.cpu())
    emit({"case": name, "reps": done, "bad_runs": bad, "nan_elems": nan, "err_word": int(ws[2][0]),
          "s": round(time.time() - t0, 1)})

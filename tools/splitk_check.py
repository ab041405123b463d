"""Stress every in-launch hand-off the engine uses and count results that differ from
the same kernel run without a hand-off (split-K = 1 / one attention partition).

The check is built so that it CAN fail:
  * fresh random inputs every repetition, so a stale slab from the previous launch
    holds a WRONG value;
  * the split-K workspace (and the attention partials) are filled with NaN before
    every launch, so a slab read before its write lands shows up as NaN;
  * outputs are NaN-poisoned before every launch, so a lost store shows up as NaN;
  * every other repetition runs beside a side-stream GEMM (uneven load).

    python tools/splitk_check.py [--reps 300] [--modes 0,1] [--out file.jsonl]

Modes (common.h handoff_last): "default" = the shipped protocols (GEMM slabs: producer
release + last-arriver acquire; attention merge: acquire), or one protocol for every
hand-off: 2 = release + acquire, 1 = acquire only, 0 = the round-2 sc1-loads-only consumer;
--modes 0,1,2,default runs them all.
"""
import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pilottai_amd import ops  # noqa: E402
from pilottai_amd.ops import kernels, reference as ref  # noqa: E402

C = kernels.require_native()
ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=300)
ap.add_argument("--modes", default="default")
ap.add_argument("--only", default="")
ap.add_argument("--out", default="")
ap.add_argument("--cached", action="store_true",
                help="hand-off workspaces in ordinary (cached) device memory instead of the shipped uncached "
                     "allocation (ops.empty_handoff), to show what the uncached memory buys")
a = ap.parse_args()
if a.cached:  # the round-3 allocation, for the comparison
    kernels.empty_handoff = lambda n, dt=torch.float32, device=None: torch.zeros(int(n), dtype=dt, device=device)
modes = [m if m == "default" else int(m) for m in a.modes.split(",")]
dev = torch.device("cuda")
NAN = float("nan")
side = torch.cuda.Stream()
big_a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
big_b = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
out_f = open(a.out, "a") if a.out else None


def emit(rec):
    line = json.dumps(rec)
    print(line, flush=True)
    if out_f:
        out_f.write(line + "\n")
        out_f.flush()


def poison_ws():
    kernels.decode_workspace(dev)[0].fill_(NAN)
    kernels.mid_workspace(dev)[0].fill_(NAN)
    kernels.prefill_workspace(dev)[0].fill_(NAN)


def load(rep):
    if rep % 2:
        with torch.cuda.stream(side):
            torch.matmul(big_a, big_b)


def compare(got, base):
    nan = torch.isnan(got) & ~torch.isnan(base)
    bad = ((got - base).abs() > 3e-2 + 2e-2 * base.abs()) | nan
    return int(bad.sum()), int(nan.sum())


def run_cfg(name, make, call, reps):
    """make() -> state with fresh inputs; call(state, splits, mode) -> output tensor."""
    for mode in modes:
        if mode == "default":
            C.handoff_set_modes(2, 1)
        else:
            C.handoff_set_acquire(mode)
        bad_runs = bad_elems = nan_elems = 0
        t0 = time.time()
        for rep in range(reps):
            st = make()
            base = call(st, 1).clone()
            poison_ws()
            load(rep)
            got = call(st, None)
            torch.cuda.synchronize()
            nb, nn = compare(got.float(), base.float())
            if nb:
                bad_runs += 1
                bad_elems += nb
                nan_elems += nn
        emit({"case": name, "mode": mode, "reps": reps, "bad_runs": bad_runs, "bad_elems": bad_elems,
              "nan_elems": nan_elems, "s": round(time.time() - t0, 1)})
    C.handoff_set_modes(2, 1)


H, KV, D = 32, 8, 4096
NQKV = (H + 2 * KV) * 128
cos_sin = ref.rope_cos_sin(4096).to(dev)
NB = 8


def qkv_rope_case(M, splits, mid=False, fm=0, fn=0):
    w = (torch.randn(NQKV, D, device=dev) * 0.05).to(torch.bfloat16)
    wp = ops.pack_decode_qkv_rope(w)

    def make():
        x = torch.randn(M, D, device=dev).to(torch.bfloat16)
        pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=dev)
        slots = torch.randperm(NB * 16, device=dev)[:M].to(torch.int32)
        return x, pos, slots

    def call(st, sp):
        x, pos, slots = st
        q = torch.full((M, H, 128), NAN, dtype=torch.bfloat16, device=dev)
        kc = torch.full((NB, KV, 16, 16, 8), NAN, dtype=torch.bfloat16, device=dev)
        vc = torch.full((NB, KV, 128, 16), NAN, dtype=torch.bfloat16, device=dev)
        s = splits if sp is None else sp
        if mid:
            ops.mid_qkv_rope(x, wp, 1e-5, q, kc, vc, pos, slots, cos_sin, H, KV, fm=fm, fn=fn, splits=s)
        else:
            ops.decode_qkv_rope(x, wp, 1e-5, q, kc, vc, pos, slots, cos_sin, H, KV, splits=s)
        used = slots.long()  # only the written cache slots: [NB, KV, 16, off, 8] / [NB, KV, 128, off]
        return torch.cat([q.flatten().float(),
                          kc.permute(0, 3, 1, 2, 4).reshape(NB * 16, -1)[used].flatten().float(),
                          vc.permute(0, 3, 1, 2).reshape(NB * 16, -1)[used].flatten().float()])
    return make, call


def gemm_case(M, N, K, epi, splits, kind, **cfg):
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    wp = ops.pack_decode_gate_up(w) if epi == "silu" else ops.pack_decode_weight(w)

    def make():
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        r = torch.randn(M, N, device=dev).to(torch.bfloat16)
        return x, r

    def call(st, sp):
        x, r = st
        s = splits if sp is None else sp
        no = N // 2 if epi == "silu" else N
        out = torch.full((M, no), NAN, dtype=torch.bfloat16, device=dev)
        kw = dict(cfg)
        if kind == "decode":
            ops.decode_gemm(x, wp, epi, norm=(epi == "silu"), resid=r if epi == "resid" else None, out=out,
                            splits=s, **kw)
        elif kind == "prefill":
            ops.prefill_gemm(x, wp, epi, resid=r if epi == "resid" else None, out=out, norm=(epi == "silu"),
                             splits=s, full=kw.get("full", -1) if s != 1 else -1)
        elif kind == "stream":  # the hand-off-free baseline: the mid kernel without a K split
            if sp == 1:
                ops.mid_gemm(x, wp, epi, resid=r if epi == "resid" else None, out=out, norm=(epi == "silu"),
                             splits=1)
            else:
                kernels.stream_workspace(dev)[0].fill_(NAN)
                ops.stream_gemm(x, wp, epi, resid=r if epi == "resid" else None, out=out, norm=(epi == "silu"),
                                plan=kw["plan"], rel=kw.get("rel"))
        else:
            ops.mid_gemm(x, wp, epi, resid=r if epi == "resid" else None, out=out, norm=(epi == "silu"),
                         splits=s, **kw)
        return out
    return make, call


def attention_case(nseq, ctx_max, part, waves=4, ctx_min=None):
    blk = 16
    torch.manual_seed(1)
    ctx = torch.randint(ctx_min or part + 1, ctx_max, (nseq,)).tolist()
    nbs = [(c + blk - 1) // blk for c in ctx]
    total = sum(nbs) + 4
    kc = torch.randn(total, KV, 16, blk, 8, device=dev).to(torch.bfloat16)
    vc = torch.randn(total, KV, 128, blk, device=dev).to(torch.bfloat16)
    perm = torch.randperm(total).tolist()
    bt = torch.zeros(nseq, max(nbs), dtype=torch.int32)
    c = 0
    for s, nb in enumerate(nbs):
        bt[s, :nb] = torch.tensor(perm[c:c + nb], dtype=torch.int32)
        c += nb
    bt = bt.to(dev)
    q_lens = [1] * nseq
    q_start = torch.arange(nseq, dtype=torch.int32, device=dev)
    dq = torch.tensor(q_lens, dtype=torch.int32, device=dev)
    dc = torch.tensor(ctx, dtype=torch.int32, device=dev)
    plans = {}
    for split in (False, True):
        items, _ = ops.build_attention_items(q_lens, ctx, H // KV, split=split, part=part, qcols=128,
                                             wide_min_tokens=0)
        it = torch.tensor(items + [(0, 0, 0, 0)], dtype=torch.int32, device=dev)
        plans[split] = (it, torch.tensor([len(items)], dtype=torch.int32, device=dev))
    maxit = max(p[0].shape[0] for p in plans.values())
    part_o = kernels.empty_handoff(maxit * KV * 16 * 128, torch.float32, dev)
    part_ml = kernels.empty_handoff(maxit * KV * 16 * 2, torch.float32, dev)
    cnt = torch.zeros(nseq * KV, dtype=torch.int32, device=dev)
    psz = torch.tensor([part], dtype=torch.int32, device=dev)

    def make():
        return torch.randn(nseq, H, 128, device=dev).to(torch.bfloat16)

    def call(q, sp):
        split = sp is None
        it, n_it = plans[split]
        part_o.fill_(NAN)
        part_ml.fill_(NAN)
        out = torch.full((nseq, H, 128), NAN, dtype=torch.bfloat16, device=dev)
        ops.paged_attention(out, part_o, part_ml, q, kc, vc, it, n_it, cnt, q_start, dq, dc, bt,
                            1.0 / math.sqrt(128), part_size=psz, waves=waves)
        return out
    return make, call


cases = []
for M, S in ((9, 3), (9, 2), (16, 2), (7, 3)):
    cases.append((f"decode_qkv_rope M{M} S{S}", lambda M=M, S=S: qkv_rope_case(M, S)))
for M in (9, 16):
    cases.append((f"decode_down_resid M{M} S2 (engine)",
                  lambda M=M: gemm_case(M, 4096, 14336, "resid", 2, "decode", nt=2, waves=16)))
cases.append(("decode_silu M12 S2", lambda: gemm_case(12, 2 * 14336, 4096, "silu", 2, "decode")))
cases.append(("mid_qkv_rope M32 fm1 fn2 S2 (engine)", lambda: qkv_rope_case(32, 2, mid=True, fm=1, fn=2)))
for M, fm, fn, S in ((32, 1, 2, 4), (64, 1, 2, 2), (128, 2, 2, 2)):
    cases.append((f"mid_o_resid M{M} fm{fm} fn{fn} S{S} (engine)",
                  lambda M=M, fm=fm, fn=fn, S=S: gemm_case(M, 4096, 4096, "resid", S, "mid", fm=fm, fn=fn)))
for M, fm, fn, S in ((32, 1, 2, 4), (64, 2, 2, 4), (128, 2, 2, 2), (256, 4, 2, 2)):
    cases.append((f"mid_down_resid M{M} fm{fm} fn{fn} S{S} (engine)",
                  lambda M=M, fm=fm, fn=fn, S=S: gemm_case(M, 4096, 14336, "resid", S, "mid", fm=fm, fn=fn)))
cases.append(("prefill o_resid M2048 S2 (256x256 tiles, every tile split)",
              lambda: gemm_case(2048, 4096, 4096, "resid", 2, "prefill", full=0)))
cases.append(("prefill gate_up_silu M2048 (768 whole + 128 tiles x S2)",
              lambda: gemm_case(2048, 28672, 4096, "silu", 2, "prefill", full=768)))
# weight-streaming kernel (gemm_stream.hip): cooperative split-K over uncached slabs; rel 0 =
# sc1 slab stores + vmcnt(0) + relaxed arrive + acquire (shipped), rel 1 = plus the producer's
# agent-scope release before arriving
for rel in (0, 1):
    for nm, M, N, K, epi, plan in (("qkv_plain M64", 64, 6144, 4096, "plain", (4, 1, 3, 2, 2, 4, 4)),
                                   ("down_resid M64", 64, 4096, 14336, "resid", (4, 1, 2, 4, 1, 8, 4)),
                                   ("o_resid M32 wk2", 32, 4096, 4096, "resid", (2, 1, 1, 4, 2, 4, 4)),
                                   ("gate_up_silu M128", 128, 28672, 4096, "silu", (8, 1, 2, 7, 1, 2, 4))):
        cases.append((f"stream {nm} S{plan[5]} rel{rel}",
                      lambda M=M, N=N, K=K, epi=epi, plan=plan, rel=rel:
                      gemm_case(M, N, K, epi, plan[5], "stream", plan=plan, rel=rel)))
cases.append(("attention decode 48 seqs part256", lambda: attention_case(48, 3000, 256)))
cases.append(("attention decode 8 seqs part512", lambda: attention_case(8, 4000, 512)))
# 256- and 512-key partitions, 4- and 8-wave workgroups, 64 x ~1,000 and
# 8 x ~2,000 keys
for nseq, lo, hi in ((64, 900, 1100), (8, 1900, 2100)):
    for part in (256, 512):
        for wv in (4, 8):
            cases.append((f"attention decode {nseq}x{lo}-{hi} part{part} w{wv}",
                          lambda nseq=nseq, lo=lo, hi=hi, part=part, wv=wv:
                          attention_case(nseq, hi, part, waves=wv, ctx_min=lo)))

for name, mk in cases:
    if a.only and a.only not in name:
        continue
    torch.manual_seed(len(name))
    try:
        make, call = mk()
        run_cfg(name, make, call, a.reps)
    except (ValueError, RuntimeError) as e:
        emit({"case": name, "error": str(e)[:200]})

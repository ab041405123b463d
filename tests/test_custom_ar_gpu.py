"""Custom P2P all-reduce (csrc/ops/custom_ar.hip, parallel/custom_ar.py) on one MI355X.

Two forms, both compared bit-exactly against a plain PyTorch fp32 sum in rank order:
* several "ranks" in one launch on one GPU (blockIdx.y = rank): the kernel's
  barrier/parity/epoch logic for W = 2..8, one-shot and two-shot, repeated calls,
  sizes that do not fill the chunk grid, and hipGraph replay;
* two processes sharing GPU 0 that exchange real IPC handles over a gloo group —
  the same setup path (`CustomAllReduce.create`) the TP engine uses over xGMI.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _C():
    from pilottai_amd.ops.kernels import require_native

    return require_native()


def _ref(ts):
    acc = torch.zeros_like(ts[0], dtype=torch.float32)
    for t in ts:
        acc += t.float()
    return acc.bfloat16()


@pytest.mark.parametrize("W", [2, 4, 8])
@pytest.mark.parametrize("two_shot", [False, True])
def test_custom_ar_local_ranks(W, two_shot):
    from pilottai_amd.parallel.custom_ar import local_group_all_reduce

    C = _C()
    state = {}
    cap = 1 << 20
    g = torch.Generator(device="cuda").manual_seed(W)
    # sizes: one vector, partial chunk, several chunks per workgroup, the full cap
    for n in [8, 4096 * 3 + 8, 8192 * 40, cap // 2]:
        for rep in range(3):  # alternate data parities
            ins = [torch.randn(n, device="cuda", generator=g).bfloat16() for _ in range(W)]
            want = _ref(ins)
            local_group_all_reduce(C, ins, cap, two_shot, state)
            torch.cuda.synchronize()
            for r in range(W):
                assert torch.equal(ins[r], want), (n, rep, r)
    err = state[(W, cap)][2]
    assert int(err.item()) == 0


def test_custom_ar_local_graph_replay():
    from pilottai_amd.parallel.custom_ar import local_group_all_reduce

    C = _C()
    W, n, cap = 4, 8192 * 16, 1 << 20
    state = {}
    bufs = [torch.empty(n, dtype=torch.bfloat16, device="cuda") for _ in range(W)]
    local_group_all_reduce(C, bufs, cap, False, state)  # allocate before capture
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            local_group_all_reduce(C, bufs, cap, False, state)
            local_group_all_reduce(C, bufs, cap, True, state)
    torch.cuda.current_stream().wait_stream(s)
    for it in range(4):
        ins = [torch.randn(n, device="cuda").bfloat16() for _ in range(W)]
        want = _ref(ins)
        want = _ref([want] * W)  # two reductions back to back
        for b, x in zip(bufs, ins):
            b.copy_(x)
        graph.replay()
        torch.cuda.synchronize()
        for r in range(W):
            assert torch.equal(bufs[r], want), (it, r)
    assert int(state[(W, cap)][2].item()) == 0


_WORKER = r"""
import json, os, sys, datetime
import torch, torch.distributed as dist
sys.path.insert(0, os.environ["ROOT"])
rank = int(sys.argv[1])
dist.init_process_group("gloo", rank=rank, world_size=2, timeout=datetime.timedelta(seconds=60))
torch.cuda.set_device(0)
from pilottai_amd.parallel.custom_ar import CustomAllReduce
car = CustomAllReduce.create(dist.group.WORLD, rank, 2, torch.device("cuda", 0), cap_bytes=1 << 20)
out = {"rank": rank, "created": car is not None, "ok": []}
if car is not None:
    g = torch.Generator(device="cuda").manual_seed(1234)
    for n in [8, 8192 + 8, 8192 * 40]:
        for rep in range(3):
            both = [torch.randn(n, device="cuda", generator=g).bfloat16() for _ in range(2)]
            want = (both[0].float() + both[1].float()).bfloat16()
            t = both[rank].clone()
            car.all_reduce(t, two_shot=bool(rep % 2))
            torch.cuda.synchronize()
            out["ok"].append(bool(torch.equal(t, want)))
    # hipGraph replay of the same call
    t = torch.empty(8192 * 4, dtype=torch.bfloat16, device="cuda")
    car.all_reduce(t)
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(gr, stream=s):
            car.all_reduce(t)
    torch.cuda.current_stream().wait_stream(s)
    for it in range(3):
        base = torch.randn(t.numel(), device="cuda", generator=g).bfloat16()
        t.copy_(base * (rank + 1))
        both = [base * 1, base * 2]
        want = (both[0].float() + both[1].float()).bfloat16()
        gr.replay(); torch.cuda.synchronize()
        out["ok"].append(bool(torch.equal(t, want)))
    # the TP step graph's small collectives on the same buffers (fp32 SUM / MAX, all-gather)
    for n in [4, 4096 + 4, 64 * 512]:
        both = [torch.randn(n, device="cuda", generator=g) for _ in range(2)]
        t = both[rank].clone()
        car.all_reduce_f32(t, "sum")
        torch.cuda.synchronize()
        out["ok"].append(bool(torch.equal(t, both[0] + both[1])))
        t = both[rank].clone()
        car.all_reduce_f32(t, "max")
        out["ok"].append(bool(torch.equal(t, torch.maximum(both[0], both[1]))))
        ids = torch.arange(n, device="cuda", dtype=torch.int32) * (rank + 1)
        got = car.all_gather(ids)
        torch.cuda.synchronize()
        want = torch.stack([torch.arange(n, device="cuda", dtype=torch.int32) * (r + 1) for r in range(2)])
        out["ok"].append(bool(torch.equal(got, want)))
    out["healthy"] = car.healthy()
    dist.barrier()
    car.close()
print("RESULT " + json.dumps(out), flush=True)
dist.destroy_process_group()
"""


def test_custom_ar_two_processes_ipc(tmp_path):
    """Two ranks on GPU 0 exchange real IPC handles (the TP setup path, minus xGMI)."""
    script = tmp_path / "car_worker.py"
    script.write_text(_WORKER)
    env = dict(os.environ, ROOT=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT="29581")
    procs = [subprocess.Popen([sys.executable, "-u", str(script), str(r)], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(2)]
    outs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, o))
    res = []
    for rc, o in outs:
        assert rc == 0, o[-3000:]
        line = [ln for ln in o.splitlines() if ln.startswith("RESULT ")][-1]
        res.append(json.loads(line[7:]))
    for r in res:
        assert r["created"], res
        assert all(r["ok"]) and r["healthy"], r


@pytest.mark.parametrize("W", [2, 4, 8])
@pytest.mark.parametrize("two_shot", [False, True])
def test_custom_ar_fused_residual_and_row_stats(W, two_shot):
    """The row-parallel TP epilogue in one launch: h += sum over ranks of
    the projection outputs, ss[row] += sum(h_new^2) of the written bf16 rows, ss_zero <- 0;
    against an fp32 PyTorch reference, bit-exact for h, at 70B (8192) and 8B (4096) widths."""
    from pilottai_amd.parallel.custom_ar import local_group_all_reduce

    C = _C()
    state = {}
    cap = 1 << 22
    g = torch.Generator(device="cuda").manual_seed(100 + W)
    for rows, d in [(1, 8192), (7, 8192), (64, 4096), (200, 8192)]:
        for rep in range(2):
            ins = [torch.randn(rows * d, device="cuda", generator=g).bfloat16() for _ in range(W)]
            h0 = torch.randn(rows, d, device="cuda", generator=g).bfloat16()
            hs = [h0.clone().reshape(-1) for _ in range(W)]  # replicated residual stream
            ss = [torch.zeros(rows, device="cuda") for _ in range(W)]
            junk = [torch.full((rows,), 5.0, device="cuda") for _ in range(W)]
            local_group_all_reduce(C, ins, cap, two_shot, state, resids=hs, ss=ss, ss_zero=junk, row_len=d)
            torch.cuda.synchronize()
            acc = h0.float().reshape(-1)
            tot = torch.zeros_like(acc)
            for t in ins:
                tot += t.float()
            want = (tot + acc).bfloat16()  # rank-order fp32 sum, then the residual, one rounding
            for r in range(W):
                assert torch.equal(hs[r], want), (rows, d, rep, r)
                torch.testing.assert_close(ss[r], want.float().view(rows, d).pow(2).sum(-1), rtol=1e-5, atol=1e-3)
                assert float(junk[r].abs().max()) == 0.0
    err = state[(W, cap)][2]
    assert int(err.item()) == 0


@pytest.mark.parametrize("W", [2, 4, 8])
def test_custom_collectives_local_ranks(W):
    """The TP step graph's small collectives (custom_ar.hip co_kernel): fp32
    SUM in rank order (bit-exact vs a PyTorch rank-order sum), MAX, and the all-gather of 4-byte
    values, interleaved with bf16 all-reduces on the same buffers / epochs, W ranks in one
    launch, sizes from one vector to several chunks per workgroup; then in hipGraph replay."""
    from pilottai_amd.parallel.custom_ar import local_group_all_reduce, local_group_collective

    C = _C()
    state = {}
    cap = 1 << 20
    g = torch.Generator(device="cuda").manual_seed(100 + W)
    for n in [4, 1024 + 4, 64 * 512, cap // 8]:
        for rep in range(2):
            xs = [torch.randn(n, device="cuda", generator=g) for _ in range(W)]
            want = torch.zeros(n, device="cuda")
            for x in xs:
                want = want + x
            ins = [x.clone() for x in xs]
            local_group_collective(C, ins, cap, "sum", state)
            torch.cuda.synchronize()
            assert all(torch.equal(t, want) for t in ins), (n, rep)
            ins = [x.clone() for x in xs]
            local_group_collective(C, ins, cap, "max", state)
            mx = torch.stack(xs).max(0).values
            assert all(torch.equal(t, mx) for t in ins), (n, rep)
            ids = [torch.randint(0, 1 << 30, (n,), device="cuda", dtype=torch.int32, generator=g) for _ in range(W)]
            outs = local_group_collective(C, ids, cap, "gather", state)
            torch.cuda.synchronize()
            assert all(torch.equal(o, torch.stack(ids)) for o in outs), (n, rep)
            bf = [torch.randn(min(8 * n, cap // 2), device="cuda", generator=g).bfloat16() for _ in range(W)]
            want_bf = _ref(bf)
            local_group_all_reduce(C, bf, cap, rep % 2 == 1, state)
            torch.cuda.synchronize()
            assert all(torch.equal(t, want_bf) for t in bf)
    assert int(state[(W, cap)][2].item()) == 0
    # hipGraph replay: gather + sum + max captured back to back
    n = 4096
    keys = [torch.empty(n, device="cuda") for _ in range(W)]
    hist = [torch.empty(n, device="cuda") for _ in range(W)]
    gout = [torch.empty(W, n, device="cuda") for _ in range(W)]
    local_group_collective(C, keys, cap, "gather", state, outs=gout)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            local_group_collective(C, keys, cap, "gather", state, outs=gout)
            local_group_collective(C, hist, cap, "sum", state)
            local_group_collective(C, keys, cap, "max", state)
    torch.cuda.current_stream().wait_stream(s)
    for it in range(3):
        kx = [torch.randn(n, device="cuda", generator=g) for _ in range(W)]
        hx = [torch.randn(n, device="cuda", generator=g) for _ in range(W)]
        for d, x in zip(keys, kx):
            d.copy_(x)
        for d, x in zip(hist, hx):
            d.copy_(x)
        graph.replay()
        torch.cuda.synchronize()
        hs = torch.zeros(n, device="cuda")
        for x in hx:
            hs = hs + x
        for r in range(W):
            assert torch.equal(gout[r], torch.stack(kx)), (it, r)
            assert torch.equal(hist[r], hs), (it, r)
            assert torch.equal(keys[r], torch.stack(kx).max(0).values), (it, r)
    assert int(state[(W, cap)][2].item()) == 0


@pytest.mark.parametrize("W", [2, 4, 8])
def test_tp_topkp_phase_kernels_match_single_gpu(W):
    """The vocab-parallel top-k / top-p threshold (csrc/ops/sampling.hip tp_topkp_kernel, four
    phases with MAX / SUM reductions over the custom collectives between them) gives every shard
    the tau of the single-GPU kernel on the whole row: greedy / untruncated rows -inf, top-k,
    top-p, both, grammar-masked rows, a row whose allowed set lies in one shard."""
    from pilottai_amd import ops
    from pilottai_amd.engine.tp_sampling import tkp_ws_floats
    from pilottai_amd.ops import reference as ref
    from pilottai_amd.parallel.custom_ar import local_group_collective

    C = _C()
    torch.manual_seed(7 + W)
    rows, V = 13, 128256
    vl = V // W
    logits = (torch.randn(rows, V, device="cuda") * 3).bfloat16()
    temp = torch.tensor([0.7, 0.0, 1.0, 0.9, 1.3, 0.5, 0.8, 1.0, 0.6, 1.1, 0.9, 0.7, 1.0], device="cuda")
    top_k = torch.tensor([40, 40, 0, 5, 0, 1, 100, 0, 20, V, 7, 0, 3], device="cuda", dtype=torch.int32)
    top_p = torch.tensor([1.0, 0.9, 0.95, 0.8, 0.5, 1.0, 0.99, 1.0, 0.3, 0.7, 1.0, 0.999, 0.6], device="cuda")
    words = (V + 31) // 32
    masks = torch.zeros(3, words, dtype=torch.int32)
    masks[0] = -1
    allowed = torch.zeros(V, dtype=torch.bool)
    allowed[torch.randperm(V)[:3000]] = True
    masks[1] = ref.pack_mask(allowed.numpy())
    one_shard = torch.zeros(V, dtype=torch.bool)
    one_shard[vl + 17: vl + 900] = True  # every allowed token in shard 1
    masks[2] = ref.pack_mask(one_shard.numpy())
    masks = masks.cuda()
    mcls = torch.tensor([-1, -1, 0, 1, 1, 2, -1, -1, 2, -1, 1, 0, -1], device="cuda", dtype=torch.int32)
    want = ops.topkp_threshold(logits, V, temp, top_k, top_p, mcls, masks)
    shards = [logits[:, w * vl:(w + 1) * vl] for w in range(W)]
    wss = [torch.zeros(tkp_ws_floats(rows), device="cuda") for _ in range(W)]
    taus = [torch.empty(rows, device="cuda") for _ in range(W)]
    r4 = (rows + 3) & ~3
    seg = {"mx": (0, r4), "h0": (r4, r4 + rows * 512), "h1": (r4 + rows * 512, r4 + rows * 1024)}
    state = {}
    cap = 1 << 20

    def phase(ph):
        for w in range(W):
            C.tp_topkp_phase(ph, taus[w], wss[w], shards[w], w * vl, V, temp, top_k, top_p, mcls, masks)

    def reduce(name, op):
        a, b = seg[name]
        local_group_collective(C, [ws[a:b] for ws in wss], cap, op, state)

    phase(0)
    reduce("mx", "max")
    phase(1)
    reduce("h0", "sum")
    phase(2)
    reduce("h1", "sum")
    phase(3)
    torch.cuda.synchronize()
    for w in range(W):
        assert torch.equal(taus[w], taus[0])
    torch.testing.assert_close(taus[0], want, atol=0, rtol=0)
    assert float(taus[0][1]) == float("-inf") and float(taus[0][7]) == float("-inf")  # greedy / untruncated

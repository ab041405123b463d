"""Tensor-parallel engine on the GPU with the custom P2P all-reduce (TP=2, 4 and 8, every rank
on GPU 0 over real IPC handles; gloo carries the host-side step headers).

Mirrors tests/test_tp_cpu.py: the TP=N engine (canonical sharded init -> exactly the TP=1
weights) must choose, at every generated position, a token the TP=1 model's fp32 reference
forward ranks as the argmax (greedy) or inside its top 20 (top-k 20 sampling), teacher-forced
on the TP run's own tokens, and keep structured output valid, with every row-parallel
all-reduce going through csrc/ops/custom_ar.hip.

The bound: TP=N rounds each rank's row-parallel partial output to bf16 before the rank-order
fp32 sum, TP=1 rounds the full sum once, so activations differ by up to N bf16 roundings
(N x 2^-9 relative) per projection; through the tiny model's 2 layers that moves a logit by well
under 1 % of the row's logit range, the tolerance used (TOL_FRAC). An exact token-for-token
match is therefore not guaranteed at near-ties; a wrong kernel or collective (a dropped shard,
a stale buffer) misses the reference's argmax by far more.
The graph-on variant is the production TP mode: every bucket captured
up front with the collectives inside, all of them on the custom P2P buffers -- the
activations' all-reduces, the sampling winners' all-gather and the top-k / top-p
threshold's MAX / SUM reductions; a hook on torch.distributed proves that no RCCL / gloo
call is made while a graph is being captured.
"""
import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


MODEL = "tiny-kv8"  # 8 KV heads: TP = 1, 2, 4 and 8 hold exact slices of the same weights
TOL_FRAC = 0.01


def _cfg(graphs=False):
    from pilottai_amd.engine.engine import EngineConfig

    return EngineConfig(model=MODEL, max_num_seqs=8, max_num_batched_tokens=128, max_model_len=512,
                        num_kv_blocks=96, use_graphs=graphs, token_buckets=[8, 16, 32, 64, 128])


_COLLECTIVES = ("all_reduce", "all_gather", "all_gather_into_tensor", "broadcast", "reduce_scatter_tensor",
                "all_to_all_single", "barrier", "all_gather_object", "broadcast_object_list")


def _hook_collectives(box):
    """Count torch.distributed collectives issued while a hipGraph is being captured."""
    import torch.distributed as dist

    for name in _COLLECTIVES:
        fn = getattr(dist, name)

        def wrapped(*a, _fn=fn, _name=name, **k):
            if torch.cuda.is_current_stream_capturing():
                box.append(_name)
            return _fn(*a, **k)
        setattr(dist, name, wrapped)


def _prompts(tok):
    return [tok.encode("Task: summarize the quarterly report."), tok.encode("Task: plan a trip")]


def _worker(rank, world, port, out_path, graphs=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from pilottai_amd.engine.engine import LLMEngine
    from pilottai_amd.parallel.comm import init_distributed, new_tp_groups

    init_distributed("gloo")
    torch.cuda.set_device(0)
    tp = new_tp_groups(world, custom_ar=True)
    assert tp.custom is not None, "custom all-reduce did not initialise"
    in_graph = []
    _hook_collectives(in_graph)
    e = LLMEngine(_cfg(graphs), device=torch.device("cuda", 0), tp=tp)
    assert e.use_graphs == graphs
    if rank != 0:
        e.follow()
        torch.distributed.destroy_process_group()
        return
    ps = _prompts(e.tok)
    greedy = e.generate(ps, temperature=0.0, max_tokens=6, ignore_eos=True)
    segs = e.grammar.compile("orchestrator.result_evaluation")
    js = e.generate([ps[0]], temperature=0.8, max_tokens=64, grammar=segs)[0]
    # top-k / top-p rows: the TP threshold (HIP phases + custom MAX / SUM) inside the graph
    tk = e.generate(ps, temperature=0.9, max_tokens=12, ignore_eos=True, top_k=20, top_p=0.9)
    e.release_followers()
    with open(out_path, "w") as f:
        json.dump({"greedy": [o.token_ids for o in greedy], "json": js.text, "calls": tp.custom.calls,
                   "healthy": tp.custom.healthy(), "graphs": len(e._graphs), "in_graph": in_graph,
                   "topk": [o.token_ids for o in tk]}, f)
    torch.distributed.destroy_process_group()


def _near_rank(model, prompt, toks, k):
    """Per generated position: (logit of the chosen token, k-th largest logit, logit range) of
    the TP=1 fp32 reference forward, teacher-forced on prompt + toks."""
    logits = model.reference_logits(prompt + toks[:-1]).float()
    out = []
    for i, t in enumerate(toks):
        row = logits[len(prompt) - 1 + i]
        out.append((float(row[t]), float(torch.topk(row, k).values[-1]), float(row.max() - row.min())))
    return out


# TP=8 with all 8 ranks on ONE GPU does not run: even with 8 all-reduce workgroups per rank and one
# hardware queue per process, some rank's peer never arrives and the 5 s all-reduce watchdog
# stops the engine (profiles/r6_tp_share_gpu.md); TP=2 / 4 run with the rehearsal settings below
@pytest.mark.parametrize("world,graphs", [(2, False), (2, True), (4, False), (4, True)])
def test_tp_engine_custom_allreduce_matches_tp1(tmp_path, world, graphs):
    out = str(tmp_path / "tp.json")
    port = _free_port()
    # all `world` ranks share GPU 0 here: every rank's all-reduce workgroups spin until their
    # peers' arrive, so the ranks' kernels must run side by side. At the default 128 all-reduce
    # workgroups per rank, 3+ spinning ranks occupy every CU and a peer's GEMM that needs a whole
    # CU never starts (round 6: TP=4 hit the 5 s all-reduce watchdog); the rehearsal runs 8
    # all-reduce workgroups per rank and one hardware queue per process. A node has one rank per GPU.
    saved = {k: os.environ.get(k) for k in ("GPU_MAX_HW_QUEUES", "PILOTTAI_CAR_WG")}
    if world >= 4:
        os.environ.update(GPU_MAX_HW_QUEUES="1", PILOTTAI_CAR_WG="8")
    try:
        mp.start_processes(_worker, args=(world, port, out, graphs), nprocs=world, join=True, start_method="spawn")
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    res = json.load(open(out))
    assert res["calls"] > 0 and res["healthy"], res
    assert [len(t) for t in res["topk"]] == [12, 12]
    if graphs:
        assert res["graphs"] >= 5  # every bucket captured up front (+ first-use variants)
        assert res["in_graph"] == [], res["in_graph"]  # no RCCL / gloo call inside a graph
    obj = json.loads(res["json"])
    assert set(obj) == {"success", "quality", "requires_retry"}

    from pilottai_amd.engine.engine import LLMEngine

    e1 = LLMEngine(_cfg(), device=torch.device("cuda", 0))
    ps = _prompts(e1.tok)
    ref = e1.generate(ps, temperature=0.0, max_tokens=6, ignore_eos=True)
    exact = sum(a == o.token_ids for a, o in zip(res["greedy"], ref))
    for p, toks in zip(ps, res["greedy"]):
        for i, (lt, top, rng) in enumerate(_near_rank(e1.model, p, toks, 1)):
            assert lt >= top - TOL_FRAC * rng, (world, i, lt, top, rng)
    for p, toks in zip(ps, res["topk"]):
        for i, (lt, kth, rng) in enumerate(_near_rank(e1.model, p, toks, 20)):
            assert lt >= kth - TOL_FRAC * rng, (world, i, lt, kth, rng)
    print(f"TP={world} graphs={graphs}: {exact}/{len(ps)} greedy sequences identical to TP=1")

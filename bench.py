#!/usr/bin/env python3
"""Flagship benchmark — BASELINE.json metric on BASELINE config 3:

    "completed agent-tasks/sec (whole node) + p50 task latency, 64 concurrent workers"
    "Manager + 64 workers, Llama-3-8B continuous-batched across N x MI355X (agent-DP)"

One process per GPU (torchrun); the 64 worker agents are sharded over the ranks
(strong scaling: the node always runs 64 concurrent workers), each rank with an
on-node Llama-3-8B engine (random-init bf16 weights, full 32-layer architecture).
ONE manager `Serve` on rank 0 orchestrates the node-wide pool: the agents of the other
ranks are reached through the node control plane (parallel/node_plane.py), the
manager's own LLM calls go to the least-loaded rank. 64 closed-loop clients on rank 0
each submit a synthetic document task, await the TaskResult, submit the next.
(`--dp-mode independent`: one Serve per rank over its own shard, round 1's layout.)

Per-task LLM work is fixed by the `fixed` control policy (core/policy.py) and the
reply schemas (source/rules.yaml): 7 LLM calls per task — orchestrator analysis,
agent task analysis, tool selection, 2 step plans (one echo-tool step), agent
evaluation, orchestrator evaluation — each prefilled in full and decoded under a
JSON grammar (sampled tokens bounded by the schema's slot sizes).

A "step" = every one of the 64 workers completes one task (64 tasks). W warmup
steps are untimed; K steps are timed between barrier + device synchronize on all
ranks; the reported time is the max over ranks. Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import secrets
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "completed agent-tasks/sec (whole node) + p50 task latency, 64 concurrent workers"

_WORDS = ("market revenue growth quarter customer product launch risk supply chain analysis report "
          "engineering latency throughput model deployment cluster memory compute budget forecast "
          "policy compliance audit review summary insight strategy partner contract region sales "
          "pipeline incident outage mitigation roadmap hiring cost margin inventory logistics").split()


def synth_document(rng: random.Random, n_words: int) -> str:
    return " ".join(rng.choice(_WORDS) for _ in range(n_words))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workers", type=int, default=64)
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--doc-words", type=int, default=120)
    ap.add_argument("--kv-gb", type=float, default=None,
                    help="KV-cache size per GPU (default: 85%% of the HBM left after the weights; 48 GB "
                         "with --share-gpu). 288 GB per MI355X: a large pool keeps the prefix cache "
                         "hitting over long runs (48 GB: 59.7%% hits over 20 steps vs 64.8%% at 160 GB)")
    ap.add_argument("--max-batched-tokens", type=int, default=2048)
    ap.add_argument("--temperature", type=float, default=0.7)
    ap.add_argument("--steps-per-task", type=int, default=1)
    ap.add_argument("--fused-max-t", type=int, default=None,
                    help="largest step on the fused packed-weight decode path (default: the model's)")
    ap.add_argument("--mid-max-t", type=int, default=None,
                    help="largest step on the LDS-DMA tiled mid-size path (default: the model's; 0 = off)")
    ap.add_argument("--prefill-max-t", type=int, default=None,
                    help="largest step on the fused packed path with the 256x256 prefill GEMMs; 0 = library path")
    ap.add_argument("--att-wide-min-tokens", type=int, default=None,
                    help="prefill tokens per step from which attention uses the 4-wave LDS-staged items")
    ap.add_argument("--no-prefix-dedup", action="store_true",
                    help="admit requests whose prefix another request is prefilling right away (no deferral)")
    ap.add_argument("--token-align", type=int, default=256, help="GEMM-friendly step sizes (0 = off)")
    ap.add_argument("--pf-midrange", default=None,
                    help="comma-separated projections (qkv,o,gate_up,down) on the prefill kernels at <= 256 tokens "
                         "per LlamaModel.PF_CFG; 'none' = mid kernel only (default: model's)")
    ap.add_argument("--att-decode-waves", type=int, default=None, choices=[4, 8],
                    help="attention workgroup width on decode-sized steps (default: model's)")
    ap.add_argument("--async-steps", type=int, default=None, choices=[0, 1],
                    help="pipelined engine steps (schedule/launch step N+1 while step N runs); default: engine's")
    ap.add_argument("--align-slack", type=int, default=96)
    ap.add_argument("--cpu", action="store_true", help="tiny model on CPU (plumbing smoke only)")
    ap.add_argument("--dp-mode", choices=["node", "independent"], default="node",
                    help="node: one manager over the node-wide pool; independent: one Serve per rank")
    ap.add_argument("--reply-tokens", type=int, default=None,
                    help="fixed length of every reply's free-text slot (workload sensitivity; default: schema sizes)")
    ap.add_argument("--memory-rows", type=int, default=0,
                    help="semantic memory on the engine's GPU with this many rows; every agent step looks it up")
    ap.add_argument("--memory-top-k", type=int, default=3)
    ap.add_argument("--memory-storage", default="q16", choices=["bf16", "q16"],
                    help="index row format: q16 (default: 16-bit fixed point, two-stage exact scan streaming "
                         "one byte per dimension, csrc/ops/similarity_q16.hip; config 4 32.4 vs 28.6 tasks/s, "
                         "profiles/r6_q16_stage1.md) or bf16 (one-pass bf16 scan)")
    ap.add_argument("--memory-min-batch", type=int, default=1,
                    help="lookups a pass waits for (up to --memory-wait-ms) before it starts")
    ap.add_argument("--memory-wait-ms", type=float, default=0.0)
    ap.add_argument("--memory-gate-tokens", type=int, default=1024,
                    help="start index passes beside engine steps of at least this many tokens (compute-bound), "
                         "0 = as soon as lookups are pending")
    ap.add_argument("--memory-gate-ms", type=float, default=30.0,
                    help="latency cap of the gate: a lookup waits at most this long for such a step")
    ap.add_argument("--embed-pooling", default="last", choices=["mean", "last"],
                    help="--embedder engine: last-token states (embedding requests reuse the prefix cache: an "
                         "agent's successive lookups share the task text) or mean pooling (no reuse)")
    ap.add_argument("--embedder", default="hashing", choices=["hashing", "engine"],
                    help="memory text encoder: feature hashing, or the serving model itself (embedding "
                         "requests in the engine's continuous batch, SURVEY N11)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal: every rank on GPU 0 (use with PILOTTAI_DIST_BACKEND=gloo)")
    ap.add_argument("--tp", type=int, default=1,
                    help="tensor-parallel degree of each agent-DP replica: --gpus N runs N/T replicas, each "
                         "one TP=T engine over T GPUs (custom P2P all-reduce); the node plane sees one rank "
                         "per replica (its TP rank 0). Default 1 = pure agent-DP (BENCHMARKS.md cost model)")
    ap.add_argument("--hybrid-latency", type=float, default=0.0,
                    help="hybrid node rehearsal on ONE GPU (VERDICT r3 item 5): rank 0 runs the real engine, "
                         "the manager Serve, the control plane and all clients; ranks > 0 are CPU processes whose "
                         "agents answer with model-free schema LLMs after this many seconds per call (the measured "
                         "per-call latency of an 8-worker GPU rank). Use with PILOTTAI_DIST_BACKEND=gloo.")
    return ap.parse_args()


async def run_rank(a, rank: int, world: int, device, tp=None, dp_group=None):
    """rank / world: global. With --tp T the agent-DP replicas are the TP groups: drank / dworld
    index the replicas, only each group's TP rank 0 runs agents and the control plane, the other
    TP ranks follow their driver's engine steps (LLMEngine.follow)."""
    import torch

    from pilottai_amd.core.agent import BaseAgent
    from pilottai_amd.core.config import AgentConfig, LLMConfig
    from pilottai_amd.core.policy import ControlPolicy
    from pilottai_amd.core.task import Task
    from pilottai_amd.engine.engine import EngineConfig, LLMEngine
    from pilottai_amd.engine.local_llm import LocalLLM
    from pilottai_amd.engine.registry import register_engine
    from pilottai_amd.parallel import comm
    from pilottai_amd.serve import Serve
    from pilottai_amd.tools.tool import Tool, echo_tool

    # workers of this rank (agent-DP sharding)
    from pilottai_amd.parallel.agent_dp import shard_workers

    from pilottai_amd.parallel.comm import TPGroup

    tp = tp or TPGroup.single()
    T = tp.size
    dworld, drank = world // T, rank // T
    n_local = len(shard_workers(a.workers, dworld, drank))
    t_init = time.time()
    if T > 1 and (a.memory_rows > 0 or a.hybrid_latency > 0 or a.dp_mode != "node"):
        raise SystemExit("--tp > 1 runs the node mode without --memory-rows / --hybrid-latency")
    if a.hybrid_latency > 0 and a.memory_rows > 0 and world > 1:
        raise SystemExit("--memory-rows needs an engine on every rank: not with --hybrid-latency")
    if a.hybrid_latency > 0 and rank > 0:
        return await run_cpu_rank(a, rank, world, n_local)
    memory = lookup = None
    if a.memory_rows > 0:
        # before the engine sizes its KV pool: the index is resident beside the model
        memory, lookup = build_memory(a, device, rank, world, node=a.dp_mode == "node" and world > 1)
    eng = LLMEngine(EngineConfig(model=a.model if not a.cpu else ("tiny" if T == 1 else "tiny-gqa4"),
                                 max_num_seqs=max(64, 2 * n_local),
                                 max_num_batched_tokens=a.max_batched_tokens,
                                 max_prefill_tokens=a.max_batched_tokens,
                                 kv_cache_gb=None if a.cpu else (a.kv_gb if a.kv_gb is not None else
                                                                 (48.0 / max(1, world) if a.share_gpu else None)),
                                 kv_cache_fraction=0.85,
                                 num_kv_blocks=4096 if a.cpu else None, seed=1234 + drank,
                                 token_align=a.token_align, align_slack=a.align_slack,
                                 decode_fused_max_t=a.fused_max_t,
                                 mid_max_t=a.mid_max_t, prefill_max_t=a.prefill_max_t,
                                 reply_tokens=a.reply_tokens,
                                 dedup_inflight_prefix=not a.no_prefix_dedup,
                                 **({"async_steps": bool(a.async_steps)} if a.async_steps is not None else {}),
                                 **({"att_decode_waves": a.att_decode_waves} if a.att_decode_waves is not None else {}),
                                 **({"pf_midrange": [k for k in a.pf_midrange.split(",") if k and k != "none"]}
                                    if a.pf_midrange is not None else {}),
                                 **({"att_wide_min_tokens": a.att_wide_min_tokens}
                                    if a.att_wide_min_tokens is not None else {})), device=device, tp=tp)
    if tp.rank != 0:  # a TP follower: replay the driver's steps until it stops the engine
        await asyncio.to_thread(eng.follow)
        return {"follower": True, "device": _device_identity(device)}
    register_engine(eng.model_cfg.name, eng)
    if memory is not None and a.embedder == "engine":
        # queries and write-backs are encoded by the serving model: final hidden states (last
        # token, or mean-pooled) of embedding requests inside the engine's continuous batch (N11)
        from pilottai_amd.memory.embedding import EngineEmbedder

        memory.embedder = EngineEmbedder(eng, dim=memory.index.dim, pool="engine", max_tokens=256,
                                         pooling=a.embed_pooling)
    if memory is not None and a.embedder == "engine" and not a.cpu:
        eng.capture_embed_graphs()  # embedding requests: no first-use captures while timed
    if lookup is not None and a.memory_gate_tokens > 0:
        lookup.attach_engine(eng, gate_tokens=a.memory_gate_tokens, max_wait_s=a.memory_gate_ms / 1000.0)
    eng.start()
    llm = LocalLLM(LLMConfig(model_name=eng.model_cfg.name, temperature=a.temperature, max_tokens=1024,
                             retry_attempts=1), engine=eng)
    policy = ControlPolicy("fixed", a.steps_per_task)
    agents = []
    for i in range(n_local):
        cfg = AgentConfig(role=f"analyst-{rank}-{i}", goal="Summarize documents and extract key findings",
                          backstory="A careful analyst agent in a document-processing workflow.",
                          max_iterations=a.steps_per_task + 1, task_timeout=900)
        agents.append(BaseAgent(cfg, llm=llm, tools=[Tool(name="echo", description="identity tool",
                                                          function=echo_tool, max_retries=1)], policy=policy,
                                memory_lookup=lookup, memory_top_k=a.memory_top_k))
    node = a.dp_mode == "node" and dworld > 1
    serve_cfg = {"name": f"bench-r{rank}", "policy": "fixed", "steps_per_task": a.steps_per_task,
                 "max_queue_size": 100000, "task_timeout": 900, "agent_wait_timeout": 900}
    async def coll(fn, *args):
        """A blocking collective off the event loop (worker ranks keep serving the control
        plane meanwhile); the thread binds this rank's GPU first (RCCL uses the current device)."""
        def run():
            if device.type == "cuda":
                torch.cuda.set_device(device)
            if fn is comm.broadcast_object or fn is comm.barrier:  # over the replicas (TP drivers)
                return fn(*args, group=dp_group)
            return fn(*args)
        return await asyncio.to_thread(run)

    serve = plane = worker = None
    if node:  # the control plane's shared secret: drawn on rank 0, broadcast to the job's ranks
        os.environ["PILOTTAI_PLANE_SECRET"] = await coll(
            comm.broadcast_object, secrets.token_hex(16) if rank == 0 else None)
    if node and drank > 0:
        # worker rank: host this shard's agents (and this GPU's engine) for the manager
        from pilottai_amd.parallel.node_plane import PlaneWorker

        for ag in agents:
            await ag.start()

        def kv_load():
            m = eng.metrics()
            return {"kv_cache_utilization": 1.0 - m.get("free_kv_blocks", 1) / max(1, m.get("total_kv_blocks", 1))}
        worker = PlaneWorker(drank, agents, llm=llm, load_fn=kv_load)
        await worker.connect()
        serving = asyncio.ensure_future(worker.serve_forever())
    elif node:
        from pilottai_amd.parallel.node_plane import DistributedLLM, NodeManager, PlaneServer

        plane = PlaneServer(dworld)
        await plane.start()
        serve = Serve(agents=agents, config={**serve_cfg, "max_concurrent_tasks": a.workers})
        mgr = NodeManager(plane, serve)
        mgr.register_local(agents)
        mgr.attach_remote_agents()
        serve._manager_llm = DistributedLLM(plane, llm)
        await serve.start()
    else:
        serve = Serve(agents=agents, manager_llm=llm, config={**serve_cfg, "max_concurrent_tasks": n_local})
        await serve.start()
    # shared-context broadcast: rank 0 fixes the workload seed for every rank
    seed = await coll(comm.broadcast_object, int(time.time()) & 0xFFFF if rank == 0 else None)
    init_s = time.time() - t_init
    n_clients = a.workers if node else n_local  # node mode: all 64 clients talk to the one manager

    latencies = []

    async def client(ci: int, n_tasks: int, rec: bool):
        rng = random.Random(seed * 1000003 + rank * 1009 + ci * 7 + (0 if rec else 99991))
        for _ in range(n_tasks):
            doc = synth_document(rng, a.doc_words)
            t0 = time.perf_counter()
            r = await serve.execute_task(Task(description=f"Summarize the document and list its key findings: {doc}"))
            dt = time.perf_counter() - t0
            if not r.success:
                raise RuntimeError(f"task failed: {r.error}")
            if rec:
                latencies.append(dt)

    async def round_(n, rec):
        if serve is not None and not (node and drank > 0):
            await asyncio.gather(*(client(i, n, rec) for i in range(n_clients)))

    lags = []

    async def lag_probe(stop):
        """Event-loop lag of this rank: how late a 10 ms sleep wakes up (the manager, the plane
        server, the clients and the engine's delivery callbacks share this loop)."""
        loop = asyncio.get_running_loop()
        while not stop.is_set():
            t = loop.time()
            await asyncio.sleep(0.01)
            lags.append(loop.time() - t - 0.01)

    if a.warmup > 0:
        await round_(a.warmup, False)
    from pilottai_amd.utils.gc_tune import freeze_heap

    freeze_heap()  # agents, serve and warm-up state: out of the timed region's GC passes
    await coll(comm.barrier)  # worker ranks keep serving the plane meanwhile
    st0 = dict(eng.stats)  # after the barrier: every rank's warmup work is behind it
    mem0 = dict(lookup.stats, device_s=lookup.lookup_device_seconds(), nlat=lookup.lat_count) \
        if lookup is not None else None
    bh0 = {b: list(v) for b, v in eng.bucket_hist.items()}
    u0 = dict(llm.usage)
    n_timed0 = len(eng.timings)
    if device.type == "cuda":
        torch.cuda.synchronize()
    if device.type == "cuda":  # marker kernels: tools/prof_summary.py --between-markers cuts profiles here
        from pilottai_amd.ops import kernels as _k

        _k.require_native().timeline_marker(0)
    t0 = time.perf_counter()
    stop_probe = asyncio.Event()
    probe = asyncio.ensure_future(lag_probe(stop_probe))
    await round_(a.steps, True)
    stop_probe.set()
    await probe
    if device.type == "cuda":
        _k.require_native().timeline_marker(1)
        torch.cuda.synchronize()
    await coll(comm.barrier)
    dt = time.perf_counter() - t0
    st1 = dict(eng.stats)
    u1 = dict(llm.usage)
    em = eng.metrics()
    mem = None
    if lookup is not None:
        dev_s = lookup.lookup_device_seconds()
        mem = {"rows": memory.index.count, "index_gb": round(memory.index.memory_bytes() / 2**30, 2),
               # node mode: ONE node-wide store, rows sharded over the ranks (memory/node_store.py)
               "store": "node-sharded" if hasattr(memory, "search_rows_blocking") else "single-index",
               "storage": memory.index.storage,
               "q16_fallbacks": memory.index.stats.get("q16_fallbacks", 0),
               "node_rounds": memory.stats.get("rounds") if hasattr(memory, "search_rows_blocking") else None,
               "lookups": lookup.stats["lookups"] - mem0["lookups"],
               # the encoder's work when the serving model embeds (--embedder engine):
               # embedding requests and their prefilled tokens inside the continuous batch
               "embedder": a.embedder,
               "embed_pooling": a.embed_pooling if a.embedder == "engine" else None,
               "embed_cached_tokens": st1.get("embed_cached_tokens", 0) - st0.get("embed_cached_tokens", 0),
               "embed_requests": st1["embed_requests"] - st0["embed_requests"],
               "embed_tokens": st1["embed_tokens"] - st0["embed_tokens"],
               "embed_token_share": round((st1["embed_tokens"] - st0["embed_tokens"]) /
                                          max(1, st1["tokens"] - st0["tokens"]), 4),
               "passes": lookup.stats["passes"] - mem0["passes"],
               # co-scheduling with compute-bound engine steps (memory/batcher.py attach_engine)
               "gate_tokens": a.memory_gate_tokens,
               "passes_beside_heavy": lookup.stats["passes_beside_heavy"] - mem0["passes_beside_heavy"],
               "passes_capped": lookup.stats["passes_capped"] - mem0["passes_capped"],
               "beside_heavy_frac": round((lookup.stats["passes_beside_heavy"] - mem0["passes_beside_heavy"]) /
                                          max(1, lookup.stats["passes"] - mem0["passes"]), 3),
               **lookup.latency_summary(mem0["nlat"]),
               "stores": lookup.stats["stores"] - mem0["stores"],
               "store_failures": lookup.stats["store_failures"] - mem0["store_failures"],
               "lookup_failures": lookup.stats["lookup_failures"] - mem0["lookup_failures"],
               # node store: hits returned to this rank's agents that another rank's shard holds
               "node_hits": memory.stats.get("hits") if hasattr(memory, "search_rows_blocking") else None,
               "node_remote_hits": memory.stats.get("remote_hits") if hasattr(memory, "search_rows_blocking")
               else None,
               # flushes whose writes and queries went through the engine in one embedding call
               "shared_embeds": lookup.stats.get("shared_embeds", 0) - mem0.get("shared_embeds", 0),
               # where a lookup's latency goes, ms per pass (embedding through the engine, the
               # gate's wait for a compute-bound step, the index pass) and per lookup (queued
               # behind the pass in flight before its own flush starts)
               "lookup_anatomy_ms": {
                   k: round(1000 * (lookup.stats.get(k + "_s", 0.0) - mem0.get(k + "_s", 0.0)) /
                            max(1, (lookup.stats["lookups"] - mem0["lookups"]) if k == "queued"
                                else (lookup.stats["passes"] - mem0["passes"])), 2)
                   for k in ("embed", "gate_wait", "search", "queued")},
               # HIP events around each pass on the lookup stream (includes any wait for
               # CUs the engine holds: an upper bound on the passes' kernel time)
               "lookup_device_s": round(dev_s - mem0["device_s"], 3),
               "lookup_ms_per_pass": round(1000 * (dev_s - mem0["device_s"]) /
                                                  max(1, lookup.stats["passes"] - mem0["passes"]), 2)}
    node_load = None
    if world > 1 and a.dp_mode == "independent":
        # node-wide load picture (parallel/agent_dp.py GlobalLoadView) after the run
        from pilottai_amd.parallel.agent_dp import GlobalLoadView, local_load

        node_load = (await coll(GlobalLoadView().update, local_load(serve)))
    requeued = 0
    by_rank = None
    if plane is not None:
        requeued = int(serve.metrics.get("requeued_tasks", 0))
        by_rank = {str(k): v for k, v in mgr.executions_by_rank().items()}
        await serve.stop()
        await plane.stop()
    elif worker is not None:
        await serving
        for ag in agents:
            await ag.stop()
    else:
        await serve.stop()
    if memory is not None and hasattr(memory, "search_rows_blocking"):
        await asyncio.to_thread(memory.stop)  # leaves once every rank has stopped
    eng.stop()
    local = {
        "dt": dt, "tasks": len(latencies), "lat": latencies, "init_s": init_s, "requeued": requeued,
        "device": _device_identity(device),
        "mem_rows": memory.index.count if memory is not None else 0,
        "loop_lag": sorted(lags), "executions_by_rank": by_rank,
        "managers": 1 if serve is not None else 0, "dp_mode": a.dp_mode if dworld > 1 else "single",
        "tokens": st1["tokens"] - st0["tokens"], "steps": st1["steps"] - st0["steps"],
        "sampled": st1["sampled"] - st0["sampled"], "calls": u1["calls"] - u0["calls"],
        "prompt_tokens": u1["prompt_tokens"] - u0["prompt_tokens"],
        "completion_tokens": u1["completion_tokens"] - u0["completion_tokens"],
        "busy_s": st1["busy_s"] - st0["busy_s"], "prefix_hit": em["prefix_cache_hit_tokens"],
        "graph_captures": st1.get("graph_captures", 0) - st0.get("graph_captures", 0),
        "prefix_defers": em["prefix_defers"],
        "spec_rows": em.get("spec_rows", 0),
        "spec_voided": em.get("spec_voided", 0),
        "async_steps": bool(eng._async),
        "host_phases": {k: st1[k] - st0[k] for k in ("host_sched_s", "host_launch_s", "device_wait_s",
                                                     "host_commit_s", "host_deliver_s")},
        "bucket_tokens": st1["bucket_tokens"] - st0["bucket_tokens"],
        "prompt_total": em["prompt_tokens"], "hbm_used_gb": em.get("hbm_used_gb", 0.0),
        "weights_gb": em.get("weights_gb", 0.0), "kv_cache_gb": em.get("kv_cache_gb", 0.0),
        "req_lat": eng.latency_summary(n_timed0), "memory": mem, "node_load": node_load,
        "buckets": {b: [v[0] - bh0.get(b, [0, 0.0])[0], v[1] - bh0.get(b, [0, 0.0])[1]]
                    for b, v in eng.bucket_hist.items()},
    }
    return local


async def run_cpu_rank(a, rank: int, world: int, n_local: int):
    """--hybrid-latency: a worker rank without a GPU or engine (agents on schema LLMs that
    answer after a fixed latency), joining rank 0's control plane like a GPU rank does."""
    from pilottai_amd.core.agent import BaseAgent
    from pilottai_amd.core.config import AgentConfig
    from pilottai_amd.core.policy import ControlPolicy
    from pilottai_amd.engine.local_llm import SchemaLLM
    from pilottai_amd.parallel import comm
    from pilottai_amd.parallel.node_plane import PlaneWorker
    from pilottai_amd.tools.tool import Tool, echo_tool

    t_init = time.time()
    llm = SchemaLLM(seed=rank, latency_s=a.hybrid_latency)
    policy = ControlPolicy("fixed", a.steps_per_task)
    agents = [BaseAgent(AgentConfig(role=f"analyst-{rank}-{i}", goal="Summarize documents and extract key findings",
                                    max_iterations=a.steps_per_task + 1, task_timeout=900), llm=llm,
                        tools=[Tool(name="echo", description="identity tool", function=echo_tool, max_retries=1)],
                        policy=policy)
              for i in range(n_local)]

    async def coll(fn, *args):
        return await asyncio.to_thread(fn, *args)

    os.environ["PILOTTAI_PLANE_SECRET"] = await coll(comm.broadcast_object, None)
    for ag in agents:
        await ag.start()
    worker = PlaneWorker(rank, agents, llm=llm)
    await worker.connect()
    serving = asyncio.ensure_future(worker.serve_forever())
    await coll(comm.broadcast_object, None)  # the workload seed
    init_s = time.time() - t_init
    await coll(comm.barrier)
    t0 = time.perf_counter()
    await coll(comm.barrier)
    dt = time.perf_counter() - t0
    await serving
    for ag in agents:
        await ag.stop()
    zero = {k: 0 for k in ("tokens", "steps", "sampled", "busy_s", "prefix_hit", "prefix_defers", "spec_rows",
                           "spec_voided", "bucket_tokens", "prompt_total", "hbm_used_gb", "graph_captures",
                           "weights_gb", "kv_cache_gb")}
    return dict(zero, dt=dt, tasks=0, lat=[], init_s=init_s, requeued=0, loop_lag=[], executions_by_rank=None,
                device=_device_identity(None),
                managers=0, dp_mode="node", calls=len(llm.calls) if hasattr(llm, "calls") else 0, prompt_tokens=0,
                completion_tokens=0, async_steps=False, host_phases={}, req_lat={}, memory=None, node_load=None,
                buckets={}, cpu_rank=True)


def _device_identity(device) -> dict:
    """What this rank actually ran on: the torch device and, for a GPU, the physical card's
    identity (UUID / PCI bus id) -- so the driver can check that an N-GPU line used N cards."""
    if device is None or device.type != "cuda":
        return {"device": "cpu", "physical": None}
    import torch

    idx = device.index if device.index is not None else torch.cuda.current_device()
    props = torch.cuda.get_device_properties(idx)
    dom, bus, dev = (getattr(props, k, None) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
    if bus is not None:
        phys = f"pci:{int(dom or 0):04x}:{int(bus):02x}:{int(dev or 0):02x}"
    else:
        phys = f"visible:{os.environ.get('HIP_VISIBLE_DEVICES', os.environ.get('CUDA_VISIBLE_DEVICES', ''))}/{idx}"
    return {"device": f"cuda:{idx}", "physical": phys, "name": props.name, "uuid": str(getattr(props, "uuid", ""))}


def build_memory(a, device, rank: int = 0, world: int = 1, node: bool = False):
    """Semantic memory co-resident with the engine: `a.memory_rows` rows
    (random unit vectors standing in for an archive of past findings, filled on the device in
    1M-row chunks) plus whatever the agents write back; one MemoryLookupBatcher shared by the
    rank's agents. Single rank: an EnhancedMemory over one HBM index. Node mode (N ranks): ONE
    node-wide store (memory/node_store.py) -- this rank holds its 1/N shard of the rows
    (global row = local row * N + rank), every lookup scans all shards in a lockstep round."""
    import torch

    from pilottai_amd.memory.batcher import MemoryLookupBatcher
    from pilottai_amd.memory.enhanced_memory import EnhancedMemory

    dim = 1024
    fallback = lambda r: f"archived finding {r}: prior document review notes"  # noqa: E731
    rows = a.memory_rows // world + (1 if rank < a.memory_rows % world else 0) if node else a.memory_rows
    cap = rows + 65536  # room for the run's write-backs
    mem = EnhancedMemory(max_size=cap, device=device, dim=dim, fallback_text=fallback,
                         storage=getattr(a, "memory_storage", "q16"))
    idx = mem.index
    idx._grow(cap)
    g = torch.Generator(device=device).manual_seed(7 + rank)
    tags = [idx.tags.bit(t) for t in ("archive", "finance", "ops", "legal")]
    done = 0
    while done < rows:
        m = min(1 << 20, rows - done)
        v = torch.randn(m, dim, device=device, generator=g, dtype=torch.float32)
        pr = torch.randint(0, 3, (m,), device=device, dtype=torch.int32, generator=g)
        tb = (1 << tags[0]) | (1 << torch.randint(1, 4, (m,), device=device, generator=g)).to(torch.int64)
        idx.add_device(v, pr, tb)
        done += m
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    if node:
        import torch.distributed as dist

        from pilottai_amd.memory.node_store import NodeSemanticStore

        # the store's own groups (every rank creates them in this order): device collectives
        # on the job's backend (RCCL), host metadata on gloo
        grp = dist.new_group(backend=dist.get_backend())
        cpu_grp = dist.new_group(backend="gloo") if dist.get_backend() != "gloo" else grp
        mem = NodeSemanticStore(idx, embedder=mem.embedder, group=grp, cpu_group=cpu_grp, fallback_text=fallback)
        mem.start()
    return mem, MemoryLookupBatcher(mem, min_batch=a.memory_min_batch, max_wait_s=a.memory_wait_ms / 1000.0)


def tp_selftest(tp, device, reps: int = 20) -> dict:
    """Start-up check of a TP group's all-reduce (bench --tp): a correctness round trip (every
    rank contributes rank-dependent values, the sum is known in closed form) and the measured
    latency of the two message sizes the cost model needs -- a 64-row decode step's o / down
    output (64 x 4,096 bf16) and a 2,048-token step's (2,048 x 4,096) -- in microseconds, max
    over the group. Collective over the TP group (all its ranks call it)."""
    import torch

    out = {"tp": tp.size, "transport": "custom-p2p" if tp.custom is not None else "process-group"}
    rows = (64, 2048)
    for n in rows:
        t = torch.full((n, 4096), float(tp.rank + 1), dtype=torch.bfloat16, device=device)
        tp.all_reduce(t)
        want = tp.size * (tp.size + 1) / 2
        ok = bool((t.float() == want).all())
        times = []
        for _ in range(reps):
            if device.type == "cuda":
                torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            tp.all_reduce(t)
            if device.type == "cuda":
                torch.cuda.synchronize(device)
            times.append(time.perf_counter() - t0)
        times.sort()
        out[f"ok_{n}x4096"] = ok
        out[f"us_{n}x4096"] = round(1e6 * times[len(times) // 2], 1)
    import torch.distributed as dist

    if tp.size > 1 and dist.is_initialized():  # the group's worst rank
        v = torch.tensor([out[f"us_{n}x4096"] for n in rows] + [0.0 if all(out[f"ok_{n}x4096"] for n in rows)
                                                               else 1.0], dtype=torch.float64)
        dist.all_reduce(v, op=dist.ReduceOp.MAX, group=tp.cpu_group)
        for i, n in enumerate(rows):
            out[f"us_{n}x4096"] = float(v[i])
        out["ok"] = v[-1].item() == 0.0
    return out


def _launch_ranks(n: int) -> int:
    """`bench.py --gpus N` (N > 1) started without a launcher: run N rank processes under
    torch.distributed.run as a CHILD process (nothing here has touched the GPU; never exec)
    and return its exit code, so the run can never silently measure one rank."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    print(f"[bench] --gpus {n} without a launcher: starting {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_launch_ranks(a.gpus))
    import torch

    from pilottai_amd.parallel import comm

    if a.share_gpu:  # RCCL refuses two ranks on one device: the rehearsal's collectives use gloo
        os.environ.setdefault("PILOTTAI_DIST_BACKEND", "gloo")
    rank, world, local_rank = comm.init_distributed()
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    if a.hybrid_latency > 0 and rank > 0:
        device = torch.device("cpu")  # hybrid rehearsal: worker ranks never touch the GPU
    elif a.cpu or not torch.cuda.is_available():
        device = torch.device("cpu")
        a.cpu = True
    else:
        dev_idx = 0 if a.share_gpu else local_rank
        torch.cuda.set_device(dev_idx)
        device = torch.device("cuda", dev_idx)
    tp = dp_group = None
    if a.tp > 1:
        if world % a.tp:
            raise SystemExit(f"--tp {a.tp} must divide --gpus {world}")
        # contiguous TP groups (GPUs 0..T-1, T..2T-1, ...: xGMI is all-to-all, any T GPUs are one
        # hop apart); the custom P2P all-reduce also in the share-GPU rehearsal (gloo groups)
        tp = comm.new_tp_groups(a.tp, custom_ar=True if a.share_gpu else None)
        dp_group = comm.new_dp_group(a.tp)
        a._tp_selftest = tp_selftest(tp, device)
        if not a._tp_selftest.get("ok", True):
            raise SystemExit(f"TP all-reduce self-test failed: {a._tp_selftest}")
    res = asyncio.run(run_rank(a, rank, world, device, tp=tp, dp_group=dp_group))
    everyone = [res]
    if world > 1:
        import torch.distributed as dist

        everyone = [None] * world
        dist.all_gather_object(everyone, res)
    gathered = [g for g in everyone if not g.get("follower")]  # one per agent-DP replica
    if rank == 0:
        dt = max(g["dt"] for g in gathered)
        tasks = sum(g["tasks"] for g in gathered)
        lats = sorted(x for g in gathered for x in g["lat"])
        p50 = lats[len(lats) // 2] if lats else 0.0
        p99 = lats[min(len(lats) - 1, int(0.99 * len(lats)))] if lats else 0.0
        tot = lambda k: sum(g[k] for g in gathered)  # noqa: E731
        lat0 = gathered[0]["req_lat"]  # rank 0's request timings (per-GPU engines are alike)
        calls = max(1, tot("calls"))
        value = tasks / dt if dt > 0 else 0.0
        # scale-run evidence: physical GPUs the ranks actually used (a --share-gpu or hybrid
        # rehearsal of N ranks on one card reports n_gpus 1), the process group RCCL / gloo saw
        phys = sorted({g["device"]["physical"] for g in everyone if g["device"]["physical"]})
        rehearsal = "hybrid" if a.hybrid_latency > 0 else ("share-gpu" if a.share_gpu and world > 1 else None)
        import torch.distributed as dist

        dist_backend = str(dist.get_backend()) if dist.is_initialized() else None
        dist_world = dist.get_world_size() if dist.is_initialized() else 1
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "tasks/s",
            "n_gpus": len(phys),
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000.0 * dt / max(1, a.steps), 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic document tasks, random-init weights",
            "config": {
                "model": "llama-3-8b" if not a.cpu else "tiny(cpu-smoke)",
                "global_batch": a.workers,
                "seq_len": round(tot("prompt_tokens") / calls, 1),
                "parallelism": f"agent-dp{len(gathered)}" + (f"-tp{a.tp}" if a.tp > 1 else ""),
                "managers": tot("managers"),
                "workers": a.workers,
                "llm_calls_per_task": round(calls / max(1, tasks), 2),
                "policy": "fixed",
            },
            "p50_task_latency_ms": round(1000 * p50, 1),
            "p99_task_latency_ms": round(1000 * p99, 1),
            "tasks": tasks,
            "seconds": round(dt, 3),
            "llm_calls": calls,
            "prompt_tokens_per_call": round(tot("prompt_tokens") / calls, 1),
            "output_tokens_per_call": round(tot("completion_tokens") / calls, 1),
            "sampled_tokens_per_call": round(tot("sampled") / calls, 1),
            "engine_tokens_per_s": round(tot("tokens") / dt, 1),
            "engine_steps": tot("steps"),
            "requeued_tasks": tot("requeued"),
            "llm_calls_per_rank": [g["calls"] for g in gathered],
            "engine_busy_frac": round(tot("busy_s") / (dt * len(gathered)), 3),
            "prefix_cache_hit_frac": round(tot("prefix_hit") / max(1, tot("prompt_total")), 3),
            "prefix_defers": tot("prefix_defers"),
            "async_steps": bool(gathered[0].get("async_steps")),
            "spec_rows": tot("spec_rows"),
            "spec_voided": tot("spec_voided"),
            "graph_pad_frac": round(1 - tot("tokens") / max(1, tot("bucket_tokens")), 3),
            # hipGraphs captured on first use inside the timed region (top-k/top-p or
            # embedding variants of a bucket; each one stalls the engine for tens of ms)
            "graph_captures_timed": tot("graph_captures"),
            # rank 0's engine thread, ms per step: schedule / copy+launch / wait for the device /
            # commit / deliver (the host phases are the device's idle time between steps)
            "step_phase_ms": {(k[:-2] if k.endswith("_s") else k): round(1000 * v / max(1, gathered[0]["steps"]), 3)
                              for k, v in gathered[0]["host_phases"].items()},
            "ttft_p50_ms": round(lat0.get("ttft_p50_ms") or 0.0, 1),
            "tpot_p50_ms": round(lat0.get("tpot_p50_ms") or 0.0, 2),
            "init_s": round(max(g["init_s"] for g in gathered), 1),
            "hbm_used_gb_per_gpu": round(max(g["hbm_used_gb"] for g in gathered), 1),
            # the weights are ONE packed copy (models/llama.py keep_dense); the KV pool takes a
            # share of what is left, so the total above does not show the freed copy
            "weights_gb_per_gpu": round(max(g.get("weights_gb", 0.0) for g in gathered), 1),
            "kv_cache_gb_per_gpu": round(max(g.get("kv_cache_gb", 0.0) for g in gathered), 1),
            # rank 0's engine steps per graph bucket: [steps, ms per step]
            "step_buckets": {str(b): [v[0], round(1000 * v[1] / max(1, v[0]), 2)]
                             for b, v in sorted(gathered[0]["buckets"].items()) if v[0] > 0},
            "reply_tokens": a.reply_tokens,
            # rank 0's event loop (manager, plane server, clients, engine deliveries): lag of a
            # 10 ms sleep over the timed region
            "loop_lag_ms": {q: round(1000 * lag[min(len(lag) - 1, int(f * len(lag)))], 2) if lag else None
                            for q, f, lag in (("p50", 0.5, gathered[0]["loop_lag"]),
                                              ("p99", 0.99, gathered[0]["loop_lag"]))},
            "executions_by_rank": gathered[0]["executions_by_rank"],
            "hybrid_latency_s": a.hybrid_latency or None,
            "rehearsal": rehearsal,
            "dist_backend": dist_backend,
            "world_size": dist_world,
            "devices": [g["device"]["device"] for g in everyone],
            "physical_devices": phys,
            "memory": (dict(gathered[0]["memory"], rows_per_rank=[g.get("mem_rows", 0) for g in gathered],
                            rows_total=sum(g.get("mem_rows", 0) for g in gathered))
                       if gathered[0]["memory"] else None),
            "node_load": gathered[0]["node_load"],
            # bench --tp: the start-up all-reduce check and latencies (BENCHMARKS.md, DP x TP cost model)
            "tp_selftest": getattr(a, "_tp_selftest", None),
            "notes": "BASELINE.md publishes no number for this config (vs_baseline null); the reference's "
                     "structural bound with a remote LLM is ~0.8 tasks/s per LLMHandler (BASELINE.md §2).",
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

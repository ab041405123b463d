#!/usr/bin/env python3
"""BASELINE config 5: hierarchical extract -> analyze -> summarize workflow on
Llama-3-70B, with delegation and the fault-tolerance path exercised.

    python benchmarks/workflow.py                         # 1 GPU, TP=1 (70B bf16 = 141 GB fits 288 GB)
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        benchmarks/workflow.py                            # TP=8 over xGMI (rank 0 drives, ranks 1-7 follow)
    python benchmarks/workflow.py --cpu                   # tiny model, plumbing check

Per workflow: Serve -> WorkflowManager, which delegates (TaskDelegator) each
stage to the best live replica (pilottai_amd/workflows/document.py); 3 structured
LLM calls per workflow sharing the document's KV through the prefix cache.
Fault injection: after a third of the timed workflows, one "analyze" replica is
crashed; FaultTolerance detects the missing heartbeat and replaces it, and the
in-flight stage is re-delegated. Synthetic documents, random-init weights.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bench import synth_document  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-70b")
    ap.add_argument("--clients", type=int, default=16)
    ap.add_argument("--workflows", type=int, default=48, help="timed workflows (total)")
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--replicas", type=int, default=2)
    ap.add_argument("--doc-words", type=int, default=300)
    ap.add_argument("--kv-gb", type=float, default=40.0)
    ap.add_argument("--no-fault", action="store_true")
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--max-batched-tokens", type=int, default=2048)
    ap.add_argument("--no-graphs", action="store_true", help="eager steps")
    ap.add_argument("--library", action="store_true", help="row-major weights on library GEMMs (no packing)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="1-GPU rehearsal of TP=N: every rank on GPU 0, gloo control plane "
                         "(PILOTTAI_DIST_BACKEND=gloo), TP all-reduces through the custom P2P kernel")
    return ap.parse_args()


async def drive(a, engine):
    from pilottai_amd.core.config import LLMConfig
    from pilottai_amd.engine.local_llm import LocalLLM
    from pilottai_amd.orchestration.fault_tolerance import FaultTolerance
    from pilottai_amd.serve import Serve
    from pilottai_amd.workflows import build_document_workflow

    llm = LocalLLM(LLMConfig(model_name=engine.model_cfg.name, temperature=0.7, max_tokens=512,
                             retry_attempts=1), engine=engine)
    mgr, kids = await build_document_workflow(llm, a.replicas)
    serve = Serve(agents=[mgr], config={"name": "workflow", "max_concurrent_tasks": a.clients,
                                        "analyze_tasks": False, "evaluate_results": False,
                                        "task_timeout": 1800, "max_queue_size": 100000})
    await serve.start()
    ft = FaultTolerance(mgr, {"health_check_interval": 0.5, "heartbeat_timeout": 2.0,
                              "resource_threshold": 1.0, "recovery_cooldown": 1.0})
    await ft.start()
    rng = random.Random(7)
    docs = [synth_document(rng, a.doc_words) for _ in range(64)]
    lat, failed = [], []
    done = {"n": 0}
    fault = {"at": a.workflows // 3, "done": a.no_fault}

    async def client(ci, n, rec):
        for j in range(n):
            doc = docs[(ci * 7 + j) % len(docs)] + f" (ref {ci}-{j})"
            t0 = time.perf_counter()
            r = await serve.execute_task({"type": "document_workflow", "document": doc,
                                          "description": f"Summarize the document: {doc}"})
            if rec:
                lat.append(time.perf_counter() - t0)
                done["n"] += 1
                if not r.success:
                    failed.append(r.error)
                if not fault["done"] and done["n"] >= fault["at"]:
                    fault["done"] = True
                    victim = next(k for k in mgr.child_agents.values() if getattr(k, "stage", "") == "analyze")
                    fault["victim"] = victim.id
                    await victim.stop()  # crash: heartbeat fails, in-flight stage fails and is re-delegated

    async def round_(total, rec):
        per = [total // a.clients + (1 if i < total % a.clients else 0) for i in range(a.clients)]
        await asyncio.gather(*(client(i, per[i], rec) for i in range(a.clients)))

    async def progress():  # long rehearsals must show life (one line per 30 s)
        while True:
            await asyncio.sleep(30)
            print(f"[workflow] done={done['n']} engine_steps={engine.stats['steps']}", file=sys.stderr, flush=True)

    prog = asyncio.ensure_future(progress())
    await round_(a.warmup, False)
    st0, u0 = dict(engine.stats), dict(llm.usage)
    t0 = time.perf_counter()
    await round_(a.workflows, True)
    dt = time.perf_counter() - t0
    st1, u1 = dict(engine.stats), dict(llm.usage)
    prog.cancel()
    await asyncio.sleep(1.5)  # let FaultTolerance finish a replacement started at the very end
    ftm = ft.get_health_metrics()
    await ft.stop()
    await mgr.delegator.stop()
    await serve.stop()
    lat.sort()
    n = len(lat)
    calls = u1["calls"] - u0["calls"]
    return {
        "metric": "hierarchical extract->analyze->summarize workflows/s (delegation + fault tolerance)",
        "value": round(n / dt, 3), "unit": "workflows/s", "n_gpus": (1 if a.share_gpu else engine.tp.size) if not a.cpu else 0,
        "rehearsal": "share-gpu" if a.share_gpu else None,
        "higher_is_better": True, "dtype": "bf16", "data": "synthetic documents, random-init weights",
        "config": {"model": engine.model_cfg.name if not a.cpu else "tiny(cpu-smoke)",
                   "parallelism": f"tp{engine.tp.size}", "clients": a.clients, "replicas_per_stage": a.replicas,
                   "doc_words": a.doc_words},
        "workflows": n, "failed": len(failed), "seconds": round(dt, 3),
        "p50_latency_ms": round(1000 * lat[n // 2], 1) if n else None,
        "p99_latency_ms": round(1000 * lat[min(n - 1, int(0.99 * n))], 1) if n else None,
        "llm_calls_per_workflow": round(calls / max(1, n), 2),
        "prompt_tokens_per_call": round((u1["prompt_tokens"] - u0["prompt_tokens"]) / max(1, calls), 1),
        "engine_tokens_per_s": round((st1["tokens"] - st0["tokens"]) / dt, 1),
        "prefix_cache_hit_frac": round(engine.metrics()["prefix_cache_hit_tokens"]
                                       / max(1, engine.metrics()["prompt_tokens"]), 3),
        "fault_injected": fault.get("victim") is not None, "ft_replacements": ftm["replacements"],
        "ft_recoveries": ftm["recoveries"], "stage_redelegations": mgr.stage_failures,
        "errors": failed[:3],
    }


def main():
    a = parse()
    import torch

    from pilottai_amd.engine.engine import EngineConfig, LLMEngine
    from pilottai_amd.parallel import comm

    rank, world, local = comm.init_distributed()
    # every TP collective of a step (activations up to 2,048 x 8,192 bf16, sampling winners,
    # top-k / top-p histograms) runs on the custom P2P buffers, so the step graphs capture the
    # TP=2 shared-GPU rehearsal too; --no-graphs keeps the eager steps
    tp = comm.new_tp_groups(world, custom_ar=True if a.share_gpu else None)
    if a.cpu or not torch.cuda.is_available():
        a.cpu = True
        device = torch.device("cpu")
        model = "tiny" if world == 1 else "tiny-gqa4"  # TP needs heads divisible by the TP size
    else:
        dev_idx = 0 if a.share_gpu else local
        torch.cuda.set_device(dev_idx)
        device = torch.device("cuda", dev_idx)
        model = a.model
    t0 = time.time()
    mbt = a.max_batched_tokens
    buckets = [b for b in (8, 16, 32, 64, 128, 256, 512, 768, 1024, 1536, 2048) if b < mbt] + [mbt]
    eng = LLMEngine(EngineConfig(model=model, max_num_seqs=max(64, 4 * a.clients), max_num_batched_tokens=mbt,
                                 kv_cache_gb=None if a.cpu else a.kv_gb, num_kv_blocks=4096 if a.cpu else None,
                                 token_buckets=buckets, use_graphs=not a.no_graphs,
                                 # one packed copy per rank (the row-major one is freed): 8 ranks x
                                 # 17.6 GB fit one card on the hand kernels; --library keeps the
                                 # row-major weights on hipBLASLt instead
                                 decode_fused=False if a.library else None),
                    device=device, tp=tp)
    init_s = time.time() - t0
    if tp.rank != 0:
        eng.follow()
    else:
        eng.start()
        try:
            out = asyncio.run(drive(a, eng))
        finally:
            eng.stop()  # also releases the follower ranks
        out["init_s"] = round(init_s, 1)
        out["graphs"] = {"use_graphs": eng.use_graphs, "captured": len(eng._graphs),
                         "replays": eng.stats.get("graph_replays", 0), "tp": tp.size,
                         "custom_collective_calls": tp.custom.calls if getattr(tp, "custom", None) else None}
        if eng.on_gpu:
            out["hbm_used_gb_per_gpu"] = round(torch.cuda.max_memory_allocated(device) / 2**30, 1)
        print(json.dumps(out), flush=True)
    if world > 1:
        comm.barrier()


if __name__ == "__main__":
    main()

"""Shared-context broadcast across 2 agent-DP ranks over gloo: rank 0's
context reaches rank 1 as token ids, both engines pre-warm it into the prefix
cache, and later agent prompts start with it (cache hits on every rank)."""
import json
import os
import socket

import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import asyncio

    import torch

    torch.set_num_threads(2)
    from pilottai_amd.core.agent import BaseAgent
    from pilottai_amd.core.config import AgentConfig, LLMConfig
    from pilottai_amd.engine.engine import EngineConfig, LLMEngine
    from pilottai_amd.engine.local_llm import LocalLLM
    from pilottai_amd.parallel.comm import init_distributed
    from pilottai_amd.serve import Serve

    init_distributed("gloo")
    eng = LLMEngine(EngineConfig(model="tiny", max_num_seqs=8, max_num_batched_tokens=256, max_model_len=1024,
                                 num_kv_blocks=256, use_graphs=False), device="cpu")
    llm = LocalLLM(LLMConfig(model_name="tiny", max_tokens=64), engine=eng)

    async def main():
        serve = Serve(agents=[BaseAgent(AgentConfig(role="w", goal="g"), llm=llm)], manager_llm=llm,
                      config={"policy": "fixed"})
        ctx = ("Company handbook: all agents summarise documents for the finance team, "
               "cite figures exactly, and flag risks. " * 4) if rank == 0 else None
        info = await serve.broadcast_context(ctx)
        cached0 = eng.metrics()["cached_kv_blocks"]
        r = await llm.apredict("Task: say ok", response_format={"schema": "orchestrator.result_evaluation"})
        return info, llm.shared_context, cached0, eng.metrics()["prefix_cache_hit_tokens"], r

    info, shared, cached0, hits, r = asyncio.run(main())
    torch.distributed.destroy_process_group()
    with open(f"{out}.{rank}", "w") as f:
        json.dump({"info": info, "shared": shared, "cached": cached0, "hits": hits, "reply": r}, f)


def test_broadcast_context_two_ranks(tmp_path):
    out = str(tmp_path / "ctx")
    mp.start_processes(_worker, args=(2, _port(), out), nprocs=2, join=True, start_method="spawn")
    res = [json.load(open(f"{out}.{r}")) for r in range(2)]
    assert res[0]["shared"] == res[1]["shared"] and res[1]["shared"].startswith("Company handbook")
    for r in res:
        assert r["info"]["tokens"] > 50 and r["info"]["prewarmed_engines"] == 1
        assert r["cached"] >= 3          # context blocks registered in the prefix cache
        assert r["hits"] >= 48           # the next prompt reused them
        json.loads(r["reply"])

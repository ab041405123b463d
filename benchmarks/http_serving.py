#!/usr/bin/env python3
"""HTTP serving throughput: C concurrent OpenAI-API clients against the engine on one GPU.

    python benchmarks/http_serving.py [--clients 64 --requests 4 --max-tokens 64]
    python benchmarks/http_serving.py --cpu          # tiny model, plumbing check

The server (pilottai_amd.serving.http_server) runs in this process on a uvicorn thread
with Llama-3-8B (random-init weights) on the GPU. Every client sends `--requests`
chat completions back to back: a synthetic ~`--prompt-words`-word document, a
structured reply constrained by the `orchestrator.result_evaluation` schema
(`--schema`) or `--max-tokens` of free text. Prints one JSON line: requests/s,
completion tokens/s, p50/p99 request latency, and the engine's own counters.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import socket
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bench import synth_document  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--requests", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--max-tokens", type=int, default=64)
    ap.add_argument("--prompt-words", type=int, default=300)
    ap.add_argument("--schema", action="store_true")
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--cpu", action="store_true")
    a = ap.parse_args()

    import httpx
    import torch
    import uvicorn

    from pilottai_amd.core.config import LLMConfig
    from pilottai_amd.engine.engine import EngineConfig, LLMEngine
    from pilottai_amd.engine.local_llm import LocalLLM
    from pilottai_amd.serving.http_server import create_app

    cpu = a.cpu or not torch.cuda.is_available()
    dev = torch.device("cpu") if cpu else torch.device("cuda", 0)
    eng = LLMEngine(EngineConfig(model="tiny" if cpu else a.model, max_num_seqs=max(64, 2 * a.clients),
                                 kv_cache_gb=None if cpu else 48.0, num_kv_blocks=2048 if cpu else None,
                                 use_graphs=not cpu), device=dev)
    eng.start()
    llm = LocalLLM(LLMConfig(model_name=eng.model_cfg.name, max_tokens=a.max_tokens, temperature=0.7), engine=eng)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    server = uvicorn.Server(uvicorn.Config(create_app(llm, eng.model_cfg.name, engine=eng), host="127.0.0.1",
                                           port=port, log_level="error"))
    th = threading.Thread(target=server.run, daemon=True)
    th.start()
    while not server.started:
        time.sleep(0.05)
    url = f"http://127.0.0.1:{port}/v1/chat/completions"

    async def run(n_req: int, record: list):
        limits = httpx.Limits(max_connections=a.clients + 8, max_keepalive_connections=a.clients + 8)
        async with httpx.AsyncClient(timeout=600, limits=limits) as c:
            async def client(ci: int):
                rng = random.Random(ci * 7919 + n_req)
                for _ in range(n_req):
                    body = {"model": eng.model_cfg.name, "max_tokens": a.max_tokens,
                            "messages": [{"role": "user", "content": "Evaluate this report: "
                                          + synth_document(rng, a.prompt_words)}]}
                    if a.schema:
                        body["response_format"] = {"type": "pilottai_schema",
                                                   "schema": "orchestrator.result_evaluation"}
                    t0 = time.perf_counter()
                    r = await c.post(url, json=body)
                    r.raise_for_status()
                    record.append((time.perf_counter() - t0, r.json()["usage"]["completion_tokens"]))

            await asyncio.gather(*(client(i) for i in range(a.clients)))

    if a.warmup:
        asyncio.run(run(a.warmup, []))
    st0 = dict(eng.stats)
    rec: list = []
    t0 = time.perf_counter()
    asyncio.run(run(a.requests, rec))
    dt = time.perf_counter() - t0
    st1 = dict(eng.stats)
    lat = sorted(x for x, _ in rec)
    out = {
        "metric": "HTTP chat completions/s", "value": round(len(rec) / dt, 2), "unit": "requests/s",
        "model": eng.model_cfg.name, "device": str(dev), "clients": a.clients, "requests": len(rec),
        "completion_tokens_per_s": round(sum(n for _, n in rec) / dt, 1),
        "p50_latency_ms": round(1000 * lat[len(lat) // 2], 1),
        "p99_latency_ms": round(1000 * lat[min(len(lat) - 1, int(0.99 * len(lat)))], 1),
        "engine_steps": st1["steps"] - st0["steps"], "engine_tokens": st1["tokens"] - st0["tokens"],
        "schema": a.schema, "max_tokens": a.max_tokens, "prompt_words": a.prompt_words,
        "data": "synthetic documents, random-init weights",
    }
    print(json.dumps(out), flush=True)
    server.should_exit = True
    th.join(timeout=10)
    eng.stop()


if __name__ == "__main__":
    main()

"""OpenAI-compatible HTTP front end for the on-node engine.

The reference reaches its model over HTTPS through litellm (`pilott/engine/llm.py:59`,
SURVEY C14); here the model runs on the MI355X in the same process, and this module
publishes it to other processes and hosts with the wire format those clients already
speak:

    GET  /                     landing page with live engine metrics (serving/site.py)
    GET  /health               liveness + engine metrics (steps, tokens/s, KV use, HBM)
    GET  /v1/models            the served model
    POST /v1/chat/completions  messages -> one completion (stream=true: SSE, one delta + [DONE])

`response_format` accepts the OpenAI forms and one extension:
* {"type": "json_schema", "json_schema": {"name": ..., "schema": {...}}}: a JSON Schema
  subset (objects, strings with maxLength or enum, bounded integers, booleans, arrays of
  strings or objects) compiled to the engine's token grammar, so the reply parses;
* {"type": "pilottai_schema", "schema": "agent.task_analysis", "fixed": {...}}: a schema
  of source/rules.yaml by name, with pinned fields. This is what
  `engine/http_llm.OpenAICompatLLM` sends, so agents on another host run the same
  constrained protocol as agents in-process.
`tools` (OpenAI function tools) produce a constrained `{"name", "arguments"}` call,
returned as `tool_calls`.

Every request becomes one `LocalLLM` call, i.e. one sequence in the engine's continuous
batch. Concurrent HTTP clients share the engine's steps exactly like in-process agents.

    python -m pilottai_amd.serving.http_server --model llama-3-8b --port 8000   # MI355X
    python -m pilottai_amd.serving.http_server --schema --port 8000             # model-free
"""
from __future__ import annotations

import argparse
import json
import time
import uuid
from typing import Any, Dict, List, Optional

from fastapi import FastAPI, HTTPException
from fastapi.responses import HTMLResponse, JSONResponse, StreamingResponse

DEFAULT_STR_TOKENS = 32


def json_schema_to_spec(js: Dict[str, Any], path: str = "") -> Any:
    """Convert a JSON Schema subset to the rules.yaml schema language (engine/grammar.py)."""
    if not isinstance(js, dict):
        raise ValueError(f"schema at {path or '<root>'} must be an object")
    t = js.get("type")
    if "enum" in js:
        vals = [str(v) for v in js["enum"]]
        if not vals or any("|" in v for v in vals):
            raise ValueError(f"unsupported enum at {path or '<root>'}")
        return "enum(" + "|".join(vals) + ")"
    if t == "object":
        props = js.get("properties")
        if props:
            return {k: json_schema_to_spec(v, f"{path}.{k}" if path else k) for k, v in props.items()}
        add = js.get("additionalProperties")
        if isinstance(add, dict) and add.get("type") == "string":
            return f"map(str({_str_tokens(add)}))"
        return "obj()"
    if t == "string":
        return f"str({_str_tokens(js)})"
    if t == "boolean":
        return "bool"
    if t == "integer":
        lo, hi = int(js.get("minimum", 0)), int(js.get("maximum", 100))
        if hi < lo or hi - lo > 1000:
            raise ValueError(f"integer range at {path or '<root>'} must span at most 1000 values")
        return f"int({lo},{hi})"
    if t == "array":
        item = js.get("items") or {"type": "string"}
        mn = int(js.get("minItems", 1))
        mx = int(js.get("maxItems", max(mn, 4)))
        if item.get("type") == "object":
            return {"objlist": max(1, mn), "item": json_schema_to_spec(item, f"{path}[]")}
        if item.get("type", "string") != "string":
            raise ValueError(f"arrays at {path or '<root>'} must hold strings or objects")
        return f"list(str({_str_tokens(item)}),{mn},{mx})"
    raise ValueError(f"unsupported schema type {t!r} at {path or '<root>'}")


def _str_tokens(js: Dict[str, Any]) -> int:
    n = js.get("maxLength")
    return max(1, int(n) // 4) if n else DEFAULT_STR_TOKENS


def _response_format(body: Dict[str, Any]) -> Optional[Dict[str, Any]]:
    rf = body.get("response_format")
    out: Dict[str, Any] = {}
    for k in ("temperature", "top_p", "top_k", "seed"):
        if body.get(k) is not None:
            out[k] = body[k]
    if not rf:
        return out or None
    kind = rf.get("type")
    if kind == "pilottai_schema":
        out.update(schema=rf["schema"], fixed=rf.get("fixed") or {})
    elif kind == "json_schema":
        js = (rf.get("json_schema") or {}).get("schema")
        if js is None:
            raise ValueError("json_schema.schema is required")
        out.update(schema=json_schema_to_spec(js), fixed={})
    elif kind == "text":
        pass
    else:
        raise ValueError(f"unsupported response_format type {kind!r}")
    return out


def _tools(body: Dict[str, Any]) -> Optional[List[Dict[str, Any]]]:
    tools = body.get("tools")
    if not tools:
        return None
    out = []
    for t in tools:
        f = t.get("function", t)
        out.append({"name": f["name"], "description": f.get("description", ""),
                    "parameters": f.get("parameters", {})})
    return out


def create_app(llm, model_name: Optional[str] = None, engine=None) -> FastAPI:
    """FastAPI app serving `llm` (a BaseLLM: LocalLLM on the GPU, SchemaLLM model-free)."""
    app = FastAPI(title="pilottai_amd", version="0.1.0")
    name = model_name or getattr(llm, "model_name", "local")
    started = time.time()

    @app.get("/", response_class=HTMLResponse)
    async def index():
        from pilottai_amd.serving.site import render

        return render(name)

    @app.get("/health")
    async def health():
        out = {"status": "ok", "model": name, "uptime_s": round(time.time() - started, 1),
               "usage": dict(getattr(llm, "usage", {}))}
        eng = engine or getattr(llm, "engine", None)
        if eng is not None:
            if getattr(eng, "failed", None) is not None:
                return JSONResponse({"status": "failed", "error": str(eng.failed)}, status_code=503)
            out["engine"] = eng.metrics()
        return out

    @app.get("/v1/models")
    async def models():
        return {"object": "list", "data": [{"id": name, "object": "model", "owned_by": "pilottai_amd"}]}

    @app.post("/v1/chat/completions")
    async def chat(body: Dict[str, Any]):
        messages = body.get("messages")
        if not messages:
            raise HTTPException(400, "messages must be a non-empty list")
        try:
            rf = _response_format(body)
            tools = _tools(body)
        except (KeyError, ValueError) as e:
            raise HTTPException(400, str(e))
        mt = body.get("max_tokens") or body.get("max_completion_tokens")
        if mt:
            rf = dict(rf or {}, max_tokens=int(mt))  # per request: the shared llm object is not mutated
        try:
            r = await llm.generate_response(messages, tools=tools, response_format=rf)
        except Exception as e:  # noqa: BLE001
            raise HTTPException(500, f"generation failed: {e}")
        cid = "chatcmpl-" + uuid.uuid4().hex[:24]
        created = int(time.time())
        finish = "tool_calls" if r.get("tool_calls") else "stop"
        msg = {"role": "assistant", "content": r["content"]}
        if r.get("tool_calls"):
            msg["tool_calls"] = r["tool_calls"]
        usage = r.get("usage", {})
        if not body.get("stream"):
            return {"id": cid, "object": "chat.completion", "created": created, "model": name,
                    "choices": [{"index": 0, "message": msg, "finish_reason": finish}], "usage": usage}

        def sse():
            first = {"id": cid, "object": "chat.completion.chunk", "created": created, "model": name,
                     "choices": [{"index": 0, "delta": msg, "finish_reason": None}]}
            last = {"id": cid, "object": "chat.completion.chunk", "created": created, "model": name,
                    "choices": [{"index": 0, "delta": {}, "finish_reason": finish}], "usage": usage}
            yield f"data: {json.dumps(first)}\n\n"
            yield f"data: {json.dumps(last)}\n\n"
            yield "data: [DONE]\n\n"

        return StreamingResponse(sse(), media_type="text/event-stream")

    return app


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--schema", action="store_true", help="model-free SchemaLLM backend (no GPU)")
    ap.add_argument("--kv-gb", type=float, default=48.0)
    a = ap.parse_args()
    import uvicorn

    from pilottai_amd.core.config import LLMConfig
    from pilottai_amd.engine.local_llm import LocalLLM, SchemaLLM

    if a.schema:
        llm = SchemaLLM(LLMConfig(model_name=a.model, provider="schema"))
        app = create_app(llm, a.model)
    else:
        import torch

        from pilottai_amd.engine.engine import EngineConfig, LLMEngine

        dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
        eng = LLMEngine(EngineConfig(model=a.model if dev.type == "cuda" else "tiny",
                                     kv_cache_gb=a.kv_gb if dev.type == "cuda" else None,
                                     num_kv_blocks=None if dev.type == "cuda" else 1024,
                                     freeze_heap=True), device=dev)
        eng.start()
        llm = LocalLLM(LLMConfig(model_name=eng.model_cfg.name, max_tokens=1024), engine=eng)
        app = create_app(llm, eng.model_cfg.name, engine=eng)
    uvicorn.run(app, host=a.host, port=a.port, log_level="warning")


if __name__ == "__main__":
    main()

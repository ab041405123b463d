"""OpenAI-compatible HTTP serving (serving/http_server.py) and the HTTP LLM client
(engine/http_llm.py) on CPU: the model-free SchemaLLM backend for the protocol, and
the tiny engine for real grammar-constrained generation through HTTP, with agents
running their full structured protocol against the remote endpoint."""
import asyncio
import json
import socket
import threading
import time

import httpx
import pytest
import uvicorn

from pilottai_amd.core.agent import BaseAgent
from pilottai_amd.core.config import AgentConfig, LLMConfig
from pilottai_amd.core.policy import ControlPolicy
from pilottai_amd.core.task import Task
from pilottai_amd.engine.local_llm import SchemaLLM, make_llm
from pilottai_amd.serving.http_server import create_app, json_schema_to_spec
from pilottai_amd.tools.tool import Tool, echo_tool


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Server:
    def __init__(self, app):
        self.port = _port()
        self.server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=self.port, log_level="error"))
        self.thread = threading.Thread(target=self.server.run, daemon=True)

    def __enter__(self):
        self.thread.start()
        t0 = time.time()
        while not self.server.started:
            assert time.time() - t0 < 30, "server did not start"
            time.sleep(0.05)
        return f"http://127.0.0.1:{self.port}/v1"

    def __exit__(self, *exc):
        self.server.should_exit = True
        self.thread.join(timeout=10)


@pytest.fixture(scope="module")
def schema_server():
    with _Server(create_app(SchemaLLM(seed=5), "schema-test")) as url:
        yield url


def _client(url):
    return make_llm(LLMConfig(provider="openai", base_url=url, model_name="schema-test", retry_attempts=1))


async def test_models_health_and_structured_reply(schema_server):
    llm = _client(schema_server)
    assert await llm.list_models() == ["schema-test"]
    r = await llm.generate_response([{"role": "user", "content": "analyse"}],
                                    response_format={"schema": "agent.task_analysis", "fixed": {"can_execute": True}})
    obj = json.loads(r["content"])
    assert obj["can_execute"] is True and "execution_plan" in obj
    assert r["usage"]["prompt_tokens"] > 0 and llm.usage["calls"] == 1
    async with httpx.AsyncClient() as c:
        h = (await c.get(schema_server.replace("/v1", "/health"))).json()
    assert h["status"] == "ok" and h["usage"]["calls"] >= 1
    await llm.aclose()


async def test_tool_calls_json_schema_stream_and_errors(schema_server):
    llm = _client(schema_server)
    r = await llm.apredict_messages([{"role": "user", "content": "use a tool"}],
                                    [{"name": "search", "description": "web", "parameters": {}}])
    assert r["tool_calls"][0]["function"]["name"] == "search"
    js = {"type": "object", "properties": {"ok": {"type": "boolean"}, "mood": {"enum": ["good", "bad"]},
                                           "tags": {"type": "array", "items": {"type": "string"}, "maxItems": 2},
                                           "score": {"type": "integer", "minimum": 1, "maximum": 5}}}
    async with httpx.AsyncClient() as c:
        body = {"model": "x", "messages": [{"role": "user", "content": "hi"}],
                "response_format": {"type": "json_schema", "json_schema": {"name": "t", "schema": js}}}
        out = (await c.post(f"{schema_server}/chat/completions", json=body)).json()
        obj = json.loads(out["choices"][0]["message"]["content"])
        assert set(obj) == {"ok", "mood", "tags", "score"} and obj["mood"] in ("good", "bad")
        assert out["object"] == "chat.completion" and out["choices"][0]["finish_reason"] == "stop"
        bad = await c.post(f"{schema_server}/chat/completions", json={"model": "x", "messages": []})
        assert bad.status_code == 400
        bad = await c.post(f"{schema_server}/chat/completions",
                           json={"model": "x", "messages": [{"role": "user", "content": "hi"}],
                                 "response_format": {"type": "xml"}})
        assert bad.status_code == 400
        body["stream"] = True
        lines = [ln for ln in (await c.post(f"{schema_server}/chat/completions", json=body)).text.split("\n")
                 if ln.startswith("data: ")]
        assert lines[-1] == "data: [DONE]" and json.loads(lines[0][6:])["choices"][0]["delta"]["content"]
    await llm.aclose()


def test_json_schema_subset_conversion():
    spec = json_schema_to_spec({"type": "object", "properties": {
        "a": {"type": "string", "maxLength": 40}, "b": {"type": "array", "items": {"type": "object",
                                                                               "properties": {"x": {"type": "boolean"}}},
                                                     "minItems": 2}}})
    assert spec == {"a": "str(10)", "b": {"objlist": 2, "item": {"x": "bool"}}}
    with pytest.raises(ValueError):
        json_schema_to_spec({"type": "number"})


async def test_agent_runs_its_protocol_over_http(schema_server):
    llm = _client(schema_server)
    a = BaseAgent(AgentConfig(role="remote", goal="g", description="d"), llm=llm,
                  tools=[Tool(name="echo", function=echo_tool, max_retries=1)], policy=ControlPolicy("fixed", 2))
    await a.start()
    r = await a.execute_task(Task(description="summarize", metadata={"tool_inputs": {"q": 1}}))
    assert r.success, r.error
    assert r.output[0]["result"]["output"] == {"echo": {"q": 1}}
    await llm.aclose()


def test_engine_backed_server_concurrent_constrained_requests():
    """The tiny CPU engine behind HTTP: concurrent clients share its continuous batch."""
    from pilottai_amd.engine.engine import EngineConfig, LLMEngine
    from pilottai_amd.engine.local_llm import LocalLLM

    eng = LLMEngine(EngineConfig(model="tiny", max_num_seqs=8, max_num_batched_tokens=256, max_model_len=1024,
                                 num_kv_blocks=256, use_graphs=False), device="cpu")
    eng.start()
    try:
        backend = LocalLLM(LLMConfig(model_name="tiny", max_tokens=96), engine=eng)
        with _Server(create_app(backend, "tiny", engine=eng)) as url:
            async def go():
                llm = make_llm(LLMConfig(provider="openai", base_url=url, model_name="tiny", retry_attempts=1,
                                         timeout=120))
                rs = await asyncio.gather(*(llm.generate_response(
                    [{"role": "user", "content": f"task {i}"}],
                    response_format={"schema": "orchestrator.result_evaluation"}) for i in range(4)))
                h = (await llm._http().get(url.replace("/v1", "/health"))).json()
                await llm.aclose()
                return rs, h

            rs, h = asyncio.run(go())
        for r in rs:
            assert set(json.loads(r["content"])) == {"success", "quality", "requires_retry"}
        assert h["status"] == "ok" and isinstance(h["engine"], dict) and h["engine"]
    finally:
        eng.stop()


def test_landing_page_sections_and_live_metrics(schema_server):
    """GET / serves the framework's page (the reference's Hero / Features /
    Agents / Performance / Footer site) with a Performance section fed by /health."""
    base = schema_server[: -len("/v1")]
    r = httpx.get(base + "/", timeout=10)
    assert r.status_code == 200 and r.headers["content-type"].startswith("text/html")
    for sid in ("navigation", "hero", "features", "agents", "performance", "footer"):
        assert f'id="{sid}"' in r.text
    assert "schema-test" in r.text and "fetch('/health')" in r.text
    h = httpx.get(base + "/health", timeout=10).json()
    assert h["status"] == "ok" and h["model"] == "schema-test"

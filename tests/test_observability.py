"""Metrics endpoint (Prometheus text over HTTP) and the span tracer."""
import asyncio
import json

from pilottai_amd.core.agent import BaseAgent
from pilottai_amd.core.config import AgentConfig, LLMConfig
from pilottai_amd.engine.local_llm import SchemaLLM
from pilottai_amd.serve import Serve
from pilottai_amd.utils.metrics_server import metrics_text, start_metrics_server
from pilottai_amd.utils.tracing import Tracer


def test_metrics_endpoint_serves_prometheus_text():
    async def main():
        llm = SchemaLLM(LLMConfig(provider="schema"))
        serve = Serve(agents=[BaseAgent(AgentConfig(role="w", goal="g"), llm=llm)], manager_llm=llm,
                      config={"policy": "fixed"})
        await serve.execute_task("Task: probe")
        server = await start_metrics_server(serve, port=0)
        port = server.sockets[0].getsockname()[1]
        r, w = await asyncio.open_connection("127.0.0.1", port)
        w.write(b"GET /metrics HTTP/1.1\r\nHost: x\r\n\r\n")
        await w.drain()
        data = (await r.read()).decode()
        w.close()
        server.close()
        await server.wait_closed()
        text = metrics_text(serve)
        await serve.stop()
        return data, text

    data, text = asyncio.run(main())
    assert data.startswith("HTTP/1.1 200")
    assert 'pilottai_completed_tasks{serve="Pilott"} 1' in text
    assert "pilottai_metrics_successful_tasks" in data


def test_tracer_chrome_json(tmp_path):
    t = Tracer()
    with t.span("agent.analyze", task="t1"):
        pass
    with t.span("engine.step"):
        pass
    p = tmp_path / "trace.json"
    t.dump(str(p))
    ev = json.load(open(p))["traceEvents"]
    assert [e["name"] for e in ev] == ["agent.analyze", "engine.step"] and ev[0]["args"]["task"] == "t1"

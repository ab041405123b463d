"""`OpenAICompatLLM`: the reference's LLMHandler contract over an OpenAI-compatible HTTP API.

The reference calls providers over HTTPS through litellm (`pilott/engine/llm.py:59-120`).
Here the same protocol (generate_response / apredict / apredict_messages, with the RPM
limiter, concurrency cap and retries of `BaseLLM`) is spoken to any
`/v1/chat/completions` endpoint — typically `pilottai_amd.serving.http_server` on
another host or in another process, whose GPU engine then batches these calls with
everything else it serves.

Structured replies: agents pass `response_format={"schema": <rules.yaml name>,
"fixed": {...}}`. Against a pilottai server that is forwarded as the
`pilottai_schema` extension (grammar-constrained on the server). Against another
OpenAI-compatible server, pass `schema_mode="json_object"` to send
`{"type": "json_object"}` instead.

    LLMConfig(provider="openai", base_url="http://10.0.0.5:8000/v1", api_key=...)
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional

from .local_llm import BaseLLM, _cfg_get


class OpenAICompatLLM(BaseLLM):
    provider = "openai"

    def __init__(self, config: Any = None, base_url: Optional[str] = None, timeout_s: float = 600.0,
                 schema_mode: str = "pilottai"):
        super().__init__(config)
        self.base_url = (base_url or _cfg_get(config, "base_url", None) or "http://127.0.0.1:8000/v1").rstrip("/")
        key = _cfg_get(config, "api_key", None)
        if key is not None and hasattr(key, "get_secret_value"):
            key = key.get_secret_value()
        self._headers = {"Authorization": f"Bearer {key}"} if key else {}
        self.timeout_s = float(_cfg_get(config, "timeout", timeout_s) or timeout_s)
        self.schema_mode = schema_mode
        self._client = None

    def _http(self):
        import httpx

        if self._client is None:
            self._client = httpx.AsyncClient(timeout=self.timeout_s, headers=self._headers)
        return self._client

    async def aclose(self):
        if self._client is not None:
            await self._client.aclose()
            self._client = None

    def _body(self, messages, response_format, tools) -> Dict[str, Any]:
        rf = dict(response_format or {})
        body: Dict[str, Any] = {"model": self.model_name, "messages": list(messages),
                                "temperature": float(rf.get("temperature", self.temperature)),
                                "top_p": float(rf.get("top_p", self.top_p)),
                                "max_tokens": int(rf.get("max_tokens", self.max_tokens))}
        if rf.get("seed") is not None:
            body["seed"] = rf["seed"]
        if tools:
            body["tools"] = self._format_tools(tools)
        elif rf.get("schema") is not None:
            if self.schema_mode == "pilottai":
                body["response_format"] = {"type": "pilottai_schema", "schema": rf["schema"],
                                           "fixed": rf.get("fixed") or {}}
            else:
                body["response_format"] = {"type": "json_object"}
        return body

    async def _complete(self, messages, response_format, tools) -> Dict[str, Any]:
        r = await self._http().post(f"{self.base_url}/chat/completions",
                                    json=self._body(messages, response_format, tools))
        if r.status_code != 200:
            raise RuntimeError(f"HTTP {r.status_code}: {r.text[:300]}")
        data = r.json()
        ch = data["choices"][0]
        msg = ch.get("message") or {}
        usage = data.get("usage") or {}
        pt, ct = int(usage.get("prompt_tokens", 0)), int(usage.get("completion_tokens", 0))
        return {"content": msg.get("content") or "", "role": msg.get("role", "assistant"),
                "tool_calls": msg.get("tool_calls"), "model": data.get("model", self.model_name),
                "usage": {"prompt_tokens": pt, "completion_tokens": ct, "total_tokens": pt + ct}}

    async def list_models(self) -> List[str]:
        r = await self._http().get(f"{self.base_url}/models")
        r.raise_for_status()
        return [m["id"] for m in r.json().get("data", [])]

"""LLM protocol adapters: the reference's `LLMHandler` contract served on-node.

Reference contract (pilott/engine/llm.py:38-219):
    await generate_response(messages, tools=None) -> {content, role, tool_calls, model, usage}
    await apredict(prompt) -> str
    await apredict_messages(messages, functions) -> dict
with a sliding-window RPM limiter, bounded concurrency and linear-backoff retries.

`LocalLLM` keeps that contract but every call becomes a request in the local
continuous batch (engine/engine.py), so 64 agents' concurrent calls share one
forward per step instead of queueing behind a 5-slot HTTP semaphore. Replies
can be constrained to a schema via `response_format` (source/rules.yaml
`schemas:`); agents and the orchestrator always pass one, so every reply parses.

Task queue on the GPU stream: an agent step's call is
`engine.submit()` -> the engine thread batches it into the next captured step on
the GPU's stream; the completion callback resolves the caller's asyncio future
with `loop.call_soon_threadsafe`, so the orchestrator's event loop never blocks
on the device.

`SchemaLLM` is a model-free implementation of the same protocol that emits
schema-valid JSON directly (used by CPU tests and the plumbing benchmark,
BASELINE config 1).
"""
from __future__ import annotations

import asyncio
import json
import logging
import random
import re
import threading
import time
from collections import deque
from typing import Any, Deque, Dict, List, Optional, Sequence, Union

from .tokenizer import END_HEADER_ID, EOT_ID, START_HEADER_ID, BOS_ID, Tokenizer

log = logging.getLogger("pilottai_amd.llm")


def encode_chat(tok: Tokenizer, messages: Sequence[Dict[str, str]]) -> List[int]:
    """Llama-3 chat layout with the same special-token ids."""
    ids = [BOS_ID]
    for m in messages:
        ids.append(START_HEADER_ID)
        ids += tok.encode(str(m.get("role", "user")))
        ids.append(END_HEADER_ID)
        ids += tok.encode("\n\n" + str(m.get("content", "")))
        ids.append(EOT_ID)
    ids.append(START_HEADER_ID)
    ids += tok.encode("assistant")
    ids.append(END_HEADER_ID)
    ids += tok.encode("\n\n")
    return ids


def _cfg_get(config: Any, key: str, default=None):
    if config is None:
        return default
    if isinstance(config, dict):
        v = config.get(key, default)
    else:
        v = getattr(config, key, default)
    if hasattr(v, "get_secret_value"):
        v = v.get_secret_value()
    return default if v is None else v


class _RateLimiter:
    """Sliding 60 s window limiter (reference llm.py:68-89)."""

    def __init__(self, max_rpm: Optional[int]):
        self.max_rpm = max_rpm
        self.calls: Deque[float] = deque()
        self.lock = asyncio.Lock()

    async def acquire(self):
        if not self.max_rpm:
            return
        async with self.lock:
            now = time.monotonic()
            while self.calls and self.calls[0] <= now - 60.0:
                self.calls.popleft()
            if len(self.calls) >= self.max_rpm:
                await asyncio.sleep(max(0.0, 60.0 - (now - self.calls[0])))
            self.calls.append(time.monotonic())


class BaseLLM:
    """Shared protocol surface (rate limit, retries, response shaping)."""

    provider = "base"

    def __init__(self, config: Any = None):
        self.config = config
        self.model_name = _cfg_get(config, "model_name", "llama-3-8b")
        self.temperature = float(_cfg_get(config, "temperature", 0.7))
        self.top_p = float(_cfg_get(config, "top_p", 1.0))
        self.top_k = int(_cfg_get(config, "top_k", 0))
        self.max_tokens = int(_cfg_get(config, "max_tokens", 2000))
        self.retry_attempts = max(1, int(_cfg_get(config, "retry_attempts", 3)))
        self.retry_delay = float(_cfg_get(config, "retry_delay", 1.0))
        mc = _cfg_get(config, "max_concurrent", None)
        self._sem = asyncio.Semaphore(int(mc)) if mc else None
        self._limiter = _RateLimiter(_cfg_get(config, "max_rpm", None))
        self.usage = {"calls": 0, "prompt_tokens": 0, "completion_tokens": 0}

    async def _complete(self, messages, response_format, tools) -> Dict[str, Any]:
        raise NotImplementedError

    async def _call(self, messages, response_format=None, tools=None) -> Dict[str, Any]:
        if not messages:
            raise ValueError("Messages cannot be empty")
        await self._limiter.acquire()
        last: Optional[BaseException] = None
        for attempt in range(self.retry_attempts):
            try:
                if self._sem:
                    async with self._sem:
                        r = await self._complete(messages, response_format, tools)
                else:
                    r = await self._complete(messages, response_format, tools)
                self.usage["calls"] += 1
                self.usage["prompt_tokens"] += r["usage"]["prompt_tokens"]
                self.usage["completion_tokens"] += r["usage"]["completion_tokens"]
                return r
            except asyncio.CancelledError:
                raise
            except Exception as e:  # noqa: BLE001
                last = e
                if attempt < self.retry_attempts - 1:
                    log.warning("LLM attempt %d failed: %s", attempt + 1, e)
                    await asyncio.sleep(self.retry_delay * (attempt + 1))
        raise RuntimeError(f"LLM call failed after {self.retry_attempts} attempts: {last}")

    # -- reference protocol -------------------------------------------------
    async def generate_response(self, messages: List[Dict[str, str]], tools: Optional[List[Dict]] = None,
                                response_format: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
        return await self._call(messages, response_format, tools)

    async def apredict(self, prompt: str, response_format: Optional[Dict[str, Any]] = None) -> str:
        if not prompt:
            raise ValueError("Prompt cannot be empty")
        r = await self._call([{"role": "user", "content": prompt}], response_format)
        return r["content"]

    async def apredict_messages(self, messages: List[Dict], functions: List[Dict]) -> Dict[str, Any]:
        return await self._call(messages, None, functions)

    @staticmethod
    def _format_tools(tools: Optional[List[Dict]]) -> List[Dict]:
        out = []
        for t in tools or []:
            if not isinstance(t, dict) or "name" not in t:
                raise ValueError("Invalid tool format")
            out.append({"type": "function", "function": {"name": t["name"],
                                                         "description": t.get("description", ""),
                                                         "parameters": t.get("parameters", {})}})
        return out


def tool_call_schema(tools: Sequence[Dict]) -> Dict[str, Any]:
    """Function-calling reply schema: {"name": <tool>, "arguments": {...}}."""
    return {"name": "str(4)", "arguments": "obj()"}


class LocalLLM(BaseLLM):
    """Reference LLMHandler contract backed by the local MI355X engine."""

    provider = "local"
    prefix_cache_layout = True  # agents put the shared task text first (core/agent.py)

    def __init__(self, config: Any = None, engine=None):
        super().__init__(config)
        if engine is None:
            from .registry import get_engine

            engine = get_engine(self.model_name)
        self.engine = engine
        # node-wide shared context (Serve.broadcast_context): a leading system
        # message whose KV every GPU pre-warmed into its prefix cache
        self.shared_context: Optional[str] = None
        self.tok: Tokenizer = engine.tok
        if engine._thread is None:
            engine.start()

    async def _complete(self, messages, response_format, tools) -> Dict[str, Any]:
        grammar = None
        fixed = None
        if tools:
            names = [t["name"] for t in tools]
            fixed = {"name": names[0]} if len(names) == 1 else None
            grammar = self.engine.grammar.compile(tool_call_schema(tools), fixed)
        elif response_format:
            schema = response_format.get("schema")
            fixed = response_format.get("fixed")
            if schema is not None:
                grammar = self.engine.grammar.compile(schema, fixed)
        if self.shared_context:
            messages = [{"role": "system", "content": self.shared_context}] + list(messages)
        ids = encode_chat(self.tok, messages)
        loop = asyncio.get_running_loop()
        fut = loop.create_future()

        def done(out):
            loop.call_soon_threadsafe(lambda: fut.done() or fut.set_result(out))

        rf = response_format or {}
        temp = float(rf.get("temperature", self.temperature))
        rid = self.engine.submit(ids, done, temperature=temp, max_tokens=int(rf.get("max_tokens", self.max_tokens)),
                                 grammar=grammar,
                                 seed=rf.get("seed"), top_k=int(rf.get("top_k", self.top_k)),
                                 top_p=float(rf.get("top_p", self.top_p)))
        try:
            out = await fut
        except asyncio.CancelledError:
            self.engine.abort(rid)
            raise
        if out.finish_reason == "error":
            raise RuntimeError("local engine failed")
        text = out.text
        tool_calls = None
        if tools:
            try:
                call = json.loads(text)
                tool_calls = [{"id": f"call_{rid}", "type": "function",
                               "function": {"name": call.get("name"),
                                            "arguments": json.dumps(call.get("arguments", {}))}}]
            except json.JSONDecodeError:
                tool_calls = None
        return {
            "content": text,
            "role": "assistant",
            "tool_calls": tool_calls,
            "model": self.engine.model_cfg.name,
            "usage": {"prompt_tokens": out.prompt_tokens, "completion_tokens": out.completion_tokens,
                      "total_tokens": out.prompt_tokens + out.completion_tokens},
            "timing": {"ttft": out.ttft, "latency": out.latency,
                       "cached_prompt_tokens": out.cached_prompt_tokens,
                       "sampled_tokens": out.sampled_tokens},
        }


# ---------------------------------------------------------------------------
# model-free schema LLM (CPU tests, plumbing benchmark)
# ---------------------------------------------------------------------------

_TYPE = re.compile(r"^(\w+)\((.*)\)$")


def fake_value(spec: Any, path: str, fixed: Dict[str, Any], rng: random.Random) -> Any:
    if path in fixed:
        return fixed[path]
    if isinstance(spec, dict):
        if "objlist" in spec:
            return [fake_value(spec["item"], f"{path}[{i}]", fixed, rng) for i in range(int(spec["objlist"]))]
        return {k: fake_value(v, f"{path}.{k}" if path else k, fixed, rng) for k, v in spec.items()}
    s = str(spec)
    if s == "bool":
        return rng.random() < 0.5
    m = _TYPE.match(s)
    kind, arg = m.group(1), m.group(2)
    if kind == "int":
        lo, hi = (int(x) for x in arg.split(","))
        return rng.randint(lo, hi)
    if kind == "str":
        return " ".join(rng.choice(["alpha", "beta", "gamma", "delta", "task", "plan"])
                        for _ in range(max(1, min(3, int(arg)))))
    if kind == "enum":
        return rng.choice(arg.split("|"))
    if kind == "list":
        if not arg:
            return []
        mx = int(arg.rsplit(",", 1)[1])
        return ["item"] * mx
    if kind == "map":
        return {"key": "value"}
    if kind == "obj":
        return {}
    raise ValueError(s)


class SchemaLLM(BaseLLM):
    """Deterministic model-free LLM: replies are schema-valid JSON (CPU / plumbing)."""

    provider = "schema"

    def __init__(self, config: Any = None, seed: int = 0, latency_s: float = 0.0):
        super().__init__(config)
        self.rng = random.Random(seed)
        self.latency_s = latency_s
        self.calls: List[Dict[str, Any]] = []
        self._lock = threading.Lock()

    async def _complete(self, messages, response_format, tools) -> Dict[str, Any]:
        from .grammar import load_schemas

        if self.latency_s:
            await asyncio.sleep(self.latency_s)
        fixed = dict((response_format or {}).get("fixed") or {})
        if tools:
            obj = {"name": fixed.get("name", tools[0]["name"]), "arguments": {}}
            content = json.dumps(obj)
            tool_calls = [{"id": "call_0", "type": "function",
                           "function": {"name": obj["name"], "arguments": "{}"}}]
        else:
            schema = (response_format or {}).get("schema")
            if schema is None:
                content = "ok"
            else:
                spec = load_schemas()[schema] if isinstance(schema, str) else schema
                with self._lock:
                    content = json.dumps(fake_value(spec, "", fixed, self.rng))
            tool_calls = None
        n_prompt = sum(len(str(m.get("content", ""))) // 4 for m in messages)
        return {"content": content, "role": "assistant", "tool_calls": tool_calls, "model": "schema",
                "usage": {"prompt_tokens": n_prompt, "completion_tokens": len(content) // 4,
                          "total_tokens": n_prompt + len(content) // 4}}


def make_llm(config: Union[Dict[str, Any], Any, None] = None, engine=None) -> BaseLLM:
    """LLM factory keyed by provider: "local" (MI355X engine, default), "schema" (model-free),
    or "openai" (any OpenAI-compatible endpoint, e.g. a remote pilottai_amd server)."""
    provider = str(_cfg_get(config, "provider", "local")).lower()
    if provider in ("schema", "fake", "mock"):
        return SchemaLLM(config)
    if provider in ("local", "pilottai", "amd", "rocm", "mi355x"):
        return LocalLLM(config, engine=engine)
    if provider in ("openai", "http", "openai_compat", "remote"):
        from .http_llm import OpenAICompatLLM

        return OpenAICompatLLM(config)
    raise ValueError(f"unsupported LLM provider {provider!r}: use 'local' (on-node engine), 'schema' "
                     "or 'openai' (an OpenAI-compatible endpoint with base_url)")

"""`LLMHandler` — the reference's provider adapter name (pilott/engine/llm.py:12-219).

`LLMHandler(config_dict)` returns the same protocol object as the reference
(generate_response / apredict / apredict_messages, RPM limiting, retries),
served by the on-node engine for provider "local" (default) or by the
model-free SchemaLLM for provider "schema".
"""
from __future__ import annotations

from typing import Any, Dict

from .local_llm import BaseLLM, LocalLLM, SchemaLLM, make_llm


class LLMHandler:
    def __new__(cls, config: Dict[str, Any] = None, engine=None) -> BaseLLM:
        if config is not None and not isinstance(config, dict) and not hasattr(config, "model_name"):
            raise ValueError("Config must be a dictionary")
        return make_llm(config or {}, engine=engine)


__all__ = ["LLMHandler", "LocalLLM", "SchemaLLM", "make_llm"]

"""Process-wide engine registry: one LLMEngine per model per process (= per GPU)."""
from __future__ import annotations

import threading
from typing import Dict, Optional

from .engine import EngineConfig, LLMEngine

_ENGINES: Dict[str, LLMEngine] = {}
_LOCK = threading.Lock()
_DEFAULTS: Dict[str, dict] = {}


def configure_engine(model: str, **overrides):
    """Set EngineConfig overrides used when `model` is first instantiated."""
    _DEFAULTS[model.lower()] = dict(overrides)


def register_engine(model: str, engine: LLMEngine):
    with _LOCK:
        _ENGINES[model.lower()] = engine


def get_engine(model: str = "llama-3-8b", **overrides) -> LLMEngine:
    key = model.lower()
    with _LOCK:
        eng = _ENGINES.get(key)
        if eng is None:
            kw = dict(_DEFAULTS.get(key, {}))
            kw.update(overrides)
            eng = LLMEngine(EngineConfig(model=key, **kw))
            _ENGINES[key] = eng
        return eng


def shutdown_engines():
    with _LOCK:
        for e in _ENGINES.values():
            e.stop()
        _ENGINES.clear()


def peek_engine(model: str) -> Optional[LLMEngine]:
    return _ENGINES.get(model.lower())

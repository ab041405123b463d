"""Agent registry / factory (reference: pilott/core/factory.py:12-150).

Class-level registry of agent types (thread-safe registration) and of active
agents, async creation under a timeout, cleanup. `create_managed_agent` is a real
async context manager (the reference decorated an async generator with
@contextmanager, App. A #36), and agent classes only need to accept a config as
their first argument — BaseAgent resolves its LLM lazily, so `BaseAgent` itself
is creatable.
"""
from __future__ import annotations

import asyncio
import logging
import threading
from contextlib import asynccontextmanager
from typing import Any, Dict, List, Optional, Type

from .agent import BaseAgent
from .config import AgentConfig
from .role import AgentRole


class AgentFactory:
    _agent_types: Dict[str, Type[BaseAgent]] = {}
    _active_agents: Dict[str, BaseAgent] = {}
    _register_lock = threading.Lock()
    _logger = logging.getLogger("pilottai_amd.factory")
    creation_timeout: float = 30.0

    @classmethod
    def register_agent_type(cls, name: str, agent_class: Type[BaseAgent]):
        if not name or not isinstance(name, str):
            raise ValueError("Agent type name must be a non-empty string")
        if not isinstance(agent_class, type) or not issubclass(agent_class, BaseAgent):
            raise TypeError("agent_class must be a subclass of BaseAgent")
        with cls._register_lock:
            if name in cls._agent_types:
                raise ValueError(f"Agent type {name} already registered")
            cls._agent_types[name] = agent_class

    @classmethod
    def unregister_agent_type(cls, name: str):
        with cls._register_lock:
            cls._agent_types.pop(name, None)

    @classmethod
    async def create_agent(cls, agent_type: str, config: Optional[AgentConfig] = None, **kwargs) -> BaseAgent:
        if not agent_type:
            raise ValueError("Agent type cannot be empty")
        if agent_type not in cls._agent_types:
            raise ValueError(f"Unknown agent type: {agent_type}. Valid types: {', '.join(cls._agent_types)}")
        agent_kw = {k: kwargs.pop(k) for k in ("llm", "llm_config", "tools", "policy", "function_calling_llm")
                    if k in kwargs}
        if config is None:
            config = AgentConfig(role=agent_type, role_type=AgentRole.WORKER,
                                 goal=f"Execute tasks as a {agent_type}",
                                 description=f"Worker agent of type {agent_type}", **kwargs)
        elif isinstance(config, dict):
            config = AgentConfig(**config)
        cls._validate_config(config)
        agent_cls = cls._agent_types[agent_type]
        agent = agent_cls(config, **agent_kw) if agent_kw else agent_cls(config)
        try:
            await asyncio.wait_for(agent.start(), timeout=cls.creation_timeout)
        except asyncio.TimeoutError:
            cls._logger.error("timeout starting agent of type %s", agent_type)
            raise
        cls._active_agents[agent.id] = agent
        return agent

    @classmethod
    @asynccontextmanager
    async def create_managed_agent(cls, agent_type: str, config: Optional[AgentConfig] = None, **kwargs):
        agent = await cls.create_agent(agent_type, config, **kwargs)
        try:
            yield agent
        finally:
            if agent.id in cls._active_agents:
                await cls.cleanup_agent(agent.id)

    @classmethod
    async def cleanup_agent(cls, agent_id: str):
        agent = cls._active_agents.pop(agent_id, None)
        if agent is None:
            return
        await agent.stop()
        cleanup = getattr(agent, "cleanup_resources", None)
        if cleanup is not None:
            await cleanup()

    @classmethod
    def list_available_types(cls) -> List[str]:
        return list(cls._agent_types)

    @classmethod
    def get_active_agents(cls) -> Dict[str, BaseAgent]:
        return dict(cls._active_agents)

    @classmethod
    async def cleanup_all_agents(cls):
        for aid in list(cls._active_agents):
            await cls.cleanup_agent(aid)

    @staticmethod
    def _validate_config(config: AgentConfig):
        if not config.role:
            raise ValueError("Agent role must be specified")
        if not config.goal:
            raise ValueError("Agent goal must be specified")
        if config.max_iterations < 1:
            raise ValueError("max_iterations must be greater than 0")
        if config.max_queue_size < 1:
            raise ValueError("max_queue_size must be greater than 0")
        if config.task_timeout < 1:
            raise ValueError("task_timeout must be greater than 0")

    @classmethod
    def create_from_spec(cls, spec: Dict[str, Any]) -> BaseAgent:
        """Synchronous construction (not started) from a {"type", "config"} dict."""
        t = spec.get("type", "base")
        agent_cls = cls._agent_types.get(t, BaseAgent)
        return agent_cls(AgentConfig(**spec["config"]))

"""pilottai_amd — an MI355X-native multi-agent orchestration engine.

Same capabilities and user API as PilottAI (Serve / agents / factory / routing /
delegation / load balancing / scaling / fault tolerance / memory / knowledge /
tools), with the remote LLM provider replaced by an on-node Llama-3 inference
engine built on hand-written CDNA4 HIP kernels (csrc/ops) and a native C++
serving runtime (csrc/runtime), scaled over a node's GPUs with RCCL.
"""
from __future__ import annotations

import importlib

__version__ = "0.1.0"

_LAZY = {
    "Serve": ("pilottai_amd.serve", "Serve"),
    "ServeConfig": ("pilottai_amd.serve", "ServeConfig"),
    "BaseAgent": ("pilottai_amd.core.agent", "BaseAgent"),
    "AgentConfig": ("pilottai_amd.core.config", "AgentConfig"),
    "LLMConfig": ("pilottai_amd.core.config", "LLMConfig"),
    "LogConfig": ("pilottai_amd.core.config", "LogConfig"),
    "AgentRole": ("pilottai_amd.core.role", "AgentRole"),
    "AgentStatus": ("pilottai_amd.core.role", "AgentStatus"),
    "Task": ("pilottai_amd.core.task", "Task"),
    "TaskResult": ("pilottai_amd.core.task", "TaskResult"),
    "TaskStatus": ("pilottai_amd.core.task", "TaskStatus"),
    "TaskPriority": ("pilottai_amd.core.task", "TaskPriority"),
    "Memory": ("pilottai_amd.core.memory", "Memory"),
    "AgentFactory": ("pilottai_amd.core.factory", "AgentFactory"),
    "TaskRouter": ("pilottai_amd.core.router", "TaskRouter"),
    "ControlPolicy": ("pilottai_amd.core.policy", "ControlPolicy"),
    "Tool": ("pilottai_amd.tools.tool", "Tool"),
    "LocalLLM": ("pilottai_amd.engine.local_llm", "LocalLLM"),
    "SchemaLLM": ("pilottai_amd.engine.local_llm", "SchemaLLM"),
    "LLMHandler": ("pilottai_amd.engine.llm_handler", "LLMHandler"),
    "EnhancedMemory": ("pilottai_amd.memory.enhanced_memory", "EnhancedMemory"),
    "KnowledgeManager": ("pilottai_amd.knowledge.knowledge_manager", "KnowledgeManager"),
    "LoadBalancer": ("pilottai_amd.orchestration.load_balancer", "LoadBalancer"),
    "DynamicScaling": ("pilottai_amd.orchestration.scaling", "DynamicScaling"),
    "FaultTolerance": ("pilottai_amd.orchestration.fault_tolerance", "FaultTolerance"),
    "TaskDelegator": ("pilottai_amd.delegation.task_delegator", "TaskDelegator"),
    "set_default_llm": ("pilottai_amd.core.agent", "set_default_llm"),
}

__all__ = list(_LAZY) + ["__version__"]


def __getattr__(name):
    if name in _LAZY:
        mod, attr = _LAZY[name]
        return getattr(importlib.import_module(mod), attr)
    raise AttributeError(f"module 'pilottai_amd' has no attribute {name!r}")

"""Core data model and agent runtime (reference: pilott/core/__init__.py)."""
from .agent import BaseAgent, set_default_llm  # noqa: F401
from .config import AgentConfig, LLMConfig, LogConfig, SecureConfig  # noqa: F401
from .factory import AgentFactory  # noqa: F401
from .memory import Memory, MemoryEntry  # noqa: F401
from .policy import ControlPolicy  # noqa: F401
from .role import AgentRole, AgentStatus  # noqa: F401
from .router import RouterConfig, TaskRouter  # noqa: F401
from .task import Task, TaskPriority, TaskResult, TaskStatus  # noqa: F401

"""Tools and knowledge sources (reference: pilott/tools/__init__.py)."""
from .knowledge import KnowledgeSource  # noqa: F401
from .tool import (Tool, ToolError, ToolMetrics, ToolPermissionError, ToolStatus,  # noqa: F401
                   ToolTimeoutError, ToolValidationError, echo_tool)

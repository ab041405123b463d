"""Tool wrapper (reference: pilott/tools/tool.py:9-217).

Wraps a user callable (sync or async) with an enable/cooldown gate, bounded
concurrency, per-attempt timeout, linear-backoff retries and metrics. Unlike the
reference it is importable under pydantic 2 (runtime state lives in private
attributes, App. A #27) and needs no separate `setup()` call.
"""
from __future__ import annotations

import asyncio
import inspect
import logging
import time
import traceback
from datetime import datetime
from enum import Enum
from typing import Any, Callable, Dict, List, Optional, Set

from pydantic import BaseModel, ConfigDict, Field, PrivateAttr


class ToolStatus(str, Enum):
    READY = "ready"
    BUSY = "busy"
    ERROR = "error"
    DISABLED = "disabled"


class ToolMetrics(BaseModel):
    usage_count: int = 0
    success_count: int = 0
    error_count: int = 0
    total_execution_time: float = 0.0
    avg_execution_time: float = 0.0
    last_execution: Optional[datetime] = None
    last_error: Optional[str] = None
    error_types: Dict[str, int] = Field(default_factory=dict)


class ToolError(Exception):
    """Base class for tool errors."""


class ToolTimeoutError(ToolError):
    pass


class ToolPermissionError(ToolError):
    pass


class ToolValidationError(ToolError):
    pass


class Tool(BaseModel):
    model_config = ConfigDict(arbitrary_types_allowed=True)

    name: str
    description: str = ""
    function: Any
    parameters: Dict[str, Any] = Field(default_factory=dict)
    permissions: List[str] = Field(default_factory=list)
    required_capabilities: List[str] = Field(default_factory=list)
    timeout: float = Field(default=30.0, gt=0)
    max_retries: int = Field(default=3, ge=0)
    retry_delay: float = Field(default=1.0, ge=0)
    cooldown_period: float = Field(default=0.0, ge=0)
    max_concurrent: int = Field(default=1, ge=1)
    enabled: bool = True
    status: ToolStatus = ToolStatus.READY
    metrics: ToolMetrics = Field(default_factory=ToolMetrics)

    _lock: Optional[asyncio.Lock] = PrivateAttr(default=None)
    _active: Set[str] = PrivateAttr(default_factory=set)
    _last_start: float = PrivateAttr(default=0.0)
    _logger: logging.Logger = PrivateAttr(default=None)

    def model_post_init(self, __ctx):
        self._logger = logging.getLogger(f"pilottai_amd.tool.{self.name}")

    async def setup(self) -> "Tool":
        """Kept for API compatibility; the tool is usable without it."""
        return self

    @property
    def active_executions(self) -> Set[str]:
        return self._active

    def _can_execute(self) -> bool:
        if not self.enabled:
            return False
        if self.cooldown_period > 0 and self._last_start and \
                time.monotonic() - self._last_start < self.cooldown_period:
            return False
        return True

    async def execute(self, execution_id: Optional[str] = None, **kwargs) -> Any:
        if not self.enabled:
            raise ToolError(f"Tool {self.name} is disabled")
        execution_id = execution_id or f"{self.name}_{time.monotonic_ns()}"
        if execution_id in self._active:
            raise ToolError(f"Duplicate execution ID: {execution_id}")
        if not self._can_execute():
            raise ToolError(f"Tool {self.name} not ready (cooldown)")
        if len(self._active) >= self.max_concurrent:
            raise ToolError("Maximum concurrent executions reached")
        self._active.add(execution_id)
        self.status = ToolStatus.BUSY
        self._last_start = time.monotonic()
        t0 = time.perf_counter()
        try:
            result = await self._execute_with_retry(**kwargs)
            self._update_metrics(True, t0)
            return result
        except asyncio.TimeoutError:
            self._update_metrics(False, t0, "TimeoutError: execution timed out")
            raise ToolTimeoutError(f"Execution timed out after {self.timeout}s")
        except Exception as e:
            self._update_metrics(False, t0, f"{type(e).__name__}: {e}")
            raise
        finally:
            self._active.discard(execution_id)
            if not self._active and self.enabled:
                self.status = ToolStatus.READY

    async def _execute_with_retry(self, **kwargs) -> Any:
        last: Optional[BaseException] = None
        attempts = max(1, self.max_retries)
        for attempt in range(attempts):
            try:
                if inspect.iscoroutinefunction(self.function):
                    return await asyncio.wait_for(self.function(**kwargs), self.timeout)
                return await asyncio.wait_for(asyncio.to_thread(self.function, **kwargs), self.timeout)
            except asyncio.TimeoutError:
                last = ToolTimeoutError(f"Timeout on attempt {attempt + 1}")
                self._logger.warning("execution timeout, attempt %d", attempt + 1)
            except Exception as e:  # noqa: BLE001
                last = e
                self._logger.debug("attempt %d failed: %s\n%s", attempt + 1, e, traceback.format_exc())
            if attempt < attempts - 1:
                await asyncio.sleep(self.retry_delay * (attempt + 1))
        raise last if last else ToolError("Execution failed after all retries")

    def _update_metrics(self, ok: bool, t0: float, error: Optional[str] = None):
        m = self.metrics
        dt = time.perf_counter() - t0
        m.usage_count += 1
        m.total_execution_time += dt
        m.avg_execution_time = m.total_execution_time / m.usage_count
        m.last_execution = datetime.now()
        if ok:
            m.success_count += 1
        else:
            m.error_count += 1
            m.last_error = error
            et = (error or "unknown").split(":")[0]
            m.error_types[et] = m.error_types.get(et, 0) + 1

    def disable(self, reason: str = ""):
        self.enabled = False
        self.status = ToolStatus.DISABLED
        if reason:
            self._logger.warning("tool disabled: %s", reason)

    def enable(self):
        self.enabled = True
        self.status = ToolStatus.READY

    def get_metrics(self) -> Dict[str, Any]:
        return {"status": self.status, "metrics": self.metrics.model_dump(),
                "active_executions": len(self._active), "enabled": self.enabled}

    @property
    def success_rate(self) -> float:
        return self.metrics.success_count / self.metrics.usage_count if self.metrics.usage_count else 0.0

    def spec(self) -> Dict[str, Any]:
        """OpenAI-style function description (function-calling LLM path)."""
        return {"name": self.name, "description": self.description, "parameters": self.parameters}

    @classmethod
    def from_callable(cls, fn: Callable, name: Optional[str] = None, **kw) -> "Tool":
        return cls(name=name or getattr(fn, "__name__", "tool"), description=(fn.__doc__ or "").strip(),
                   function=fn, **kw)


def echo_tool(**kwargs) -> Dict[str, Any]:
    """Identity tool used by the plumbing benchmark (BASELINE config 1)."""
    return {"echo": kwargs}

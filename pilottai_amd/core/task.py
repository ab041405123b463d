"""Task / TaskResult data model (reference: pilott/core/task.py:11-363).

Serialized form matches the reference so task/memory checkpoints
interoperate. Intended behaviour is implemented where the reference is broken
(SURVEY App. A):
  #14 dependencies are ids of *other* tasks: only a self-dependency is a cycle
      here; graph-level cycles are checked by `check_dependency_cycles`;
  #15 parent_task_id / subtasks / required_skills are real fields;
  #16 TaskPriority compares by rank (LOW < MEDIUM < HIGH < CRITICAL);
  #17 complexity=None is allowed;
  #18 copy() issues a fresh id unless `keep_id=True` and applies updates;
  #19 a failed result on an IN_PROGRESS task moves it to RETRY while retries remain;
  #20 no cleanup in __del__ on half-built objects.
"""
from __future__ import annotations

import asyncio
import os
import uuid
from contextlib import asynccontextmanager
from datetime import datetime
from enum import Enum
from pathlib import Path
from typing import Any, Dict, Iterable, List, Optional, Set

from pydantic import BaseModel, ConfigDict, Field, PrivateAttr, field_validator


class TaskStatus(str, Enum):
    PENDING = "pending"
    IN_PROGRESS = "in_progress"
    COMPLETED = "completed"
    FAILED = "failed"
    DELEGATED = "delegated"
    RETRY = "retry"
    CANCELLED = "cancelled"
    TIMEOUT = "timeout"


_PRIO_RANK = {"low": 0, "medium": 1, "high": 2, "critical": 3}


class TaskPriority(str, Enum):
    LOW = "low"
    MEDIUM = "medium"
    HIGH = "high"
    CRITICAL = "critical"

    @property
    def rank(self) -> int:
        return _PRIO_RANK[self.value]

    def _cmp_rank(self, other):
        if isinstance(other, TaskPriority):
            return other.rank
        if isinstance(other, str) and other.lower() in _PRIO_RANK:
            return _PRIO_RANK[other.lower()]
        return None

    # rank order, not lexicographic str order (App. A #16); all four operators are
    # defined explicitly because str already provides them
    def __lt__(self, other):
        r = self._cmp_rank(other)
        return NotImplemented if r is None else self.rank < r

    def __le__(self, other):
        r = self._cmp_rank(other)
        return NotImplemented if r is None else self.rank <= r

    def __gt__(self, other):
        r = self._cmp_rank(other)
        return NotImplemented if r is None else self.rank > r

    def __ge__(self, other):
        r = self._cmp_rank(other)
        return NotImplemented if r is None else self.rank >= r

    def __hash__(self):
        return hash(self.value)

    def __eq__(self, other):
        if isinstance(other, Enum):
            return self.value == other.value
        return self.value == other

    @classmethod
    def coerce(cls, v: Any) -> "TaskPriority":
        if isinstance(v, TaskPriority):
            return v
        if isinstance(v, (int, float)):
            return [cls.LOW, cls.MEDIUM, cls.HIGH, cls.CRITICAL][max(0, min(3, int(v) - 1 if v > 0 else 0))]
        s = str(getattr(v, "value", v)).lower()
        return cls(s) if s in _PRIO_RANK else cls.MEDIUM


def _uuid4_str() -> str:
    """str(uuid.uuid4()) at a fifth of its cost (one urandom read, no UUID object)."""
    b = bytearray(os.urandom(16))
    b[6] = (b[6] & 0x0F) | 0x40
    b[8] = (b[8] & 0x3F) | 0x80
    h = b.hex()
    return f"{h[:8]}-{h[8:12]}-{h[12:16]}-{h[16:20]}-{h[20:]}"


class TaskResult(BaseModel):
    model_config = ConfigDict(arbitrary_types_allowed=True)

    success: bool
    output: Any = None
    error: Optional[str] = None
    execution_time: float = 0.0
    metadata: Dict[str, Any] = Field(default_factory=dict)
    resources_cleaned: bool = False
    completion_time: Optional[datetime] = None  # set at construction (model_post_init)
    # Hot-path notes (benchmarks/plumbing.py, pydantic 2.13): mutable defaults use
    # default_factory (a literal [] / {} default is deep-copied per instance, ~4x the cost),
    # private attributes are created lazily, and model_post_init writes the instance dict
    # directly (pydantic's __setattr__ costs ~1-2 us per assignment).
    _file_handles: Optional[Set[Any]] = PrivateAttr(default=None)
    _temp_files: Optional[Set[Path]] = PrivateAttr(default=None)

    def model_post_init(self, __ctx):
        if self.completion_time is None:
            self.__dict__["completion_time"] = datetime.now()

    def register_file_handle(self, h: Any):
        if self._file_handles is None:
            self._file_handles = set()
        self._file_handles.add(h)

    def register_temp_file(self, p):
        if self._temp_files is None:
            self._temp_files = set()
        self._temp_files.add(Path(p))

    def cleanup_resources(self):
        self._file_handles = self._file_handles or set()
        self._temp_files = self._temp_files or set()
        for h in list(self._file_handles):
            try:
                h.close()
            except Exception:  # noqa: BLE001
                pass
        self._file_handles.clear()
        for p in list(self._temp_files):
            try:
                p.unlink()
            except Exception:  # noqa: BLE001
                pass
        self._temp_files.clear()
        self.resources_cleaned = True


class Task(BaseModel):
    model_config = ConfigDict(arbitrary_types_allowed=True, validate_assignment=False)

    id: str = ""  # a fresh uuid4 when not given (model_post_init)
    description: str
    status: TaskStatus = TaskStatus.PENDING
    priority: TaskPriority = TaskPriority.MEDIUM
    async_execution: bool = False
    max_retries: int = Field(default=3, ge=0)
    retry_count: int = Field(default=0, ge=0)
    timeout: Optional[float] = None
    deadline: Optional[datetime] = None
    created_at: Optional[datetime] = None  # set at construction
    started_at: Optional[datetime] = None
    completed_at: Optional[datetime] = None
    context: List["Task"] = Field(default_factory=list)
    tools: List[str] = Field(default_factory=list)
    config: Dict[str, Any] = Field(default_factory=dict)
    dependencies: List[str] = Field(default_factory=list)
    output_file: Optional[Path] = None
    result: Optional[TaskResult] = None
    complexity: Optional[int] = None
    metadata: Dict[str, Any] = Field(default_factory=dict)
    # fields the reference used but never declared (App. A #15)
    parent_task_id: Optional[str] = None
    subtasks: List[str] = Field(default_factory=list)
    required_skills: List[str] = Field(default_factory=list)
    type: Optional[str] = None

    _locks: Optional[Dict[str, asyncio.Lock]] = PrivateAttr(default=None)
    _file_handles: Optional[Set[Any]] = PrivateAttr(default=None)
    _temp_files: Optional[Set[Path]] = PrivateAttr(default=None)

    def model_post_init(self, __ctx):
        d = self.__dict__  # direct writes: pydantic's __setattr__ is the slow part of a Task
        if not d["id"]:
            d["id"] = _uuid4_str()
        if d["created_at"] is None:
            d["created_at"] = datetime.now()
        if d["dependencies"] and d["id"] in d["dependencies"]:
            raise ValueError(f"Circular dependency: task {d['id']} depends on itself")

    # private resources, created on first use (most tasks never lock or open anything)
    def _res(self, name: str, make):
        priv = self.__pydantic_private__
        v = priv.get(name)
        if v is None:
            v = priv[name] = make()
        return v

    # -- validators -----------------------------------------------------------
    @field_validator("priority", mode="before")
    @classmethod
    def _prio(cls, v):
        return TaskPriority.coerce(v)

    @field_validator("deadline")
    @classmethod
    def _deadline(cls, v):
        if v is not None and v < datetime.now():
            raise ValueError("Deadline cannot be in the past")
        return v

    @field_validator("complexity")
    @classmethod
    def _complexity(cls, v):
        if v is not None and not 1 <= v <= 10:
            raise ValueError("Complexity must be between 1 and 10")
        return v

    @field_validator("output_file")
    @classmethod
    def _outfile(cls, v):
        if v is None:
            return None
        v = Path(v)
        if v.exists() and not v.is_file():
            raise ValueError("Output path exists but is not a file")
        return v

    # -- locking / resources ----------------------------------------------------
    async def acquire_lock(self, resource: str, timeout: float = 5.0) -> bool:
        if not resource:
            raise ValueError("Resource name cannot be empty")
        lock = self._res("_locks", dict).setdefault(resource, asyncio.Lock())
        try:
            await asyncio.wait_for(lock.acquire(), timeout=timeout)
            return True
        except asyncio.TimeoutError:
            return False

    def release_lock(self, resource: str):
        lock = (self._locks or {}).get(resource)
        if lock is not None and lock.locked():
            lock.release()

    @asynccontextmanager
    async def resource_lock(self, resource: str):
        ok = await self.acquire_lock(resource)
        if not ok:
            raise TimeoutError(f"could not lock {resource}")
        try:
            yield
        finally:
            self.release_lock(resource)

    def register_file_handle(self, h: Any):
        if h is None:
            raise ValueError("File handle cannot be None")
        self._res("_file_handles", set).add(h)

    def register_temp_file(self, p):
        if not p:
            raise ValueError("Path cannot be None")
        self._res("_temp_files", set).add(Path(p))

    def cleanup_resources(self):
        for h in list(self._file_handles or ()):
            try:
                h.close()
            except Exception:  # noqa: BLE001
                pass
        if self._file_handles:
            self._file_handles.clear()
        for p in list(self._temp_files or ()):
            try:
                p.unlink()
            except Exception:  # noqa: BLE001
                pass
        if self._temp_files:
            self._temp_files.clear()
        for name in list(self._locks or ()):
            self.release_lock(name)
        if self._locks:
            self._locks.clear()
        if self.result is not None:
            self.result.cleanup_resources()

    # -- lifecycle ----------------------------------------------------------------
    def is_expired(self) -> bool:
        return self.deadline is not None and datetime.now() > self.deadline

    @property
    def is_overdue(self) -> bool:
        return self.is_expired()

    def can_retry(self) -> bool:
        return (self.status in (TaskStatus.FAILED, TaskStatus.TIMEOUT, TaskStatus.IN_PROGRESS)
                and self.retry_count < self.max_retries and not self.is_expired())

    def mark_started(self):
        if self.status not in (TaskStatus.PENDING, TaskStatus.RETRY, TaskStatus.DELEGATED):
            raise ValueError(f"Cannot start task in {self.status} status")
        self.status = TaskStatus.IN_PROGRESS
        self.started_at = datetime.now()

    def mark_completed(self, result: TaskResult):
        if not result.success and self.can_retry():
            self.status = TaskStatus.RETRY
            self.retry_count += 1
        else:
            self.status = TaskStatus.COMPLETED if result.success else TaskStatus.FAILED
        self.completed_at = datetime.now()
        self.result = result

    def mark_failed(self, error: str):
        self.status = TaskStatus.FAILED
        self.completed_at = datetime.now()
        dt = (self.completed_at - self.started_at).total_seconds() if self.started_at else 0.0
        self.result = TaskResult(success=False, output=None, error=error, execution_time=dt)
        self.retry_count += 1

    def update_status(self, status: TaskStatus, **kwargs):
        self.status = TaskStatus(status)
        if self.status == TaskStatus.IN_PROGRESS and not self.started_at:
            self.started_at = datetime.now()
        elif self.status in (TaskStatus.COMPLETED, TaskStatus.FAILED):
            self.completed_at = datetime.now()
        for k, v in kwargs.items():
            if k in type(self).model_fields:
                setattr(self, k, v)

    @property
    def duration(self) -> Optional[float]:
        if self.started_at and self.completed_at:
            return (self.completed_at - self.started_at).total_seconds()
        return None

    def add_subtask(self, subtask: "Task"):
        subtask.parent_task_id = self.id
        if subtask.id not in self.subtasks:
            self.subtasks.append(subtask.id)

    # -- serialisation -------------------------------------------------------------
    def to_dict(self) -> Dict[str, Any]:
        return self.model_dump(mode="json", exclude_none=True)

    def dict(self, *args, **kwargs) -> Dict[str, Any]:  # pydantic-v1 style alias used by agents
        return self.model_dump(*args, **kwargs)

    def copy(self, *, keep_id: bool = False, update: Optional[Dict[str, Any]] = None, **kwargs) -> "Task":
        """Copy with updates; a fresh id/status unless keep_id (App. A #18)."""
        data = self.model_dump()
        if not keep_id:
            data.update(id=_uuid4_str(), status=TaskStatus.PENDING, result=None,
                        started_at=None, completed_at=None)
        data.update(update or {})
        data.update(kwargs)
        return Task(**{k: v for k, v in data.items() if k in type(self).model_fields})

    def to_prompt(self) -> str:
        p = f"Task: {self.description}\n"
        if self.context:
            p += "\nContext:\n" + "\n".join(f"- {t.description}" for t in self.context)
        if self.required_skills:
            p += f"\nRequired Skills: {', '.join(self.required_skills)}"
        if self.tools:
            p += f"\nAvailable Tools: {', '.join(self.tools)}"
        return p

    @classmethod
    def from_any(cls, obj: Any) -> "Task":
        """Accept a Task, a description string, or a documented-API dict task
        (e.g. {"type": "process_pdf", "file_path": ...}, README.md:97-100)."""
        if isinstance(obj, Task):
            return obj
        if isinstance(obj, str):
            return cls(description=obj)
        if isinstance(obj, dict):
            known = {k: v for k, v in obj.items() if k in cls.model_fields}
            extra = {k: v for k, v in obj.items() if k not in cls.model_fields}
            if "description" not in known:
                import json

                known["description"] = obj.get("description") or json.dumps(obj, default=str)
            md = dict(known.get("metadata") or {})
            md.update(extra)
            known["metadata"] = md
            return cls(**known)
        raise TypeError(f"cannot build a Task from {type(obj).__name__}")


Task.model_rebuild()


def check_dependency_cycles(tasks: Iterable[Task]) -> None:
    """Raise ValueError if the dependency graph over `tasks` has a cycle."""
    graph = {t.id: list(t.dependencies) for t in tasks}
    state: Dict[str, int] = {}

    def visit(n: str, stack: List[str]):
        s = state.get(n, 0)
        if s == 1:
            raise ValueError("Circular dependency detected: " + " -> ".join(stack + [n]))
        if s == 2:
            return
        state[n] = 1
        for d in graph.get(n, []):
            visit(d, stack + [n])
        state[n] = 2

    for n in graph:
        visit(n, [])

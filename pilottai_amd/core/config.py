"""Validated configuration models (reference: pilott/core/config.py:10-249).

One `AgentConfig` replaces the reference's two conflicting copies
(pilott/core/agent.py:19-29 and pilott/core/config.py:103-249): it
carries both field families, with `max_iter`/`max_iterations` and
`allow_delegation`/`can_delegate` kept in sync, so BaseAgent and the control-plane
services read the same object. Save/load round-trips (App. A #37).

`SecureConfig` is the reference's Fernet store: the same key-file format and the same
tokens (AES-128-CBC + HMAC-SHA256), implemented in the standard library by
`core/fernet.py` because `cryptography` is not importable here, so key files and
encrypted values move between the two frameworks unchanged.
"""
from __future__ import annotations

import base64
import json
import shutil
from pathlib import Path
from typing import Any, Dict, List, Optional

from pydantic import BaseModel, ConfigDict, Field, SecretStr, field_validator, model_validator

from .fernet import Fernet, InvalidToken
from .role import AgentRole


class SecureConfig:
    """Fernet-encrypted sensitive config values (reference: pilott/core/config.py:10-38).

    The key file holds a Fernet key (44 url-safe base64 bytes), as the reference writes
    it. A 32-byte raw key (this class's pre-Fernet format) is read as the same 32 key
    bytes."""

    def __init__(self, key_path: Optional[Path] = None):
        self._key_path = Path(key_path) if key_path else None
        if self._key_path and self._key_path.exists():
            raw = self._key_path.read_bytes()
            if len(raw) == 32:  # legacy raw key: check the length BEFORE any strip (a random
                self.key = base64.urlsafe_b64encode(raw)  # key may start/end with a whitespace byte)
            else:
                self.key = raw.strip()  # Fernet key (44 url-safe base64 bytes, maybe + newline)
        else:
            self.key = Fernet.generate_key()
            if self._key_path:
                self._key_path.parent.mkdir(parents=True, exist_ok=True)
                self._key_path.write_bytes(self.key)
        self.cipher = Fernet(self.key)

    def encrypt(self, value: str) -> bytes:
        if not value:
            raise ValueError("Cannot encrypt empty value")
        return self.cipher.encrypt(value.encode())

    def decrypt(self, token: bytes) -> str:
        if not token:
            raise ValueError("Cannot decrypt empty value")
        try:
            return self.cipher.decrypt(token).decode()
        except InvalidToken as e:
            raise ValueError(f"Invalid token: {e}") from e

    def cleanup(self):
        try:
            if self._key_path and self._key_path.exists():
                self._key_path.unlink()
        except Exception:  # noqa: BLE001
            pass


class LLMConfig(BaseModel):
    """LLM selection. provider "local" = the on-node MI355X engine (default)."""
    model_config = ConfigDict(arbitrary_types_allowed=True, use_enum_values=True,
                              protected_namespaces=())

    model_name: str = "llama-3-8b"
    provider: str = "local"
    api_key: SecretStr = SecretStr("")
    temperature: float = Field(default=0.7, ge=0.0, le=2.0)
    top_p: float = Field(default=1.0, gt=0.0, le=1.0)   # nucleus truncation (1 = off)
    top_k: int = Field(default=0, ge=0)                 # top-k truncation (0 = off)
    max_tokens: int = Field(default=2000, gt=0)
    function_calling_model: Optional[str] = None
    system_template: Optional[str] = None
    prompt_template: Optional[str] = None
    retry_attempts: int = Field(default=3, ge=0)
    retry_delay: float = Field(default=1.0, ge=0.0)
    timeout: float = Field(default=30.0, gt=0)
    max_rpm: Optional[int] = Field(default=None, gt=0)
    max_concurrent: Optional[int] = Field(default=None, gt=0)
    base_url: Optional[str] = None  # provider "openai": an OpenAI-compatible endpoint (serving/http_server.py)

    @field_validator("api_key", mode="before")
    @classmethod
    def _key(cls, v):
        return v if isinstance(v, SecretStr) else SecretStr(str(v or ""))

    def to_dict(self) -> Dict[str, Any]:
        return {"model_name": self.model_name, "provider": self.provider, "temperature": self.temperature,
                "top_p": self.top_p, "top_k": self.top_k, "max_tokens": self.max_tokens,
                "function_calling_model": self.function_calling_model}

    def handler_config(self) -> Dict[str, Any]:
        d = self.model_dump()
        d["api_key"] = self.api_key.get_secret_value()
        return d


class LogConfig(BaseModel):
    model_config = ConfigDict(arbitrary_types_allowed=True)

    verbose: bool = False
    log_to_file: bool = False
    log_dir: Path = Field(default=Path("logs"))
    log_format: str = "%(asctime)s - %(name)s - %(levelname)s - %(message)s"
    log_level: str = Field(default="INFO", pattern="^(DEBUG|INFO|WARNING|ERROR|CRITICAL)$")
    max_file_size: int = Field(default=10 * 1024 * 1024)
    backup_count: int = Field(default=5, ge=0)
    log_rotation: str = Field(default="midnight")

    @model_validator(mode="after")
    def _mkdir(self):
        if self.log_to_file:
            self.log_dir = Path(self.log_dir)
            self.log_dir.mkdir(parents=True, exist_ok=True)
        return self


class AgentConfig(BaseModel):
    model_config = ConfigDict(arbitrary_types_allowed=True, use_enum_values=False)

    role: str
    role_type: AgentRole = AgentRole.WORKER
    goal: str = ""
    description: str = ""
    backstory: Optional[str] = None
    knowledge: List[str] = Field(default_factory=list)
    knowledge_sources: List[str] = Field(default_factory=list)
    tools: List[str] = Field(default_factory=list)
    required_capabilities: List[str] = Field(default_factory=list)
    specializations: List[str] = Field(default_factory=list)
    max_iterations: int = Field(default=20, gt=0)
    max_iter: Optional[int] = Field(default=None, gt=0)
    max_rpm: Optional[int] = Field(default=None, gt=0)
    max_execution_time: Optional[int] = Field(default=None, gt=0)
    retry_limit: int = Field(default=2, ge=0)
    code_execution_mode: str = Field(default="safe", pattern="^(safe|restricted|unrestricted)$")
    memory_enabled: bool = True
    verbose: bool = False
    can_delegate: bool = False
    allow_delegation: Optional[bool] = None
    use_cache: bool = True
    can_execute_code: bool = False
    max_child_agents: int = Field(default=10, gt=0)
    max_queue_size: int = Field(default=100, gt=0)
    max_task_complexity: int = Field(default=5, ge=1, le=10)
    delegation_threshold: float = Field(default=0.7, ge=0.0, le=1.0)
    max_concurrent_tasks: int = Field(default=5, gt=0)
    task_timeout: int = Field(default=300, gt=0)
    resource_limits: Dict[str, float] = Field(default_factory=lambda: {
        "cpu_percent": 80.0, "memory_percent": 80.0, "disk_percent": 80.0})
    websocket_enabled: bool = True
    websocket_host: str = "localhost"
    websocket_port: int = Field(default=8765, ge=1024, le=65535)
    additional_config: Dict[str, Any] = Field(default_factory=dict)

    @field_validator("role_type", mode="before")
    @classmethod
    def _role_type(cls, v):
        if isinstance(v, str) and v.startswith("AgentRole."):
            v = v.split(".", 1)[1].lower()  # files written by the reference
        return AgentRole(getattr(v, "value", v))

    @field_validator("resource_limits")
    @classmethod
    def _limits(cls, v):
        for k, val in v.items():
            if val <= 0 or val > 100:
                raise ValueError(f"Resource limit {k} must be between 0 and 100")
        return v

    @model_validator(mode="after")
    def _sync_aliases(self):
        # max_iter (agent-side name) <-> max_iterations; allow_delegation <-> can_delegate
        if self.max_iter is None:
            self.max_iter = self.max_iterations
        else:
            self.max_iterations = self.max_iter
        if self.allow_delegation is None:
            self.allow_delegation = self.can_delegate
        else:
            self.can_delegate = self.allow_delegation
        return self

    def to_dict(self) -> Dict[str, Any]:
        d = self.model_dump(mode="json")
        d["role_type"] = self.role_type.value
        return d

    @classmethod
    def from_file(cls, path) -> "AgentConfig":
        path = Path(path)
        if not path.exists():
            raise FileNotFoundError(f"Config file not found: {path}")
        try:
            data = json.loads(path.read_text())
        except json.JSONDecodeError as e:
            raise ValueError(f"Invalid JSON in config file: {e}")
        return cls(**data)

    @property
    def has_sensitive_data(self) -> bool:
        pats = ("password", "secret", "key", "token", "auth")
        d = self.to_dict()
        return any(p in str(k).lower() or p in str(v).lower() for k, v in d.items() for p in pats)

    def save_to_file(self, path):
        path = Path(path)
        backup = None
        try:
            if path.exists():
                backup = path.with_suffix(path.suffix + ".bak")
                shutil.copy2(path, backup)
            path.parent.mkdir(parents=True, exist_ok=True)
            tmp = path.with_suffix(path.suffix + ".tmp")
            tmp.write_text(json.dumps(self.to_dict(), indent=2))
            tmp.replace(path)
            if backup and backup.exists():
                backup.unlink()
        except Exception as e:
            if backup and backup.exists():
                shutil.copy2(backup, path)
            raise ValueError(f"Failed to save config: {e}")

"""Agent role / status vocabularies (reference: pilott/core/role.py, status.py)."""
from enum import Enum


class AgentRole(str, Enum):
    ORCHESTRATOR = "orchestrator"
    WORKER = "worker"
    HYBRID = "hybrid"

    def __str__(self) -> str:  # "worker", not "AgentRole.WORKER" (App. A #37)
        return self.value


class AgentStatus(str, Enum):
    IDLE = "idle"
    BUSY = "busy"
    WAITING = "waiting"
    ERROR = "error"
    STOPPED = "stopped"

    def __str__(self) -> str:
        return self.value

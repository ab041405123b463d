"""Framework-level exceptions shared by the orchestrator and the node control plane."""


class AgentLostError(RuntimeError):
    """The agent executing a task disappeared before finishing it (its rank / GPU died or
    left the node). The task did not complete there; the orchestrator re-queues it on a
    surviving agent (parallel/node_plane.py, Serve._execute_task)."""

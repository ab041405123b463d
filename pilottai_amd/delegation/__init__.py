from .task_delegator import DelegationMetrics, TaskDelegator  # noqa: F401

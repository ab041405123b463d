"""Control-plane services that run against an orchestrator (Serve or a manager agent)."""
from .fault_tolerance import AgentHealth, FaultTolerance, FaultToleranceConfig, GPUHealthProbe, HealthStatus  # noqa: F401
from .load_balancer import LoadBalancer, LoadBalancerConfig, LoadMetrics  # noqa: F401
from .scaling import DynamicScaling, ScalingConfig, ScalingMetrics  # noqa: F401

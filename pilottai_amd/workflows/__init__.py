"""Ready-made multi-agent workflows built from the public API."""
from .document import STAGES, StageAgent, WorkflowManager, build_document_workflow  # noqa: F401

from .knowledge_manager import CacheEntry, KnowledgeManager  # noqa: F401
from pilottai_amd.tools.knowledge import KnowledgeSource  # noqa: F401

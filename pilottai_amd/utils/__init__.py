"""Logging, checkpointing and metrics utilities."""
from .logger import (CustomRotatingFileHandler, JsonFormatter, LogContext, add_log_context,  # noqa: F401
                     create_audit_logger, setup_log_cleanup, setup_logger)

"""Logging utilities (reference: pilott/utils/logger.py:14-207).

setup_logger: console text handler + optional JSON main/error logs rotated at
midnight (or by size) and gzip-compressed on rotation; LogContext / add_log_context
attach structured fields; create_audit_logger writes an append-only JSON audit
trail. Unlike the reference, the core classes use these utilities.
"""
from __future__ import annotations

import gzip
import json
import logging
import os
import shutil
import time
from logging.handlers import RotatingFileHandler, TimedRotatingFileHandler
from pathlib import Path
from typing import Any, Dict, Optional

from pilottai_amd.core.config import LogConfig


class CustomRotatingFileHandler(TimedRotatingFileHandler):
    """Timed rotation with gzip compression of rotated files."""

    def __init__(self, filename, when="midnight", backupCount=5, encoding="utf-8", **kw):
        super().__init__(filename, when=when, backupCount=backupCount, encoding=encoding, **kw)
        self.namer = lambda name: name + ".gz"
        self.rotator = self._gzip_rotator

    @staticmethod
    def _gzip_rotator(source: str, dest: str):
        with open(source, "rb") as fi, gzip.open(dest, "wb") as fo:
            shutil.copyfileobj(fi, fo)
        os.remove(source)


class JsonFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        d: Dict[str, Any] = {
            "timestamp": self.formatTime(record, "%Y-%m-%dT%H:%M:%S") + f".{int(record.msecs):03d}",
            "level": record.levelname, "logger": record.name, "message": record.getMessage(),
            "module": record.module, "function": record.funcName, "line": record.lineno,
        }
        ctx = getattr(record, "context", None)
        if ctx:
            d["context"] = ctx
        for k, v in record.__dict__.items():
            if k.startswith("ctx_"):
                d[k[4:]] = v
        if record.exc_info:
            d["exception"] = self.formatException(record.exc_info)
        return json.dumps(d, default=str)


def setup_logger(name: str, config: Optional[LogConfig] = None, agent_id: Optional[str] = None) -> logging.Logger:
    config = config or LogConfig()
    logger = logging.getLogger(name if agent_id is None else f"{name}.{agent_id}")
    logger.setLevel(logging.DEBUG if config.verbose else getattr(logging, config.log_level))
    logger.propagate = False
    for h in list(logger.handlers):
        logger.removeHandler(h)
    ch = logging.StreamHandler()
    ch.setFormatter(logging.Formatter(config.log_format))
    logger.addHandler(ch)
    if config.log_to_file:
        d = Path(config.log_dir)
        d.mkdir(parents=True, exist_ok=True)
        base = logger.name.replace("/", "_")
        if config.log_rotation in ("size", "bytes"):
            fh = RotatingFileHandler(d / f"{base}.log", maxBytes=config.max_file_size,
                                     backupCount=config.backup_count, encoding="utf-8")
        else:
            fh = CustomRotatingFileHandler(d / f"{base}.log", when=config.log_rotation,
                                           backupCount=config.backup_count)
        fh.setFormatter(JsonFormatter())
        logger.addHandler(fh)
        eh = CustomRotatingFileHandler(d / f"{base}.error.log", when="midnight", backupCount=config.backup_count)
        eh.setLevel(logging.ERROR)
        eh.setFormatter(JsonFormatter())
        logger.addHandler(eh)
    return logger


def setup_log_cleanup(log_dir, max_age_days: int = 30) -> int:
    """Delete rotated logs older than `max_age_days`; returns the number removed."""
    n = 0
    cutoff = time.time() - max_age_days * 86400
    for f in Path(log_dir).glob("*.gz"):
        if f.stat().st_mtime < cutoff:
            f.unlink()
            n += 1
    return n


class LogContext:
    """`with LogContext(logger, task_id=...):` adds fields to every record."""

    def __init__(self, logger: logging.Logger, **context):
        self.logger = logger
        self.context = context
        self._filter = None

    def __enter__(self):
        ctx = self.context

        class _F(logging.Filter):
            def filter(self, record):
                record.context = {**getattr(record, "context", {}), **ctx}
                return True

        self._filter = _F()
        self.logger.addFilter(self._filter)
        for h in self.logger.handlers:
            h.addFilter(self._filter)
        return self.logger

    def __exit__(self, *exc):
        self.logger.removeFilter(self._filter)
        for h in self.logger.handlers:
            h.removeFilter(self._filter)


def add_log_context(logger: logging.Logger, **context) -> logging.LoggerAdapter:
    class _A(logging.LoggerAdapter):
        def process(self, msg, kwargs):
            kwargs.setdefault("extra", {})["context"] = self.extra
            return msg, kwargs

    return _A(logger, context)


def create_audit_logger(log_dir="logs", name: str = "audit") -> logging.Logger:
    d = Path(log_dir)
    d.mkdir(parents=True, exist_ok=True)
    logger = logging.getLogger(f"pilottai_amd.{name}")
    logger.setLevel(logging.INFO)
    logger.propagate = False
    if not any(isinstance(h, CustomRotatingFileHandler) for h in logger.handlers):
        h = CustomRotatingFileHandler(d / f"{name}.log", when="midnight", backupCount=90)
        h.setFormatter(JsonFormatter())
        logger.addHandler(h)
    return logger

"""Prompt rules + robust JSON reply parsing (reference: pilott/pilott.py:29-66,603-639,
pilott/core/agent.py:32-56,397-402).

One PromptManager serves both agents and the orchestrator. Templates are valid
str.format templates and every placeholder is checked before formatting, so a
missing argument is a clear error instead of a KeyError deep inside format.
"""
from __future__ import annotations

import json
import re
import string
from functools import lru_cache
from pathlib import Path
from typing import Any, Dict, Optional

import yaml

RULES_PATH = Path(__file__).resolve().parent.parent / "source" / "rules.yaml"


@lru_cache(maxsize=4)
def load_rules(path: str = str(RULES_PATH)) -> Dict[str, Any]:
    with open(path, "r") as f:
        return yaml.safe_load(f)


class PromptManager:
    def __init__(self, section: str, rules: Optional[Dict[str, Any]] = None):
        self.section = section
        self.rules = rules or load_rules()
        if section not in self.rules:
            raise ValueError(f"rules file has no {section!r} section")

    def template(self, kind: str) -> str:
        sec = self.rules[self.section]
        if kind not in sec:
            raise ValueError(f"Invalid prompt type: {self.section}.{kind}")
        return sec[kind]

    @staticmethod
    def placeholders(template: str):
        return {f for _, f, _, _ in string.Formatter().parse(template) if f}

    def format_prompt(self, kind: str, **kwargs) -> str:
        tpl = self.template(kind)
        missing = self.placeholders(tpl) - set(kwargs)
        if missing:
            raise ValueError(f"Missing required parameters for {self.section}.{kind}: {sorted(missing)}")
        return tpl.format(**kwargs)

    def schema_name(self, kind: str) -> Optional[str]:
        name = f"{self.section}.{kind}"
        return name if name in self.rules.get("schemas", {}) else None


def _balanced_objects(s: str):
    """Yield substrings that are balanced {...} objects (string-aware)."""
    depth = 0
    start = -1
    in_str = False
    esc = False
    for i, c in enumerate(s):
        if in_str:
            if esc:
                esc = False
            elif c == "\\":
                esc = True
            elif c == '"':
                in_str = False
            continue
        if c == '"':
            in_str = True
        elif c == "{":
            if depth == 0:
                start = i
            depth += 1
        elif c == "}" and depth > 0:
            depth -= 1
            if depth == 0:
                yield s[start:i + 1]


def parse_json_response(response: Any) -> Dict[str, Any]:
    """Parse an LLM reply into a dict: accepts dict replies, ```json fences, bare
    objects embedded in prose (a working version of the reference's `(?R)`
    fallback, App. A #21)."""
    if isinstance(response, dict):
        if "content" in response and isinstance(response.get("content"), str):
            response = response["content"]
        else:
            return response
    if not isinstance(response, str):
        raise ValueError(f"Invalid JSON response: unsupported type {type(response).__name__}")
    text = response.strip()
    m = re.search(r"```(?:json)?\s*(.*?)```", text, re.S)
    if m:
        text = m.group(1).strip()
    try:
        obj = json.loads(text)
        if isinstance(obj, dict):
            return obj
    except json.JSONDecodeError:
        pass
    for cand in _balanced_objects(text):
        try:
            obj = json.loads(cand)
            if isinstance(obj, dict):
                return obj
        except json.JSONDecodeError:
            continue
    raise ValueError(f"Invalid JSON response: {response[:200]!r}")

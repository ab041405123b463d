"""Compile reply schemas (source/rules.yaml `schemas:`) into token-level grammars.

A compiled grammar is a list of segments understood by the native automaton
(csrc/runtime/grammar.h): forced literal token runs, one-token choices from a
mask class, bounded string bodies and bounded string lists. Mask classes are
rows of a GPU-resident bitmask tensor [classes, vocab/32] that the sampling
kernel applies in place (csrc/ops/sampling.hip).

`fixed` pins values by dotted path (e.g. ``{"next_step.tool": "echo"}``): the
orchestrator/agents use it for their deterministic control policy and for
fields only the caller can know (tool names), see core/llm_policy.py.
"""
from __future__ import annotations

import json
import re
import threading
from functools import lru_cache
from pathlib import Path
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import yaml

from .tokenizer import Tokenizer

LIT, CHOICE, STR, LIST = 0, 1, 2, 3
MAX_CLASSES = 64

Segment = Tuple[int, List[int], int, int, int, int, int, int, int]


@lru_cache(maxsize=1)
def load_schemas() -> Dict[str, Any]:
    path = Path(__file__).resolve().parent.parent / "source" / "rules.yaml"
    return yaml.safe_load(path.read_text()).get("schemas", {})


class MaskRegistry:
    """Named token classes -> bitmask rows (uploaded to the GPU by the engine)."""

    def __init__(self, tok: Tokenizer):
        self.tok = tok
        self._lock = threading.Lock()
        self.names: Dict[str, int] = {}
        self.rows: List[np.ndarray] = []
        self.version = 0
        self._safe = tok.string_safe_mask()
        self.quote = tok.token_id('"')
        self.list_sep = tok.token_id('", "')
        self.list_close = tok.token_id('"]')
        for t in (self.quote, self.list_sep, self.list_close):
            assert t >= 0
        self.cls_str = self._add("str", self._safe | self._onehot([self.quote]))
        self.cls_str_body = self._add("str_body", self._safe.copy())  # no closing quote: forced length
        self.cls_list = self._add("list", self._safe | self._onehot([self.list_sep, self.list_close]))
        self.cls_list_last = self._add("list_last", self._safe | self._onehot([self.list_close]))
        self.cls_bool = self.enum(["true", "false"])
        self.cls_any = -1

    def _onehot(self, ids: Sequence[int]) -> np.ndarray:
        m = np.zeros(self.tok.vocab_size, dtype=bool)
        m[list(ids)] = True
        return m

    def _add(self, name: str, mask: np.ndarray) -> int:
        with self._lock:
            if name in self.names:
                return self.names[name]
            if len(self.rows) >= MAX_CLASSES:
                raise RuntimeError("too many grammar mask classes")
            self.rows.append(mask)
            self.names[name] = len(self.rows) - 1
            self.version += 1
            return self.names[name]

    def enum(self, values: Sequence[str]) -> int:
        ids = []
        for v in values:
            t = self.tok.token_id(v)
            if t < 0:
                raise ValueError(f"enum value {v!r} is not a single vocabulary token")
            ids.append(t)
        return self._add("enum:" + "|".join(values), self._onehot(ids))

    def int_range(self, lo: int, hi: int) -> int:
        return self.enum([str(i) for i in range(lo, hi + 1)])

    def packed(self) -> np.ndarray:
        """int32 [len(rows), ceil(V/32)] packed bitmasks."""
        from pilottai_amd.ops.reference import pack_mask

        with self._lock:
            return np.stack([pack_mask(r).numpy() for r in self.rows])


_TYPE_RE = re.compile(r"^(\w+)\((.*)\)$")

# The free-text slot of each reply schema that `reply_tokens` resizes (the workload
# sensitivity knob of bench.py --reply-tokens); schemas without one get a trailing
# "notes" string. The reference's replies are unconstrained prose up to
# max_tokens=2000 (pilott/core/config.py:52); the default schemas keep them short.
REPLY_SLOTS = {
    "agent.task_analysis": "alignment",
    "agent.step_planning": "next_step.expected_outcome",
    "agent.result_evaluation": "reasoning",
    "workflow.summarize": "summary",
}


class GrammarCompiler:
    def __init__(self, tok: Tokenizer, reg: Optional[MaskRegistry] = None, reply_tokens: Optional[int] = None):
        self.tok = tok
        self.reg = reg or MaskRegistry(tok)
        # reply_tokens = N: every named schema's free-text slot (REPLY_SLOTS, else an added
        # "notes" field) is exactly N tokens long — N sampled tokens per call at least
        self.reply_tokens = int(reply_tokens) if reply_tokens else None
        self._cache: Dict[Tuple[str, str], List[Segment]] = {}
        self._lock = threading.Lock()
        # pre-register every class used by the shipped schemas so the GPU mask
        # table is complete before the first graph capture
        for name in load_schemas():
            self.compile(name)

    # -- public ---------------------------------------------------------------
    def compile(self, schema: Any, fixed: Optional[Dict[str, Any]] = None) -> List[Segment]:
        fixed = fixed or {}
        key = None
        if isinstance(schema, str):
            key = (schema, json.dumps(fixed, sort_keys=True, default=str))
            with self._lock:
                if key in self._cache:
                    return self._cache[key]
            spec = load_schemas()[schema]
        else:
            spec = schema
        reply = None
        if self.reply_tokens and isinstance(schema, str) and isinstance(spec, dict):
            reply = REPLY_SLOTS.get(schema)
            if reply is None:
                spec = {**spec, "notes": f"str({self.reply_tokens})"}
                reply = "notes"
        parts: List[Any] = []
        self._value(spec, "", fixed, parts, reply)
        segs = self._finalize(parts)
        if key is not None:
            with self._lock:
                self._cache[key] = segs
        return segs

    # -- internals --------------------------------------------------------------
    def _lit(self, parts, text: str):
        if parts and isinstance(parts[-1], str):
            parts[-1] += text
        else:
            parts.append(text)

    def _value(self, spec: Any, path: str, fixed: Dict[str, Any], parts: List[Any], reply: Optional[str] = None):
        if path in fixed:
            self._lit(parts, json.dumps(fixed[path]))
            return
        if isinstance(spec, dict):
            if "objlist" in spec:
                n = int(spec["objlist"])
                self._lit(parts, "[")
                for i in range(n):
                    if i:
                        self._lit(parts, ", ")
                    self._value(spec["item"], f"{path}[{i}]", fixed, parts, reply)
                self._lit(parts, "]")
                return
            self._lit(parts, "{")
            for i, (k, v) in enumerate(spec.items()):
                self._lit(parts, (", " if i else "") + json.dumps(str(k)) + ": ")
                self._value(v, f"{path}.{k}" if path else str(k), fixed, parts, reply)
            self._lit(parts, "}")
            return
        s = str(spec).strip()
        reg = self.reg
        if s == "bool":
            parts.append((CHOICE, [], reg.cls_bool, -1, -1, -1, 0, 1, 1))
            return
        m = _TYPE_RE.match(s)
        if not m:
            raise ValueError(f"bad schema type {s!r} at {path!r}")
        kind, arg = m.group(1), m.group(2).strip()
        if kind == "int":
            lo, hi = (int(x) for x in arg.split(","))
            parts.append((CHOICE, [], reg.int_range(lo, hi), -1, -1, -1, 0, 1, 1))
        elif kind == "str":
            self._lit(parts, '"')
            if reply is not None and path == reply:
                n = self.reply_tokens
                parts.append((STR, [], reg.cls_str, reg.cls_str_body, reg.quote, -1, n, n, 1))
            else:
                parts.append((STR, [], reg.cls_str, -1, reg.quote, -1, int(arg), 1, 1))
        elif kind == "enum":
            self._lit(parts, '"')
            parts.append((CHOICE, [], reg.enum(arg.split("|")), -1, -1, -1, 0, 1, 1))
            self._lit(parts, '"')
        elif kind == "list":
            if not arg:
                self._lit(parts, "[]")
                return
            im = re.match(r"^str\((\d+)\)\s*,\s*(\d+)\s*,\s*(\d+)$", arg)
            if not im:
                raise ValueError(f"unsupported list item {arg!r} at {path!r}")
            n, mn, mx = (int(x) for x in im.groups())
            if mx <= 0:
                self._lit(parts, "[]")
                return
            self._lit(parts, '["')
            parts.append((LIST, [], reg.cls_list, reg.cls_list_last, reg.list_close, reg.list_sep, n,
                          max(1, mn), mx))
        elif kind == "map":
            im = re.match(r"^str\((\d+)\)$", arg)
            n = int(im.group(1)) if im else 4
            self._lit(parts, '{"')
            parts.append((STR, [], reg.cls_str, -1, reg.quote, -1, max(1, n // 2), 1, 1))
            self._lit(parts, ': "')
            parts.append((STR, [], reg.cls_str, -1, reg.quote, -1, n, 1, 1))
            self._lit(parts, "}")
        elif kind == "obj":
            self._lit(parts, "{}")
        else:
            raise ValueError(f"unknown schema type {kind!r} at {path!r}")

    def _finalize(self, parts: List[Any]) -> List[Segment]:
        segs: List[Segment] = []
        for p in parts:
            if isinstance(p, str):
                segs.append((LIT, self.tok.encode(p), -1, -1, -1, -1, 0, 1, 1))
            else:
                segs.append(p)
        return segs


def max_output_tokens(segs: Sequence[Segment]) -> int:
    """Upper bound on the tokens a grammar can emit (sizes max_tokens)."""
    n = 0
    for kind, toks, _c, _cl, _e, _s, mt, _mn, mx in segs:
        if kind == LIT:
            n += len(toks)
        elif kind == CHOICE:
            n += 1
        elif kind == STR:
            n += mt + 1
        elif kind == LIST:
            n += mx * (mt + 1)
    return n

"""Task / memory checkpoint and resume (SURVEY §5 "Checkpoint / resume", App. D).

A checkpoint is a directory:
    state.json        versioned JSON: orchestrator config, every Task (reference
                      `Task.to_dict()` form), completed / failed TaskResults, the
                      pending task ids, orchestrator Memory (MemoryEntry form) and
                      each agent's AgentConfig + EnhancedMemory (MemoryItem form)
    index_<k>/        every distinct semantic index the agents' EnhancedMemories use
                      (SemanticIndex.save: packed.npy = the fragment-major bf16 rows as
                      uint16, priority/tagbits/expiry.npy, meta.json), streamed from the
                      device in chunks; each agent entry names its index ("index_ref") and
                      every MemoryItem its row, so resume needs no re-embedding
Writes go to a temp dir that is renamed into place, so a crash never leaves a
half-written checkpoint. Only JSON and .npy (allow_pickle=False) are read back.
"""
from __future__ import annotations

import asyncio
import json
import os
import shutil
import tempfile
from datetime import datetime
from pathlib import Path
from typing import Any, Dict

FORMAT_VERSION = 1


def _task_json(t) -> Dict[str, Any]:
    d = t.model_dump(mode="json", exclude_none=True)
    d["metadata"] = {k: v for k, v in d.get("metadata", {}).items() if not str(k).startswith("_")}
    return d


def save_serve_checkpoint(serve, path, save_index: bool = True) -> str:
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    tmp = Path(tempfile.mkdtemp(prefix=".ckpt-", dir=str(path.parent)))
    pending = [tid for tid, t in serve.tasks.items()
               if tid not in serve.completed_tasks and tid not in serve.failed_tasks and not t.subtasks]
    agents = []
    indexes: Dict[int, int] = {}  # id(SemanticIndex) -> k (agents may share one store)
    index_stats = []
    for a in serve.agents.values():
        cfg = getattr(a, "config", None)
        entry = {"id": a.id, "type": type(a).__name__, "config": cfg.to_dict() if hasattr(cfg, "to_dict") else {}}
        mem = getattr(a, "_memory", None)
        if mem is not None and hasattr(mem, "to_dict"):
            entry["enhanced_memory"] = mem.to_dict()
            idx = getattr(mem, "index", None)
            if save_index and idx is not None and hasattr(idx, "save"):
                if id(idx) not in indexes:
                    indexes[id(idx)] = k = len(indexes)
                    index_stats.append(dict(idx.save(tmp / f"index_{k}"), index=k))
                entry["index_ref"] = indexes[id(idx)]
        agents.append(entry)
    state = {
        "format_version": FORMAT_VERSION,
        "saved_at": datetime.now().isoformat(),
        "serve": serve.config.model_dump(mode="json"),
        "tasks": [_task_json(t) for t in serve.tasks.values()],
        "pending": pending,
        "completed": {k: v.model_dump(mode="json") for k, v in serve.completed_tasks.items()},
        "failed": {k: v.model_dump(mode="json") for k, v in serve.failed_tasks.items()},
        "memory": serve.memory.to_dict() if serve.memory is not None else None,
        "metrics": dict(serve.metrics),
        "agents": agents,
        "indexes": index_stats,
    }
    (tmp / "state.json").write_text(json.dumps(state, indent=1, default=str))
    # crash-safe swap: the previous checkpoint is renamed aside (not deleted) until the new
    # one is in place; a crash between the two renames leaves it at <path>.bak, which
    # load_checkpoint falls back to
    bak = path.with_name(path.name + ".bak")
    if path.exists():
        if bak.exists():
            shutil.rmtree(bak)  # <path> is a complete checkpoint: the older .bak is redundant
        os.replace(path, bak)
    # else: an earlier save was interrupted between its renames and <path>.bak is the only good
    # checkpoint -- keep it until the new one is in place
    os.replace(tmp, path)
    if bak.exists():
        shutil.rmtree(bak)
    return str(path)


def load_checkpoint(path) -> Dict[str, Any]:
    path = Path(path)
    f = path / "state.json"
    if not f.exists():
        bak = path.with_name(path.name + ".bak") / "state.json"
        if bak.exists():  # interrupted swap (save_serve_checkpoint): the previous checkpoint
            f = bak
    st = json.loads(f.read_text())
    if st.get("format_version") != FORMAT_VERSION:
        raise ValueError(f"unsupported checkpoint format {st.get('format_version')}")
    return st


async def restore_serve_checkpoint(serve, path, requeue: bool = True) -> int:
    """Restore results, memory and tasks into `serve`; re-queue pending tasks."""
    from pilottai_amd.core.memory import Memory
    from pilottai_amd.core.task import Task, TaskResult

    st = load_checkpoint(path)
    for k, v in st["completed"].items():
        serve.completed_tasks[k] = TaskResult(**v)
    for k, v in st["failed"].items():
        serve.failed_tasks[k] = TaskResult(**v)
    if st.get("memory") is not None and serve.memory is not None:
        serve.memory = Memory.from_dict(st["memory"])
    by_id = {}
    for td in st["tasks"]:
        td = dict(td)
        if td.get("deadline") and datetime.fromisoformat(td["deadline"]) < datetime.now():
            td.pop("deadline")  # an expired deadline cannot be re-validated; the task is restored without it
        t = Task(**td)
        by_id[t.id] = t
        serve.tasks[t.id] = t
    saved_agents = {a["id"]: a for a in st.get("agents", [])}
    # a restarted process has new agent ids: fall back to the role (Serve keys agents by role,
    # reference pilott/pilott.py:93), each saved entry used once
    by_role: Dict[str, list] = {}
    for e in st.get("agents", []):
        by_role.setdefault(str(e.get("config", {}).get("role")), []).append(e)
    used = set()
    root = Path(path) if (Path(path) / "state.json").exists() else Path(path).with_name(Path(path).name + ".bak")
    restored: Dict[int, Any] = {}  # index_ref -> SemanticIndex loaded from the checkpoint
    for a in serve.agents.values():
        s = saved_agents.get(a.id)
        if s is None:
            role = str(getattr(getattr(a, "config", None), "role", None))
            s = next((e for e in by_role.get(role, []) if e["id"] not in used and e["id"] not in
                      {x.id for x in serve.agents.values()}), None)
        if s is not None:
            used.add(s["id"])
        if s and "enhanced_memory" in s:
            mem = a.enhanced_memory
            k = s.get("index_ref")
            ok = False
            if k is not None and (root / f"index_{k}" / "meta.json").exists():
                if k not in restored:
                    from pilottai_amd.memory.semantic_index import SemanticIndex

                    cur = mem.index
                    restored[k] = SemanticIndex.load(root / f"index_{k}", device=cur.device,
                                                     growable=cur.growable, max_capacity=cur.max_capacity)
                mem.index = restored[k]
                ok = True
            await mem.load_dict(s["enhanced_memory"], index_restored=ok)
    n = 0
    if requeue:
        if not serve._started:
            await serve.start()
        for tid in st["pending"]:
            t = by_id.get(tid)
            if t is None:
                continue
            t.status = t.status.__class__("pending")
            serve._futures.setdefault(t.id, asyncio.get_running_loop().create_future())
            await serve._enqueue(t)
            n += 1
    return n

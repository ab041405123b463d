"""Task / memory checkpoint and resume (SURVEY §5 "Checkpoint / resume", App. D).

A checkpoint is a directory:
    state.json        versioned JSON: orchestrator config, every Task (reference
                      `Task.to_dict()` form), completed / failed TaskResults, the
                      pending task ids, orchestrator Memory (MemoryEntry form) and
                      each agent's AgentConfig + EnhancedMemory (MemoryItem form)
    index.npy         optional raw semantic-index shard (bf16 rows as uint16,
                      numpy header -> np.load(mmap_mode="r") then one H2D copy)
    index_meta.json   row metadata for index.npy
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

import numpy as np

FORMAT_VERSION = 1


def _task_json(t) -> Dict[str, Any]:
    d = t.model_dump(mode="json", exclude_none=True)
    d["metadata"] = {k: v for k, v in d.get("metadata", {}).items() if not str(k).startswith("_")}
    return d


def save_serve_checkpoint(serve, path) -> str:
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    tmp = Path(tempfile.mkdtemp(prefix=".ckpt-", dir=str(path.parent)))
    pending = [tid for tid, t in serve.tasks.items()
               if tid not in serve.completed_tasks and tid not in serve.failed_tasks and not t.subtasks]
    agents = []
    for a in serve.agents.values():
        cfg = getattr(a, "config", None)
        entry = {"id": a.id, "type": type(a).__name__, "config": cfg.to_dict() if hasattr(cfg, "to_dict") else {}}
        mem = getattr(a, "_memory", None)
        if mem is not None and hasattr(mem, "to_dict"):
            entry["enhanced_memory"] = mem.to_dict()
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
    for a in serve.agents.values():
        s = saved_agents.get(a.id)
        if s and "enhanced_memory" in s:
            await a.enhanced_memory.load_dict(s["enhanced_memory"])
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


def save_index(index, path) -> str:
    """Dump a SemanticIndex to index.npy (+ index_meta.json) for mmap reload."""
    path = Path(path)
    path.mkdir(parents=True, exist_ok=True)
    n = index.count
    vec = index.read_rows(0, n).contiguous().view(dtype=__import__("torch").int16).cpu().numpy().view(np.uint16)
    np.save(path / "index.npy", vec, allow_pickle=False)
    meta = {"dim": index.dim, "count": n, "size": index.size, "epoch": index.epoch,
            "priority": index.priority[:n].cpu().tolist(), "tagbits": index.tagbits[:n].cpu().tolist(),
            "expiry": index.expiry[:n].cpu().tolist(), "tags": index.tags.bits,
            "row_tags": {str(k): sorted(v) for k, v in index.row_tags_py.items()}}
    (path / "index_meta.json").write_text(json.dumps(meta))
    return str(path)


def load_index(path, device=None):
    import torch

    from pilottai_amd.memory.semantic_index import SemanticIndex

    path = Path(path)
    meta = json.loads((path / "index_meta.json").read_text())
    arr = np.load(path / "index.npy", mmap_mode="r", allow_pickle=False)
    n = meta["count"]
    idx = SemanticIndex(dim=meta["dim"], capacity=max(1, n), device=device)
    idx.write_range(0, torch.from_numpy(np.ascontiguousarray(arr).view(np.int16)).view(torch.bfloat16))
    idx.priority[:n] = torch.tensor(meta["priority"], dtype=torch.int32)
    idx.tagbits[:n] = torch.tensor(meta["tagbits"], dtype=torch.int64)
    idx.expiry[:n] = torch.tensor(meta["expiry"], dtype=torch.float32)
    idx.size = meta["size"]
    idx.epoch = meta["epoch"]
    idx.tags.bits = dict(meta["tags"])
    idx.row_tags_py = {int(k): frozenset(v) for k, v in meta["row_tags"].items()}
    return idx

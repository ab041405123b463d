"""Agents of the hierarchical PDF pipeline (reference:
docs/examples/pdf_processing/example_agents.py:13-415).

    Manager ──► Extractor (pdf_extractor tool)
            ──► Evaluator (structure checks + LLM quality verdict, JSON schema)
            ──► Generator (LLM analysis over the text, semantic memory of past runs)

Differences from the reference, by design: the manager awaits each child's
`execute_task` instead of polling an unprocessed queue (reference
`_wait_for_task`, :85-102, never sees a result because nothing drains
`agent.tasks`), every agent returns a `TaskResult`, and all LLM calls go to the
on-node engine (grammar-constrained where the reply is parsed).
"""
from __future__ import annotations

import json
import time
from datetime import datetime
from typing import Any, Dict, Union

from pilottai_amd.core.agent import BaseAgent
from pilottai_amd.core.task import Task, TaskResult

from .pdf_extractor import PDFExtractorTool


def _task(task: Union[Task, Dict[str, Any]]) -> Task:
    return Task.from_any(task)


class ManagerAgent(BaseAgent):
    async def evaluate_task_suitability(self, task) -> float:
        return 1.0

    def _child(self, cls_name: str) -> BaseAgent:
        for a in self.child_agents.values():
            if type(a).__name__ == cls_name:
                return a
        raise ValueError(f"Required agent type {cls_name} not found")

    async def execute_task(self, task) -> TaskResult:
        task = _task(task)
        t0 = time.perf_counter()
        path = task.metadata.get("file_path")
        extraction = await self._child("ExtractorAgent").execute_task(
            Task(description=f"Extract the text of {path}", metadata={"type": "extract", "file_path": path}))
        if not extraction.success:
            return TaskResult(success=False, error="Extraction failed", output={"details": extraction.output},
                              execution_time=time.perf_counter() - t0)
        evaluation = await self._child("EvaluatorAgent").execute_task(
            Task(description="Validate the extracted content",
                 metadata={"type": "evaluate", "content": extraction.output}))
        generation: Dict[str, Any] = {"status": "skipped"}
        if evaluation.success and (evaluation.output or {}).get("is_valid_json"):
            g = await self._child("GeneratorAgent").execute_task(
                Task(description="Analyse the document", metadata={"type": "generate", "content": extraction.output}))
            generation = g.output if g.success else {"status": "error", "error": g.error}
        return TaskResult(success=True, execution_time=time.perf_counter() - t0,
                          output={"status": "success", "extraction": extraction.output,
                                  "evaluation": evaluation.output, "generation": generation})


class ExtractorAgent(BaseAgent):
    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.add_tool(PDFExtractorTool())

    async def evaluate_task_suitability(self, task) -> float:
        return 1.0 if _task(task).metadata.get("type") == "extract" else 0.0

    async def execute_task(self, task) -> TaskResult:
        task = _task(task)
        t0 = time.perf_counter()
        res = await self.tools["pdf_extractor"].execute(file_path=str(task.metadata.get("file_path")))
        ok = res.get("status") == "success"
        out = {"status": res.get("status"), "content": res.get("content", {}),
               "metadata": {"filename": res.get("filename"), "total_pages": res.get("total_pages", 0)}}
        return TaskResult(success=ok, output=out, error=None if ok else res.get("error"),
                          execution_time=time.perf_counter() - t0)


class EvaluatorAgent(BaseAgent):
    async def evaluate_task_suitability(self, task) -> float:
        return 1.0 if _task(task).metadata.get("type") == "evaluate" else 0.0

    async def execute_task(self, task) -> TaskResult:
        task = _task(task)
        t0 = time.perf_counter()
        content = task.metadata.get("content") or {}
        checks = {
            "is_valid_json": _json_roundtrips(content),
            "has_content": bool(content.get("content")),
            "has_metadata": bool(content.get("metadata")),
        }
        # LLM verdict on the extraction (schema-constrained: always parseable)
        verdict = await self._llm_json("result_evaluation", task_description=task.description,
                                       result=json.dumps(content)[:2000])
        out = {**checks, "llm_verdict": verdict, "timestamp": datetime.now().isoformat()}
        return TaskResult(success=checks["is_valid_json"], output=out, execution_time=time.perf_counter() - t0)


class GeneratorAgent(BaseAgent):
    async def evaluate_task_suitability(self, task) -> float:
        return 1.0 if _task(task).metadata.get("type") == "generate" else 0.0

    async def execute_task(self, task) -> TaskResult:
        task = _task(task)
        t0 = time.perf_counter()
        content = task.metadata.get("content") or {}
        if not content:
            return TaskResult(success=False, error="No content provided for generation")
        mem = self.enhanced_memory
        similar = await mem.semantic_search(json.dumps(content)[:4000], limit=5) if len(mem) else []
        text = _prepare_text(content)
        messages = [{"role": "system", "content": f"Goal: {self.config.goal}. "
                                                  "Generate insights based on the provided content."},
                    {"role": "user", "content": text}]
        resp = await self.llm.generate_response(messages)
        result = {"status": "success", "content": resp.get("content", ""), "timestamp": datetime.now().isoformat(),
                  "metadata": {"similar_docs_found": len(similar), "input_length": len(text)}}
        await mem.store_semantic(json.dumps(result), {"type": "generation_result"})
        return TaskResult(success=True, output=result, execution_time=time.perf_counter() - t0)


def _json_roundtrips(obj: Any) -> bool:
    try:
        return json.loads(json.dumps(obj)) == obj
    except (TypeError, ValueError):
        return False


def _prepare_text(content: Dict[str, Any]) -> str:
    md = content.get("metadata", {})
    parts = [f"Document: {md.get('filename', 'Unknown')}", f"Total Pages: {md.get('total_pages', 0)}", "\nContent:"]
    for page, txt in sorted((content.get("content") or {}).items()):
        if isinstance(txt, str) and txt:
            parts.append(f"\n{page}: {txt.strip()}")
    return "\n".join(parts)

"""Hierarchical PDF pipeline on the on-node engine (reference:
docs/examples/pdf_processing/main.py:1-103).

    python -m examples.pdf_processing.main [--pdf file.pdf] [--model llama-3-8b] [--provider local]

Without --pdf a two-page sample is generated. On a machine without a GPU the
`tiny` test model runs on the CPU; `--provider schema` needs no model at all.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import tempfile
from typing import Dict, Optional

from pilottai_amd import Serve
from pilottai_amd.core.config import AgentConfig, LLMConfig
from pilottai_amd.core.role import AgentRole
from pilottai_amd.engine.llm_handler import LLMHandler
from pilottai_amd.tools import pdf

from .example_agents import EvaluatorAgent, ExtractorAgent, GeneratorAgent, ManagerAgent


def create_llm_config(model: str = "llama-3-8b", provider: str = "local") -> LLMConfig:
    return LLMConfig(model_name=model, provider=provider, temperature=0.7, max_tokens=256)


async def setup_pipeline(llm_config: Optional[LLMConfig] = None) -> Serve:
    llm_config = llm_config or create_llm_config()
    llm = LLMHandler(llm_config)  # one engine-backed handle shared by every agent
    cfgs = {
        "manager": AgentConfig(role="manager", role_type=AgentRole.ORCHESTRATOR,
                               goal="Manage PDF processing workflow",
                               description="Coordinates PDF extraction and validation", can_delegate=True),
        "extractor": AgentConfig(role="extractor", role_type=AgentRole.WORKER, goal="Extract content from PDFs",
                                 description="Processes PDF files and extracts content"),
        "evaluator": AgentConfig(role="evaluator", role_type=AgentRole.WORKER, goal="Validate extraction results",
                                 description="Ensures extraction output is valid JSON"),
        "generator": AgentConfig(role="Content Analyzer", role_type=AgentRole.WORKER,
                                 goal="Analyze PDF content and provide insights",
                                 description="Analyzes documents and provides detailed summaries",
                                 memory_enabled=True),
    }
    manager = ManagerAgent(cfgs["manager"], llm=llm)
    for cls, key in ((ExtractorAgent, "extractor"), (EvaluatorAgent, "evaluator"), (GeneratorAgent, "generator")):
        await manager.add_child_agent(cls(cfgs[key], llm=llm))
    serve = Serve(name="PDF Processing System", verbose=False,
                  config={"analyze_tasks": False, "evaluate_results": False})
    await serve.add_agent(manager)
    await serve.start()
    return serve


async def process_pdf(pdf_path: str, llm_config: Optional[LLMConfig] = None) -> Dict:
    if not os.path.exists(pdf_path):
        raise FileNotFoundError(f"PDF not found: {pdf_path}")
    serve = await setup_pipeline(llm_config)
    try:
        result = await serve.execute_task({"type": "process_pdf", "file_path": pdf_path})
        return result.output if result.success else {"status": "error", "error": result.error}
    finally:
        await serve.stop()


def sample_pdf(path: str) -> str:
    pdf.write_simple_pdf(path, [
        "Quarterly operations report\nRevenue grew 12 percent quarter over quarter.\nTwo incidents were mitigated.",
        "Outlook\nHiring continues in the platform team.\nSupply chain risk is moderate.",
    ])
    return path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pdf")
    ap.add_argument("--model", default=None)
    ap.add_argument("--provider", default="local", choices=["local", "schema"])
    a = ap.parse_args()
    import torch

    model = a.model or ("llama-3-8b" if torch.cuda.is_available() else "tiny")
    path = a.pdf or sample_pdf(os.path.join(tempfile.mkdtemp(), "sample_doc.pdf"))
    out = asyncio.run(process_pdf(path, create_llm_config(model, a.provider)))
    print(json.dumps(out, indent=2, default=str)[:4000])
    from pilottai_amd.engine.registry import shutdown_engines

    shutdown_engines()


if __name__ == "__main__":
    main()

"""PDF extraction tool (reference: docs/examples/pdf_processing/pdf_extractor.py:1-40).

Uses the framework's dependency-free extractor (pilottai_amd/tools/pdf.py) in
place of pypdf; same result shape: {status, filename, total_pages, content}.
"""
from __future__ import annotations

import asyncio
from typing import Any, Dict

from pilottai_amd.tools import pdf
from pilottai_amd.tools.tool import Tool


async def _extract(file_path: str) -> Dict[str, Any]:
    try:
        out = await asyncio.to_thread(pdf.extract_file, file_path)
        return {"status": "success", **out}
    except Exception as e:  # noqa: BLE001 — reported, as in the reference tool
        return {"status": "error", "error": str(e)}


def PDFExtractorTool() -> Tool:
    return Tool(name="pdf_extractor", description="Extracts text from PDFs", function=_extract,
                parameters={"file_path": {"type": "string", "description": "Path to PDF file"}},
                max_retries=1, timeout=60.0)

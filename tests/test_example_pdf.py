"""The hierarchical PDF example end to end on CPU, plus the PDF
text extractor on generated files and on the reference's sample PDF (read as
plain bytes; skipped when the reference tree is absent)."""
import asyncio
import os

import pytest

from pilottai_amd.tools import pdf

REF_SAMPLE = "/root/reference/docs/examples/pdf_processing/sample_doc.pdf"


def test_pdf_roundtrip(tmp_path):
    p = str(tmp_path / "a.pdf")
    pdf.write_simple_pdf(p, ["Line one (with parens) \\ and a backslash\nSecond line", "Page two"])
    out = pdf.extract_file(p)
    assert out["total_pages"] == 2
    assert out["content"]["page_1"] == "Line one (with parens) \\ and a backslash\nSecond line"
    assert out["content"]["page_2"] == "Page two"
    # uncompressed streams parse too
    pdf.write_simple_pdf(p, ["plain"], compress=False)
    assert pdf.extract_text(open(p, "rb").read()) == ["plain"]


@pytest.mark.skipif(not os.path.exists(REF_SAMPLE), reason="reference sample not present")
def test_reference_sample_pdf_cid_font():
    # Type0 / Identity-H font with a ToUnicode CMap, glyph-by-glyph positioning
    assert pdf.extract_text(open(REF_SAMPLE, "rb").read()) == ["What is the capital of india?"]


@pytest.mark.parametrize("provider,model", [("schema", "tiny"), ("local", "tiny")])
def test_pdf_pipeline_end_to_end(tmp_path, provider, model):
    from examples.pdf_processing.main import create_llm_config, process_pdf, sample_pdf
    from pilottai_amd.engine.registry import shutdown_engines

    path = sample_pdf(str(tmp_path / "doc.pdf"))
    try:
        out = asyncio.run(process_pdf(path, create_llm_config(model, provider)))
    finally:
        shutdown_engines()
    assert out["status"] == "success"
    assert out["extraction"]["metadata"]["total_pages"] == 2
    assert "Revenue grew 12 percent" in out["extraction"]["content"]["page_1"]
    ev = out["evaluation"]
    assert ev["is_valid_json"] and ev["has_content"]
    assert set(ev["llm_verdict"]) >= {"success", "quality_score"}
    gen = out["generation"]
    assert gen["status"] == "success" and gen["metadata"]["input_length"] > 50

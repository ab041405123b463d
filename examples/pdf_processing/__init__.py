"""Hierarchical PDF pipeline example (reference: docs/examples/pdf_processing/)."""

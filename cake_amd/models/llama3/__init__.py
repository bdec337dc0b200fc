"""Llama-3 text model (cake-core/src/models/llama3)."""

"""Stable Diffusion 1.5 / 2.1 / XL / Turbo (cake-core/src/models/sd)."""

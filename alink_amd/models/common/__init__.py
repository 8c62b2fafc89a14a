"""Shared model-side utilities (device feature matrices, statistics)."""

"""Evaluation metrics and summaries."""

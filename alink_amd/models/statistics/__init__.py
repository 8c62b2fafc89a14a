"""Statistics: summaries, correlation, hypothesis tests."""

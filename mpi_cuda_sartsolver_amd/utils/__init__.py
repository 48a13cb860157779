"""Configuration, timing/profiling and synthetic-problem helpers."""

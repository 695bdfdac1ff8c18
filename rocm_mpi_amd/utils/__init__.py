"""Metrics (T_eff), visualisation, profiling, checkpointing, config helpers."""

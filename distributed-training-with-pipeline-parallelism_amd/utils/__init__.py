"""Utilities: profiling/timeline + bubble accounting, checkpointing, metrics, launch."""

"""Benchmarks: reference-compatible API, sweeps, reports."""

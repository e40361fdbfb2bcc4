"""Utilities: profiling / tracing (profiling.py) and fault injection (faults.py)."""

"""Utilities: profiling / tracing (profiling.py), fault injection (faults.py),
throughput monitoring and the Prometheus exporter (metrics.py)."""

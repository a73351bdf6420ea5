"""Observability: throughput meter, roctx ranges, structured logs, profiler helpers."""

"""Golden-vector generation shim: memory_profiler is only used with --track_mem (src/utils.py:292)."""


def memory_usage(*a, **k):
    raise RuntimeError("memory_profiler is not available in this image")

"""Tracing and timing: roctx ranges visible in rocprofv3 traces, plus wall-clock
accumulators (the reference's ``tm`` tables, asyncsgd/goot.lua:24-26, BiCNN/bicnn.lua:17-28).

``range("name")`` emits roctxRangePushA/Pop through the rocprofiler-sdk roctx library (the
one rocprofv3 ``--marker-trace`` intercepts on ROCm 7; libroctx64 as fallback) when it is present and
tracing is enabled (``MPIT_TRACE=1`` or ``Pcontrol(1)``); it is a no-op otherwise.
``Timers`` accumulate seconds per key; ``device=True`` timers synchronise the GPU first
so they measure device time, not launch time.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time
from collections import defaultdict

_lib = None
_enabled = os.environ.get("MPIT_TRACE", "0") == "1"


def _roctx():
    global _lib
    if _lib is None:
        _lib = False
        for name in ("librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1",
                     "libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _lib = lib
                break
            except OSError:
                continue
    return _lib or None


def enable(flag: bool = True):
    global _enabled
    _enabled = bool(flag)


def enabled() -> bool:
    return _enabled


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    lib = _roctx() if _enabled else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def mark(name: str):
    lib = _roctx() if _enabled else None
    if lib is not None:
        lib.roctxMarkA(name.encode())


class Timers:
    def __init__(self):
        self.total = defaultdict(float)
        self.count = defaultdict(int)

    @contextlib.contextmanager
    def __call__(self, key: str, device: bool = False):
        if device:
            import torch

            if torch.cuda.is_available():
                torch.cuda.synchronize()
        t0 = time.perf_counter()
        with range(key):
            yield
        if device:
            import torch

            if torch.cuda.is_available():
                torch.cuda.synchronize()
        self.total[key] += time.perf_counter() - t0
        self.count[key] += 1

    def add(self, key: str, seconds: float):
        self.total[key] += seconds
        self.count[key] += 1

    def summary(self) -> dict:
        return {k: {"total_s": round(v, 6), "calls": self.count[k], "avg_ms": round(1000 * v / max(1, self.count[k]), 4)}
                for k, v in sorted(self.total.items())}

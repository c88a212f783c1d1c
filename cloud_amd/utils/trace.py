"""roctx ranges for rocprofv3 timelines.

``with trace.range("fwd"): ...`` pushes/pops a roctx range (``libroctx64``)
around the data load, forward, backward, bucket all-reduce and optimizer step,
so ``rocprofv3 --marker-trace`` (or ``run(..., profile=True)``) shows the
framework phases above the kernels.  Disabled unless ``CLOUD_AMD_TRACE=1``; when
disabled, or when libroctx64 is missing, ranges cost one attribute lookup.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

_lib = None
_enabled = None


def enabled() -> bool:
    global _enabled, _lib
    if _enabled is None:
        _enabled = os.environ.get("CLOUD_AMD_TRACE", "0") == "1"
        if _enabled:
            try:
                _lib = ctypes.CDLL("libroctx64.so")
                _lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                _lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            except OSError:
                _enabled = False
    return _enabled


def push(name: str):
    if enabled():
        _lib.roctxRangePushA(name.encode())


def pop():
    if enabled():
        _lib.roctxRangePop()


def mark(name: str):
    if enabled():
        _lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    if not enabled():
        yield
        return
    _lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        _lib.roctxRangePop()

"""ROCTx ranges + per-failure stage timestamps.

``trace_range("scan")`` pushes/pops a roctx range (visible in
``rocprofv3 --marker-trace`` timelines) when ``libroctx64`` is loadable, and is
a no-op otherwise. ``StageClock`` records detect -> collect -> scan -> prefill
-> decode -> store timestamps for one failure; the pipeline feeds them into the
Prometheus stage histograms.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time

_lib = None
_tried = False


def _roctx():
    global _lib, _tried
    if _tried:
        return _lib
    _tried = True
    if os.environ.get("OAMD_ROCTX", "1") == "0":
        return None
    # rocprofv3 (rocprofiler-sdk) intercepts the SDK's roctx; the legacy roctracer
    # libroctx64 (also bundled with torch) is only a fallback for older tools
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cands = [os.path.join(rocm, "lib", "librocprofiler-sdk-roctx.so"), "librocprofiler-sdk-roctx.so",
             "libroctx64.so", os.path.join(rocm, "lib", "libroctx64.so")]
    try:
        import torch

        cands.append(os.path.join(os.path.dirname(torch.__file__), "lib", "libroctx64.so"))
    except Exception:  # noqa: BLE001
        pass
    for c in cands:
        try:
            lib = ctypes.CDLL(c)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _lib = lib
            break
        except (OSError, AttributeError):
            continue
    return _lib


@contextlib.contextmanager
def trace_range(name: str):
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxMarkA(name.encode())


class StageClock:
    __slots__ = ("t0", "stamps")

    def __init__(self):
        self.t0 = time.perf_counter()
        self.stamps: list[tuple[str, float]] = []

    def stamp(self, stage: str) -> float:
        t = time.perf_counter()
        self.stamps.append((stage, t))
        return t

    def durations(self) -> dict[str, float]:
        out, prev = {}, self.t0
        for name, t in self.stamps:
            out[name] = t - prev
            prev = t
        return out

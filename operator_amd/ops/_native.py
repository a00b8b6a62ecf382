"""Loader for the in-tree native extensions.

The gfx950 kernel module (``operator_amd._C``) is REQUIRED whenever a GPU tensor
reaches an op: there is no silent eager fallback on the device. CPU tensors use
the plain-PyTorch reference implementations (operator_amd.ops.reference), which
exist for the CPU test tier and for numerics checks of the HIP kernels.
"""
from __future__ import annotations

import importlib
import os
import threading

import torch  # noqa: F401  (must be imported before _C: one HIP runtime per process)

_lock = threading.Lock()
_C = None
_P = None
_err: Exception | None = None


def _try_build() -> None:
    if os.environ.get("OAMD_NO_AUTOBUILD"):
        return
    from operator_amd import _build

    _build.build()


def kernels():
    """Return the compiled gfx950 kernel module, building it in-tree if needed."""
    global _C, _err
    if _C is not None:
        return _C
    with _lock:
        if _C is not None:
            return _C
        try:
            _C = importlib.import_module("operator_amd._C")
        except ImportError as e:  # not built yet
            try:
                _try_build()
                _C = importlib.import_module("operator_amd._C")
            except Exception as e2:  # pragma: no cover - exercised only without hipcc
                _err = e2
                raise RuntimeError(f"operator_amd._C (gfx950 kernels) unavailable: {e2}") from e
    return _C


def patterns():
    """Return the CPU pattern compiler / packer / scorer module."""
    global _P
    if _P is not None:
        return _P
    with _lock:
        if _P is None:
            try:
                _P = importlib.import_module("operator_amd._patterns")
            except ImportError:
                from operator_amd import _build

                _build.build_patterns()
                _P = importlib.import_module("operator_amd._patterns")
    return _P


def native_available() -> bool:
    try:
        kernels()
        return True
    except Exception:
        return False

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


def _check_fresh(mod_name: str, src_globs: tuple[str, ...]) -> None:
    """Refuse an in-tree extension older than any of its sources: a GPU run of stale
    kernels (e.g. a host-side contract the old binary does not implement) can fault the
    device. OAMD_ALLOW_STALE=1 skips the check."""
    if os.environ.get("OAMD_ALLOW_STALE"):
        return
    import glob

    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    so = glob.glob(os.path.join(root, "operator_amd", mod_name + ".*.so"))
    if not so:
        return
    built = min(os.path.getmtime(f) for f in so)
    srcs = [f for g in src_globs for f in glob.glob(os.path.join(root, g))]
    newer = [os.path.relpath(f, root) for f in srcs if os.path.getmtime(f) > built + 1.0]
    if newer:
        raise RuntimeError(f"operator_amd.{mod_name} is older than {newer[:4]}: rebuild with "
                           "`python -m operator_amd._build` (or set OAMD_ALLOW_STALE=1)")


def kernels():
    """Return the compiled gfx950 kernel module, building it in-tree if needed."""
    global _C, _err
    if _C is not None:
        return _C
    with _lock:
        if _C is not None:
            return _C
        _check_fresh("_C", ("csrc/kernels/*", "csrc/*.cpp"))
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
            _check_fresh("_patterns", ("csrc/patterns/*",))
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

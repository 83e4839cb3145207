"""Loader for the in-tree native extensions.

The GPU path never falls back silently: if a CUDA/HIP tensor reaches an op and
``_fm_hip`` is missing or was built for another architecture, the op raises.
(The reference loads one TF op library the same way, tffm/fm_ops.py:5-8.)
"""

from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mods: dict[str, object] = {}


class NativeExtensionError(RuntimeError):
    pass


def _load(name: str, build_kind: str):
    with _lock:
        if name in _mods:
            return _mods[name]
        try:
            mod = importlib.import_module(f"fast_tffm_amd._native.{name}")
        except ImportError as first:
            if os.environ.get("FM_NO_AUTOBUILD") == "1":
                raise NativeExtensionError(
                    f"native extension {name} is not built; run `python -m fast_tffm_amd.build_native`") from first
            from fast_tffm_amd import build_native

            try:
                if build_kind == "cpu":
                    build_native.build_cpu()
                else:
                    build_native.build_hip()
                mod = importlib.import_module(f"fast_tffm_amd._native.{name}")
            except Exception as e:  # noqa: BLE001
                raise NativeExtensionError(f"could not build/load native extension {name}: {e}") from e
        _mods[name] = mod
        return mod


def cpu():
    """Host module: parser, hash64, CPU step kernels."""
    return _load("_fm_cpu", "cpu")


class _SyncChecked:
    """FM_SYNC_LAUNCH=1: every kernel entry point synchronises the device after its
    launches, so a fault is reported by the Python frame of the op that caused it
    (debugging aid; never on for timing runs)."""

    def __init__(self, mod):
        self._mod = mod

    def __getattr__(self, name):
        f = getattr(self._mod, name)
        if not callable(f):
            return f

        def wrapped(*args, **kw):
            import torch

            out = f(*args, **kw)
            try:
                torch.cuda.synchronize()
            except Exception as e:  # noqa: BLE001
                raise RuntimeError(f"_fm_hip.{name} faulted: {e}") from e
            return out

        return wrapped


_SYNC = os.environ.get("FM_SYNC_LAUNCH", "0") == "1"


def hip():
    """gfx950 module: GPU step kernels. Raises if unavailable."""
    var = os.environ.get("FM_HIP_VARIANT")  # A/B builds (build_native --variant)
    mod = _load(f"_fm_hip_{var}", "hip") if var else _load("_fm_hip", "hip")
    return _SyncChecked(mod) if _SYNC else mod


def loaded_paths() -> dict[str, str]:
    return {k: getattr(v, "__file__", "?") for k, v in _mods.items()}

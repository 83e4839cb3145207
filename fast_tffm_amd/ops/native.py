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


def _load(name: str, build_kind: str, variant: str | None = None):
    """Import an in-tree module, (re)building it first when it is missing or was not built
    from the current sources (content hash embedded in the binary, see build_native)."""
    with _lock:
        if name in _mods:
            return _mods[name]
        from fast_tffm_amd import build_native as bn

        if build_kind == "cpu":
            target, want = bn.cpu_target(), bn.cpu_hash()
        else:
            target, want = bn.hip_target(variant), bn.hip_hash(variant)
        have = bn.embedded_hash(target)
        if have != want:
            why = "is not built" if have is None else f"is stale (built from {have}, sources are {want})"
            if os.environ.get("FM_NO_AUTOBUILD") == "1":
                raise NativeExtensionError(f"native extension {name} {why}; run `python -m fast_tffm_amd.build_native`")
            print(f"[fast_tffm_amd] native extension {name} {why}: building", flush=True)
            try:
                if build_kind == "cpu":
                    bn.build_cpu()
                else:
                    bn.build_hip(variant=variant)
            except Exception as e:  # noqa: BLE001
                raise NativeExtensionError(f"could not build native extension {name}: {e}") from e
        try:
            mod = importlib.import_module(f"fast_tffm_amd._native.{name}")
        except ImportError as e:
            raise NativeExtensionError(f"could not load native extension {name}: {e}") from e
        if getattr(mod, "BUILD_HASH", None) != want:
            raise NativeExtensionError(f"{name}: loaded module hash {getattr(mod, 'BUILD_HASH', None)} != {want}")
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
    mod = _load(f"_fm_hip_{var}", "hip", var) if var else _load("_fm_hip", "hip")
    return _SyncChecked(mod) if _SYNC else mod


def loaded_paths() -> dict[str, str]:
    return {k: getattr(v, "__file__", "?") for k, v in _mods.items()}


def build_hashes() -> dict[str, str]:
    """Content hashes of the loaded native modules (reported by bench.py)."""
    return {k: getattr(v, "BUILD_HASH", "?") for k, v in _mods.items()}

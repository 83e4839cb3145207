"""Build the native extensions in-tree (fast_tffm_amd/_native/).

* ``_fm_cpu``: host C++ (g++ -O3 -fopenmp): libsvm parser, Hash64, CPU step
  kernels.  Needed everywhere (CPU tests, data pipeline).
* ``_fm_hip``: gfx950 HIP (hipcc --offload-arch=gfx950): the GPU hot path.

The reference builds one TF op library with a monkey-patched setuptools
(reference setup.py:88-201); here each module is one explicit compiler
invocation, so the build is reproducible from a shell and needs neither
hipify nor torch's cpp_extension JIT.

Usage:  python -m fast_tffm_amd.build_native [--cpu-only|--hip-only] [--force]
"""

from __future__ import annotations

import argparse
import glob
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
OUT = os.path.join(PKG, "_native")
ARCH = os.environ.get("FM_OFFLOAD_ARCH", "gfx950")

CPU_SOURCES = ["cpu/module.cpp", "cpu/parser.cpp", "cpu/kernels.cpp", "cpu/loader.cpp", "cpu/bincsr.cpp"]
HIP_SOURCES = ["hip/module.hip"]
# A/B build variants of the gfx950 module: name -> preprocessor defines (module _fm_hip_<name>,
# selected at run time with FM_HIP_VARIANT=<name>; tools/gpu_ab.sh).  Same-box kernel comparisons
# of a change against its predecessor; a variant is deleted with the losing code path once the
# A/B is recorded under profiles/ (round 1-2's nocap / unr* / fwdw* / fp8packed went that way).
from fast_tffm_amd.build_variants import HIP_VARIANTS  # noqa: E402  (not hashed: flags are)


_EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"  # resolved once (lazy init is not thread-safe)


def _ext_suffix() -> str:
    return _EXT_SUFFIX


def _py_includes() -> list[str]:
    import pybind11

    incs = {sysconfig.get_paths()["include"], sysconfig.get_paths()["platinclude"], pybind11.get_include()}
    return [f"-I{p}" for p in sorted(incs)]


# Rebuild decisions use a content hash, never mtimes: the hash covers every source and
# header the module is compiled from, the compiler command line (flags, defines, arch) and
# this file.  The hash is compiled into the module (``BUILD_HASH`` attribute and a
# ``FMBUILDHASH:<hex>`` marker in the binary), so a loader can check -- without importing
# it -- that a shipped .so was built from the sources next to it (ops/native.py).
HASH_MARKER = b"FMBUILDHASH:"


def _dep_files(kind: str) -> list[str]:
    if kind == "cpu":
        pats = ["cpu/*.cpp", "cpu/*.h", "*.h"]
    else:
        pats = ["hip/*.hip", "hip/*.h", "*.h"]
    out = []
    for p in pats:
        out += glob.glob(os.path.join(CSRC, p))
    return sorted(set(out))


def source_hash(kind: str, flags: list[str]) -> str:
    """sha256 (hex, 32 chars) of the sources, headers, flags and this builder."""
    h = hashlib.sha256()
    h.update(("\0".join(flags)).encode())
    for f in _dep_files(kind) + [os.path.abspath(__file__)]:
        h.update(os.path.relpath(f, PKG).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:32]


def embedded_hash(target: str) -> str | None:
    """The FMBUILDHASH marker of a built module (scanned from the file, not imported)."""
    try:
        with open(target, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(HASH_MARKER)
    if i < 0:
        return None
    return data[i + len(HASH_MARKER): i + len(HASH_MARKER) + 32].decode("ascii", "replace")


def _stale(target: str, want: str) -> bool:
    return embedded_hash(target) != want


def _run(cmd: list[str]) -> None:
    print("[build_native]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _cpu_flags() -> list[str]:
    return ["-O3", "-std=c++17", "-fPIC", "-shared", "-fopenmp", "-fvisibility=hidden"]


def cpu_target() -> str:
    return os.path.join(OUT, "_fm_cpu" + _ext_suffix())


def cpu_hash() -> str:
    return source_hash("cpu", _cpu_flags() + CPU_SOURCES)


def build_cpu(force: bool = False) -> str:
    os.makedirs(OUT, exist_ok=True)
    target = cpu_target()
    want = cpu_hash()
    if force or _stale(target, want):
        cxx = os.environ.get("CXX", "g++")
        tmp = target + ".tmp"
        cmd = [cxx, *_cpu_flags(), f'-DFM_BUILD_HASH="{want}"', *_py_includes(),
               *[os.path.join(CSRC, s) for s in CPU_SOURCES], "-o", tmp]
        _run(cmd)
        os.replace(tmp, target)
    return target


def hipcc_path() -> str | None:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    return None


def _hip_flags(variant: str | None) -> list[str]:
    name = hip_module_name(variant)
    return [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden",
            "-Wno-unused-result", f"-DFM_HIP_MODULE={name}", *(HIP_VARIANTS[variant] if variant else [])]


def hip_module_name(variant: str | None = None) -> str:
    return "_fm_hip" + (f"_{variant}" if variant else "")


def hip_target(variant: str | None = None) -> str:
    return os.path.join(OUT, hip_module_name(variant) + _ext_suffix())


def hip_hash(variant: str | None = None) -> str:
    return source_hash("hip", _hip_flags(variant) + HIP_SOURCES)


def build_hip(force: bool = False, variant: str | None = None) -> str:
    os.makedirs(OUT, exist_ok=True)
    target = hip_target(variant)
    want = hip_hash(variant)
    if force or _stale(target, want):
        hipcc = hipcc_path()
        if hipcc is None:
            raise RuntimeError("hipcc not found; cannot build the gfx950 extension")
        tmp = target + ".tmp"
        cmd = [hipcc, *_hip_flags(variant), f'-DFM_BUILD_HASH="{want}"', *_py_includes(), f"-I{CSRC}",
               *[os.path.join(CSRC, s) for s in HIP_SOURCES], "-o", tmp]
        _run(cmd)
        os.replace(tmp, target)
    return target


def build_all(force: bool = False, cpu: bool = True, hip: bool = True) -> list[str]:
    jobs = []
    with ThreadPoolExecutor(max_workers=2) as ex:
        if cpu:
            jobs.append(ex.submit(build_cpu, force))
        if hip:
            jobs.append(ex.submit(build_hip, force))
        return [j.result() for j in jobs]


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--cpu-only", action="store_true")
    ap.add_argument("--hip-only", action="store_true")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--variant", choices=sorted(HIP_VARIANTS), help="build an A/B variant of the HIP module")
    a = ap.parse_args(argv)
    if a.variant:
        print("built", build_hip(a.force, a.variant))
        return 0
    outs = build_all(force=a.force, cpu=not a.hip_only, hip=not a.cpu_only)
    for o in outs:
        print("built", o)
    return 0


if __name__ == "__main__":
    sys.exit(main())
